// sha2.h — SHA-512 (ed25519 challenge hash) and SHA-256 (tendermint address, pool
// cache key) compression functions, one message per lane.
//
// 64-bit rotates and shifts are written as v_alignbit_b32 pairs (hipcc otherwise emits
// two half-rate 64-bit shifts and two ORs per rotate); 64-bit adds lower to one
// v_lshl_add_u64.  The 80-round loop is fully unrolled with a 16-word ring so every
// schedule word stays in VGPRs (no scratch).  Callers supply already
// padded big-endian blocks: the host packs SignBytes with the FIPS 180-4 padding of the
// full R || A || M input (DESIGN.md §Data layout), so the device never branches on length.
#pragma once
#include "fe.h"

namespace txv {

// n is a compile-time constant at every call site (the rounds are unrolled)
TXV_HD uint64_t rotr64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t a = n < 32 ? hi : lo, b = n < 32 ? lo : hi;   // rotate by 32 = swap halves
  const int m = n & 31;
  if (m == 0) return ((uint64_t)a << 32) | b;
  return ((uint64_t)__builtin_amdgcn_alignbit(b, a, m) << 32) | __builtin_amdgcn_alignbit(a, b, m);
#else
  return (x >> n) | (x << (64 - n));
#endif
}
// x >> n for 0 < n < 32
TXV_HD uint64_t shr64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((uint64_t)(hi >> n) << 32) | __builtin_amdgcn_alignbit(hi, lo, n);
#else
  return x >> n;
#endif
}
// three-input XOR and majority of 64-bit words: one v_bitop3_b32 per half on gfx950 (truth
// tables 0x96 / 0xE8; symmetric in their inputs) instead of two v_xor_b32 / a bfi + xor
#ifndef TXV_SHA_BITOP3
#define TXV_SHA_BITOP3 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && TXV_SHA_BITOP3
// (lo, hi) words as one 64-bit register pair (an OR of shifted halves lowers to v_lshl_add_u64)
__device__ __forceinline__ uint64_t pair64(uint32_t lo, uint32_t hi) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  u32x2 v;
  v.x = lo;
  v.y = hi;
  return __builtin_bit_cast(uint64_t, v);
}
#endif
TXV_HD uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__) && TXV_SHA_BITOP3
  return pair64(__builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x96),
                __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0x96));
#else
  return a ^ b ^ c;
#endif
}
TXV_HD uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__) && TXV_SHA_BITOP3
  return pair64(__builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0xE8),
                __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0xE8));
#else
  return (a & b) | (c & (a | b));
#endif
}
TXV_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
TXV_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}
// 8 little-endian bytes (two LE u32 words lo, hi) as a big-endian u64 word
TXV_HD uint64_t be64_from_le32(uint32_t lo, uint32_t hi) {
  return ((uint64_t)bswap32(lo) << 32) | bswap32(hi);
}

TXV_HD uint64_t sha512_k(int i) {
  const uint64_t K[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};
  return K[i];
}

TXV_HD void sha512_init(uint64_t st[8]) {
  st[0] = 0x6a09e667f3bcc908ULL; st[1] = 0xbb67ae8584caa73bULL; st[2] = 0x3c6ef372fe94f82bULL;
  st[3] = 0xa54ff53a5f1d36f1ULL; st[4] = 0x510e527fade682d1ULL; st[5] = 0x9b05688c2b3e6c1fULL;
  st[6] = 0x1f83d9abfb41bd6bULL; st[7] = 0x5be0cd19137e2179ULL;
}

// one compression; w[16] is consumed (overwritten by the schedule).  Rounds 0-15 are
// unrolled; rounds 16-79 run as 4 iterations of a 16-round unrolled body, so every w[]
// index is static (no indexed register access) and the 8 working variables return to
// their registers at each back-edge.
#define TXV_SHA512_ROUND(I, J, SCHED)                                                       \
  {                                                                                        \
    uint64_t wi;                                                                           \
    if (SCHED) {                                                                           \
      const uint64_t w15 = w[((J) + 1) & 15], w2 = w[((J) + 14) & 15];                      \
      const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));           \
      const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));            \
      wi = w[(J) & 15] + s0 + w[((J) + 9) & 15] + s1;                                      \
      w[(J) & 15] = wi;                                                                    \
    } else {                                                                               \
      wi = w[J];                                                                           \
    }                                                                                      \
    const uint64_t S1 = xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));              \
    const uint64_t ch = g ^ (e & (f ^ g));                                                 \
    const uint64_t t1 = h + S1 + ch + sha512_k(I) + wi;                                     \
    const uint64_t S0 = xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));              \
    const uint64_t mj = maj64(a, b, c);                                                    \
    const uint64_t t2 = S0 + mj;                                                           \
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;                    \
  }

TXV_HD void sha512_block(uint64_t st[8], uint64_t w[16]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int j = 0; j < 16; ++j) TXV_SHA512_ROUND(j, j, false)
#pragma unroll 1
  for (int i0 = 16; i0 < 80; i0 += 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j) TXV_SHA512_ROUND(i0 + j, j, true)
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// two independent compressions with their rounds interleaved (K1a's paired variant): every round
// of one message has the other's as independent neighbours, so a wave's dependent SHA-512 chain
// issues with ILP 2 instead of waiting on itself
#define TXV_SHA512_ROUND2(I, J, SCHED, W, A, B, C, D, E, F, G, H)                           \
  {                                                                                        \
    uint64_t wi;                                                                           \
    if (SCHED) {                                                                           \
      const uint64_t w15 = W[((J) + 1) & 15], w2 = W[((J) + 14) & 15];                      \
      const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));           \
      const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));            \
      wi = W[(J) & 15] + s0 + W[((J) + 9) & 15] + s1;                                      \
      W[(J) & 15] = wi;                                                                    \
    } else {                                                                               \
      wi = W[J];                                                                           \
    }                                                                                      \
    const uint64_t S1 = xor3_64(rotr64(E, 14), rotr64(E, 18), rotr64(E, 41));              \
    const uint64_t ch = G ^ (E & (F ^ G));                                                 \
    const uint64_t t1 = H + S1 + ch + sha512_k(I) + wi;                                     \
    const uint64_t S0 = xor3_64(rotr64(A, 28), rotr64(A, 34), rotr64(A, 39));              \
    const uint64_t mj = maj64(A, B, C);                                                    \
    const uint64_t t2 = S0 + mj;                                                           \
    H = G; G = F; F = E; E = D + t1; D = C; C = B; B = A; A = t1 + t2;                    \
  }

TXV_HD void sha512_block2(uint64_t st0[8], uint64_t w0[16], uint64_t st1[8], uint64_t w1[16]) {
  uint64_t a0 = st0[0], b0 = st0[1], c0 = st0[2], d0 = st0[3], e0 = st0[4], f0 = st0[5], g0 = st0[6], h0 = st0[7];
  uint64_t a1 = st1[0], b1 = st1[1], c1 = st1[2], d1 = st1[3], e1 = st1[4], f1 = st1[5], g1 = st1[6], h1 = st1[7];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    TXV_SHA512_ROUND2(j, j, false, w0, a0, b0, c0, d0, e0, f0, g0, h0)
    TXV_SHA512_ROUND2(j, j, false, w1, a1, b1, c1, d1, e1, f1, g1, h1)
  }
#pragma unroll 1
  for (int i0 = 16; i0 < 80; i0 += 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      TXV_SHA512_ROUND2(i0 + j, j, true, w0, a0, b0, c0, d0, e0, f0, g0, h0)
      TXV_SHA512_ROUND2(i0 + j, j, true, w1, a1, b1, c1, d1, e1, f1, g1, h1)
    }
  }
  st0[0] += a0; st0[1] += b0; st0[2] += c0; st0[3] += d0; st0[4] += e0; st0[5] += f0; st0[6] += g0; st0[7] += h0;
  st1[0] += a1; st1[1] += b1; st1[2] += c1; st1[3] += d1; st1[4] += e1; st1[5] += f1; st1[6] += g1; st1[7] += h1;
}
#undef TXV_SHA512_ROUND2
#undef TXV_SHA512_ROUND

TXV_HD uint32_t sha256_k(int i) {
  const uint32_t K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  return K[i];
}

TXV_HD void sha256_init(uint32_t st[8]) {
  st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}

TXV_HD void sha256_block(uint32_t st[8], uint32_t w[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) wi = w[i];
    else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = g ^ (e & (f ^ g));
    uint32_t t1 = h + S1 + ch + sha256_k(i) + wi;
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) | (c & (a | b));
    uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// SHA-256 of exactly 32 bytes given as 8 little-endian-loaded u32 words of the byte
// string (i.e. word i = bytes[4i..4i+3] read little-endian).  Output: 8 BE state words.
TXV_HD void sha256_32bytes(uint32_t out[8], const uint32_t in_le[8]) {
  uint32_t st[8], w[16];
  sha256_init(st);
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = bswap32(in_le[i]);
  w[8] = 0x80000000u;
#pragma unroll
  for (int i = 9; i < 15; ++i) w[i] = 0;
  w[15] = 256;
  sha256_block(st, w);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = st[i];
}

// SHA-256 of len bytes at p (any alignment), big-endian state words (TxHash digests: the
// exchange names of the sets, kernels_flow.hip, and the ingest route's shard, kernels_route.hip)
TXV_HD void sha256_bytes(const uint8_t* p, uint32_t n, uint32_t st[8]) {
  sha256_init(st);
  const uint32_t nblk = (n + 9 + 63) / 64;       // message + 0x80 + 8-byte length
  for (uint32_t b = 0; b < nblk; ++b) {
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      uint32_t v = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t k = 64u * b + 4u * (uint32_t)t + (uint32_t)q;   // byte index in the padded message
        uint32_t byte = 0;
        if (k < n) byte = p[k];
        else if (k == n) byte = 0x80u;
        v = (v << 8) | byte;
      }
      w[t] = v;
    }
    if (b == nblk - 1) { w[14] = (uint32_t)((uint64_t)n >> 29); w[15] = n << 3; }
    sha256_block(st, w);
  }
}

}  // namespace txv
