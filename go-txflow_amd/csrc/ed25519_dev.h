// ed25519_dev.h — per-lane ed25519 building blocks shared by the verify, table-build,
// keygen and sign kernels.
//
// Verification follows golang.org/x/crypto/ed25519.Verify @c2843e01d9a2 (external; the
// reference calls it at types/tx_vote.go:115 via tendermint PubKeyEd25519.VerifyBytes):
//   reject len(sig) != 64 | sig[63] & 0xE0 | undecodable A | s >= L,
//   k = SHA-512(R || A || M) mod L, accept iff encode([s]B + [k](-A)) == R bytewise.
// The double scalar multiplication is evaluated doubling-free over fixed-base radix-2^W
// tables (ge.h half-Niels entries): T_P[i][j] = j * 2^(W i) * P for i < 256/W, j <= 2^(W-1)
// (j = 0 the identity), so [s]B + [k](-A) = sum_i T_B[i][s_i] - T_A[i][k_i] with signed
// digits.  This is exact group arithmetic, hence the same point and encoding as x/crypto's
// sliding-window GeDoubleScalarMultVartime.  Entries are 128 B (one line):
//   W = 4:  64 positions x    9 entries x 128 B =    73,728 B per point (B fits in LDS)
//   W = 8:  32 positions x  129 entries x 128 B =   528,384 B per point (L2/MALL resident)
//   W = 20: 13 positions x 2^19+1 entries x 128 B = 872 MB per point (HBM)
//   W = 21: 12 positions (11 x 2^20+1, the top one 2^21+9 entries) = 1.70 GB per point (Tab<21>)
// ceil(256/W_B) + ceil(256/W_A) table additions per verification, the first of them free
// (the accumulator starts as the first B entry's point).
#pragma once
#include "fe.h"
#include "sc.h"
#include "sha2.h"
#include "ge.h"

namespace txv {

template <int W>
struct Tab {
  static constexpr int kPositions = (256 + W - 1) / W;
  static constexpr int kEntries = (1 << (W - 1)) + 1;
  static constexpr bool kLongTop = false;     // see Tab<21>
  static constexpr int kTopEntries = kEntries;
  static constexpr size_t kWords = (size_t)kPositions * kEntries * kEntryWords;   // > 2^31 at W = 24
  // K0 lanes per point: one per (position, chunk of 8 multiples)
  static constexpr uint64_t kBuildLanes = (uint64_t)kPositions * ((kEntries - 1) / 8);
};

// Radix 2^21 over 253 bits: 12 positions, one table addition fewer than radix 2^20's 13 (every
// verified scalar is below L < 2^253).  Eleven signed digits in [-2^20, 2^20) cannot reach 2^252,
// so the top position (bits 231..252) takes an unsigned digit: the remaining scalar plus the
// carry, at most floor((L - 1) / 2^231) + 1 = 2^21 + 1.  Positions 0..10 hold 2^20 + 1 entries,
// the top one 2^21 + 9 (K0 builds it in chunks of 8; entries above 2^21 + 1 are never read), so
// T[pos][idx] stays at entry pos * kEntries + idx: 1.70 GB per point, against 0.87 GB at W = 20.
template <>
struct Tab<21> {
  static constexpr int kPositions = 12;
  static constexpr int kEntries = (1 << 20) + 1;
  static constexpr bool kLongTop = true;
  static constexpr int kTopEntries = (1 << 21) + 9;
  static constexpr size_t kWords = ((size_t)(kPositions - 1) * kEntries + kTopEntries) * kEntryWords;
  static constexpr uint64_t kBuildLanes = (uint64_t)(kPositions - 1) * ((kEntries - 1) / 8) + (kTopEntries - 1) / 8;
};

// legacy W = 4 names (keygen/sign and the host emulation)
constexpr int kTabPositions = Tab<4>::kPositions;
constexpr int kTabEntries = Tab<4>::kEntries;
constexpr int kTableWords = Tab<4>::kWords;

// message words are stored big-endian (SHA-native), zero beyond the message length.
struct MsgView {
  const uint64_t* words;   // column base for this lane: words[w * stride]
  uint32_t stride;         // column stride (in u64 words)
  uint32_t n_words;        // stored words per message
  uint32_t len;            // message length in bytes
};

TXV_HD uint64_t msg_word(const MsgView& m, uint32_t w) {
  return w < m.n_words ? m.words[(size_t)w * m.stride] : 0ull;
}

// number of 128-byte SHA-512 blocks for prefix_bytes + len
TXV_HD uint32_t sha512_nblocks(uint32_t total_len) { return (total_len + 17u + 127u) / 128u; }

// SHA-512 of pre[0..pre_words) || M, pre given as big-endian words.  Result as 16
// little-endian u32 limbs of the 512-bit digest interpreted little-endian (ScReduce input).
TXV_HD void sha512_prefixed(uint32_t digest_le[16], const uint64_t* pre, int pre_words, const MsgView& m) {
  uint64_t st[8];
  sha512_init(st);
  const uint32_t total = 8u * (uint32_t)pre_words + m.len;
  const uint32_t nblk = sha512_nblocks(total);
  const uint32_t pad_word = total >> 3, pad_shift = 56u - 8u * (total & 7u);
  const uint32_t last = 16u * nblk - 1u;
  for (uint32_t b = 0; b < nblk; ++b) {
    uint64_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      uint32_t gw = 16u * b + (uint32_t)t;
      uint64_t v;
      if (b == 0 && t < pre_words) v = pre[t];
      else v = msg_word(m, gw - (uint32_t)pre_words);
      if (gw == pad_word) v |= 0x80ull << pad_shift;
      if (gw == last) v = (uint64_t)total * 8u;
      w[t] = v;
    }
    sha512_block(st, w);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    digest_le[2 * k] = bswap32((uint32_t)(st[k] >> 32));
    digest_le[2 * k + 1] = bswap32((uint32_t)st[k]);
  }
}

// Same digest with the next block's message words loaded before the current block is
// compressed, so a vote's HBM latency is exposed once instead of once per block (K1a: the
// C2 SignBytes make 2 blocks).  Costs 16 u64 registers of look-ahead.
TXV_HD void sha512_prefixed_pf(uint32_t digest_le[16], const uint64_t* pre, int pre_words, const MsgView& m) {
  uint64_t st[8];
  sha512_init(st);
  const uint32_t total = 8u * (uint32_t)pre_words + m.len;
  const uint32_t nblk = sha512_nblocks(total);
  const uint32_t pad_word = total >> 3, pad_shift = 56u - 8u * (total & 7u);
  const uint32_t last = 16u * nblk - 1u;
  uint64_t nx[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) nx[t] = t < pre_words ? pre[t] : msg_word(m, (uint32_t)(t - pre_words));
  for (uint32_t b = 0; b < nblk; ++b) {
    uint64_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const uint32_t gw = 16u * b + (uint32_t)t;
      uint64_t v = nx[t];
      if (gw == pad_word) v |= 0x80ull << pad_shift;
      if (gw == last) v = (uint64_t)total * 8u;
      w[t] = v;
    }
    if (b + 1 < nblk) {
#pragma unroll
      for (int t = 0; t < 16; ++t) nx[t] = msg_word(m, 16u * (b + 1) + (uint32_t)t - (uint32_t)pre_words);
    }
    sha512_block(st, w);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    digest_le[2 * k] = bswap32((uint32_t)(st[k] >> 32));
    digest_le[2 * k + 1] = bswap32((uint32_t)st[k]);
  }
}

// two digests with their compressions interleaved (sha512_block2): blocks up to the longer
// message's count, the shorter one's extra blocks computed on zeros and discarded
TXV_HD void sha512_prefixed2(uint32_t dig0[16], const uint64_t* pre0, const MsgView& m0, uint32_t dig1[16],
                             const uint64_t* pre1, const MsgView& m1, int pre_words) {
  uint64_t st0[8], st1[8];
  sha512_init(st0);
  sha512_init(st1);
  const uint32_t tot0 = 8u * (uint32_t)pre_words + m0.len, tot1 = 8u * (uint32_t)pre_words + m1.len;
  const uint32_t nb0 = sha512_nblocks(tot0), nb1 = sha512_nblocks(tot1), nb = nb0 > nb1 ? nb0 : nb1;
  const uint32_t pw0 = tot0 >> 3, ps0 = 56u - 8u * (tot0 & 7u), last0 = 16u * nb0 - 1u;
  const uint32_t pw1 = tot1 >> 3, ps1 = 56u - 8u * (tot1 & 7u), last1 = 16u * nb1 - 1u;
  for (uint32_t b = 0; b < nb; ++b) {
    uint64_t w0[16], w1[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const uint32_t gw = 16u * b + (uint32_t)t;
      uint64_t v0 = (b == 0 && t < pre_words) ? pre0[t] : msg_word(m0, gw - (uint32_t)pre_words);
      uint64_t v1 = (b == 0 && t < pre_words) ? pre1[t] : msg_word(m1, gw - (uint32_t)pre_words);
      if (gw == pw0) v0 |= 0x80ull << ps0;
      if (gw == last0) v0 = (uint64_t)tot0 * 8u;
      if (gw == pw1) v1 |= 0x80ull << ps1;
      if (gw == last1) v1 = (uint64_t)tot1 * 8u;
      w0[t] = v0;
      w1[t] = v1;
    }
    uint64_t s0[8], s1[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { s0[k] = st0[k]; s1[k] = st1[k]; }
    sha512_block2(s0, w0, s1, w1);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (b < nb0) st0[k] = s0[k];
      if (b < nb1) st1[k] = s1[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    dig0[2 * k] = bswap32((uint32_t)(st0[k] >> 32));
    dig0[2 * k + 1] = bswap32((uint32_t)st0[k]);
    dig1[2 * k] = bswap32((uint32_t)(st1[k] >> 32));
    dig1[2 * k + 1] = bswap32((uint32_t)st1[k]);
  }
}

// table entry fetch: T[pos][idx] from a flat word array, (qp, qm) swapped for -Q (neg): the
// swap is the choice of which 16-byte-aligned half of the line is loaded as which
template <int W, typename Ptr>
TXV_HD void load_entry_w(Ptr tab, int pos, int idx, bool neg, fe10& qp, fe10& qm, fe10& qd) {
#if defined(TXV_EXP_L2_TABLES)   // experiment only: every lookup hits one entry (L1/L2 resident)
  const size_t base = (size_t)(1 + (idx & 1)) * kEntryWords;
#else
  const size_t base = (size_t)(uint32_t)(pos * Tab<W>::kEntries + idx) * kEntryWords;
#endif
#ifndef TXV_ENTRY_LOADS
#define TXV_ENTRY_LOADS 1
#endif
#if TXV_ENTRY_LOADS == 2
  // the whole line as 8 x 16-byte loads, the sign swap as per-lane selects
  const uint4* e4 = reinterpret_cast<const uint4*>(&tab[base]);
  uint32_t w[32];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint4 x = e4[j];
    w[4 * j] = x.x; w[4 * j + 1] = x.y; w[4 * j + 2] = x.z; w[4 * j + 3] = x.w;
  }
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    qd.v[i] = w[kEntryQd + i];
    qm.v[i] = neg ? w[i] : w[kEntryQm + i];
    qp.v[i] = neg ? w[kEntryQm + i] : w[i];
  }
#else
  // in the order ge10_madd consumes them (qd, then qm, then qp), so each product can start as
  // soon as its own operand has landed (vmcnt counts in issue order)
  const uint32_t op = neg ? kEntryQm : 0u, om = neg ? 0u : kEntryQm;
  const uint2* d2 = reinterpret_cast<const uint2*>(&tab[base + kEntryQd]);
  const uint2 d0 = d2[0];
  const uint4 d1 = reinterpret_cast<const uint4*>(d2 + 1)[0], d3 = reinterpret_cast<const uint4*>(d2 + 1)[1];
  const uint4* m4 = reinterpret_cast<const uint4*>(&tab[base + om]);
  const uint4 m0 = m4[0], m1 = m4[1];
  const uint2 m2 = reinterpret_cast<const uint2*>(m4 + 2)[0];
  const uint4* p4 = reinterpret_cast<const uint4*>(&tab[base + op]);
  const uint4 p0 = p4[0], p1 = p4[1];
  const uint2 p2 = reinterpret_cast<const uint2*>(p4 + 2)[0];
  qp.v[0] = p0.x; qp.v[1] = p0.y; qp.v[2] = p0.z; qp.v[3] = p0.w;
  qp.v[4] = p1.x; qp.v[5] = p1.y; qp.v[6] = p1.z; qp.v[7] = p1.w; qp.v[8] = p2.x; qp.v[9] = p2.y;
  qm.v[0] = m0.x; qm.v[1] = m0.y; qm.v[2] = m0.z; qm.v[3] = m0.w;
  qm.v[4] = m1.x; qm.v[5] = m1.y; qm.v[6] = m1.z; qm.v[7] = m1.w; qm.v[8] = m2.x; qm.v[9] = m2.y;
  qd.v[0] = d0.x; qd.v[1] = d0.y; qd.v[2] = d1.x; qd.v[3] = d1.y;
  qd.v[4] = d1.z; qd.v[5] = d1.w; qd.v[6] = d3.x; qd.v[7] = d3.y; qd.v[8] = d3.z; qd.v[9] = d3.w;
#endif
}

// Streaming signed radix-2^W digit of a 256-bit scalar held in 8 words: returns the low
// digit in [-2^(W-1), 2^(W-1)) (with the running carry) and shifts the scalar right by W.
// Works for any W <= 16 (digits may straddle words); ~10 VALU ops per digit.
template <int W>
TXV_HD int next_digit(uint32_t s[8], uint32_t& carry) {
  constexpr uint32_t mask = (1u << W) - 1u, half = 1u << (W - 1);
  const uint32_t d = (s[0] & mask) + carry;        // [0, 2^W]
  carry = (d + half) >> W;                          // 1 iff d >= 2^(W-1)
#pragma unroll
  for (int i = 0; i < 7; ++i) s[i] = (s[i] >> W) | (s[i + 1] << (32 - W));
  s[7] >>= W;
  return (int)d - (int)(carry << W);
}

// digit of table position `pos` (in order, pos = 0, 1, ...): next_digit<W>, except for a
// long-top table's last position, whose digit is the whole remaining scalar plus the carry
// (non-negative, <= 2^21 + 1 for W = 21; s < 2^253)
template <int W>
TXV_HD int table_digit(uint32_t s[8], uint32_t& carry, int pos) {
  if constexpr (Tab<W>::kLongTop) {
    if (pos == Tab<W>::kPositions - 1) return (int)(s[0] + carry);
  }
  return next_digit<W>(s, carry);
}

// every signed radix-2^W digit of a scalar < 2^253 at once: digit i from bits [W i, W i + W) plus
// the carry of digit i - 1, exactly the sequence table_digit<W> produces (the split K1b kernel)
template <int W, int N>
TXV_HD void signed_digits(const uint32_t s[8], int d[N]) {
  constexpr uint32_t mask = (1u << W) - 1u, half = 1u << (W - 1);
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int b = W * i, w = b >> 5, o = b & 31;
    uint32_t win = s[w] >> o;
    if (o + W > 32 && w + 1 < 8) win |= s[w + 1] << (32 - o);
    if (Tab<W>::kLongTop && i == Tab<W>::kPositions - 1) {   // table_digit: the rest + carry
      static_assert(!Tab<W>::kLongTop || W * (Tab<W>::kPositions - 1) % 32 + 22 <= 32, "top digit in one word");
      d[i] = (int)(win + carry);
      break;
    }
    const uint32_t dd = (win & mask) + carry;
    carry = (dd + half) >> W;
    d[i] = (int)dd - (int)(carry << W);
  }
}

// sum_i T_B[i][s_i] + T_A[i][-k_i] over raw scalars s, k < 2^253 (digits of k negated,
// giving [k](-A)); digits are produced on the fly, so any windows < 32 work (a long-top WA
// table's last digit by table_digit).  The base
// point's table may use a wider window WB than the validators' WA (one table serves every
// vote, so it can take gigabytes of HBM).  The walk runs in fe10 (ge10_madd); the result is
// handed back in radix 2^32 (X, Y, Z; T is not produced).
template <int WB, int WA, typename PtrB, typename PtrA>
TXV_HD ge_ext double_scalarmult_w2(PtrB tb, PtrA ta, const uint32_t s_in[8], const uint32_t k_in[8], bool use_a) {
  static_assert(WB >= WA, "B window must be at least the A window");
  uint32_t s[8], k[8], cs = 0, ck = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) { s[i] = s_in[i]; k[i] = k_in[i]; }
  fe10 qp, qm, qd;
  ge10_ext P;
  {
    const int ds = next_digit<WB>(s, cs);
    load_entry_w<WB>(tb, 0, ds < 0 ? -ds : ds, ds < 0, qp, qm, qd);
    P = ge10_from_entry(qp, qm);
  }
  for (int pos = 0; pos < Tab<WA>::kPositions; ++pos) {
    if (pos > 0 && pos < Tab<WB>::kPositions) {
      const int ds = next_digit<WB>(s, cs);
      load_entry_w<WB>(tb, pos, ds < 0 ? -ds : ds, ds < 0, qp, qm, qd);
      P = ge10_madd(P, qp, qm, qd, ds < 0);
    }
    if (use_a) {
      const int dk = table_digit<WA>(k, ck, pos);
      load_entry_w<WA>(ta, pos, dk < 0 ? -dk : dk, dk > 0, qp, qm, qd);
      P = ge10_madd(P, qp, qm, qd, dk > 0);
    }
  }
  ge_ext R;
  R.X = fe_from_fe10(P.X);
  R.Y = fe_from_fe10(P.Y);
  R.Z = fe_from_fe10(P.Z);
  R.T = fe_zero();
  return R;
}
template <int W, typename PtrB, typename PtrA>
TXV_HD ge_ext double_scalarmult_w(PtrB tb, PtrA ta, const uint32_t s_in[8], const uint32_t k_in[8], bool use_a) {
  return double_scalarmult_w2<W, W>(tb, ta, s_in, k_in, use_a);
}

// [s]B (+ [k](-A)) with the radix-16 tables (keygen / sign / host emulation)
template <typename PtrB, typename PtrA>
TXV_HD ge_ext double_scalarmult_fixed(PtrB tb, PtrA ta, const uint32_t s[8], const uint32_t k[8], bool use_a) {
  return double_scalarmult_w<4>(tb, ta, s, k, use_a);
}

// [m]P for a small positive m (double-and-add from the top bit)
TXV_HD ge_ext ge_mul_small(const ge_ext& P, uint32_t m) {
  ge_ext R = P;
  int top = 31 - __builtin_clz(m);
  for (int b = top - 1; b >= 0; --b) {
    R = ge_dbl(R);
    if ((m >> b) & 1u) R = ge_add(R, P);
  }
  return R;
}

// the base point's canonical encoding (little-endian words)
TXV_HD void base_point_words(uint32_t w[8]) {
  const uint32_t b[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                         0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = b[i];
}

}  // namespace txv
