// kernels_verify.hip — gfx950 kernels for TxVote signature work.
//
//   txv_k_build_tables  (K0)  per validator: address = SHA-256(pub)[:20] (tendermint
//                              PubKeyEd25519.Address, called at types/tx_vote.go:111),
//                              ref10 decode of A, radix-2^W fixed-base half-Niels table of A
//                              (128-byte fe10 entries, ge.h).  Also run once on the base point B.
//   txv_k_challenge     (K1a) per vote: x/crypto ed25519.Verify's scalar checks and
//                              k = SHA-512(R || A || SignBytes) mod L (types/tx_vote.go:115)
//   txv_k_scalarmult_multi (K1b) V votes per lane: [s]B + [k](-A) over the tables, gathered
//                              cooperatively into LDS (one line per 8 lanes), one shared
//                              inversion, canonical encoding compared with R
//   txv_k_keygen / txv_k_sign  load generator mirroring MockPV.SignTxVote
//                              (types/priv_validator.go:83-95): RFC 8032 signing on device.
//
// Launch geometry: 512-thread workgroups; K1b walks an XCD-contiguous eighth of the work list
// per group of blocks (blocks b, b+8, ... share an XCD) and runs at 2 waves/SIMD with V = 8
// (batches of >= 768K votes) or V = 4 (configured); smaller batches run one vote per lane
// (txv_k_scalarmult_points + txv_k_batch_encode, 4 waves/SIMD).
#include <algorithm>
#include <cstdlib>

#include "ed25519_dev.h"
#include "fe_inv_var.h"
#include "txv_device.h"

using namespace txv;

// K1a's SHA-512 may load block b+1's message words before compressing block b (measured equal:
// K1a 298 vs 299-306 us at 116 vs 99 VGPRs, profiles/r01/k1a_prefetch; off)
#ifndef TXV_K1A_PREFETCH
#define TXV_K1A_PREFETCH 0
#endif

// K1b's shared inversion: the variable-time divstep inverse (fe_inv_var.h) or the Fermat
// chain; the value is the same either way (encoding canonicalises)
#ifndef TXV_INV_VAR
#define TXV_INV_VAR 1
#endif
__device__ __forceinline__ fe verify_invert(const fe& z) {
#if TXV_INV_VAR
  return fe_invert_var(z);
#else
  return fe_invert(z);
#endif
}

// ---------------------------------------------------------------- K0: tables
// One lane per (point, position, chunk of 8 multiples): P_i = 2^(W i) A by W*i doublings,
// then (8c+1..8c+8) * P_i, batch-inverted (Montgomery's trick) into affine Niels entries.
template <int W>
__global__ void __launch_bounds__(64) txv_k_build_tables(const uint32_t* __restrict__ pubs_le, uint32_t n_points,
                                                          uint32_t* __restrict__ tables,
                                                          uint8_t* __restrict__ decode_ok,
                                                          uint32_t* __restrict__ addr_words,
                                                          const uint32_t* __restrict__ out_slot) {
  constexpr int chunks = (Tab<W>::kEntries - 1) / 8;
  constexpr uint64_t per_point = Tab<W>::kBuildLanes;
  const uint64_t gid = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  const uint32_t pt = (uint32_t)(gid / per_point);
  const int t = (int)(gid % per_point);
  if (pt >= n_points) return;
  // a long-top table's last position takes the lanes past the others' (kTopEntries - 1) / 8 chunks
  constexpr int last = Tab<W>::kPositions - 1;
  const bool top = Tab<W>::kLongTop && t >= last * chunks;
  const int pos = top ? last : t / chunks, c = top ? t - last * chunks : t % chunks;
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = pubs_le[pt * 8 + i];
  if (t == 0 && addr_words) {
    uint32_t h[8];
    sha256_32bytes(h, w);
    // first 20 bytes of the big-endian digest, stored as 5 little-endian-loaded words
#pragma unroll
    for (int i = 0; i < 5; ++i) addr_words[pt * 5 + i] = bswap32(h[i]);
  }
  ge_ext A;
  bool ok = ge_decode(A, w);
  if (t == 0 && decode_ok) decode_ok[pt] = ok ? 1 : 0;
  ge_ext P = A;
  for (int i = 0; i < W * pos; ++i) P = ge_dbl(P);
  ge_ext M[8];
  M[0] = ge_mul_small(P, 8u * c + 1u);
#pragma unroll
  for (int j = 1; j < 8; ++j) M[j] = ge_add(M[j - 1], P);
  fe pref[8];
  pref[0] = M[0].Z;
#pragma unroll
  for (int j = 1; j < 8; ++j) pref[j] = fe_mul(pref[j - 1], M[j].Z);
  fe inv = fe_invert(pref[7]);
  uint32_t* out = tables + (size_t)(out_slot ? out_slot[pt] : pt) * Tab<W>::kWords + (size_t)pos * Tab<W>::kEntries * kEntryWords;
#pragma unroll
  for (int j = 7; j >= 0; --j) {
    fe zi = j ? fe_mul(inv, pref[j - 1]) : inv;
    if (j) inv = fe_mul(inv, M[j].Z);
    ge_niels n = ge_to_niels(M[j], zi);
    entry_words(out + (8 * c + j + 1) * kEntryWords, n.ypx, n.ymx, n.xy2d);
  }
  if (c == 0) entry_identity(out);
}

// ---------------------------------------------------------------- K1: verify
// the table slot of validator v: txv_set_validators keeps each key's tables in one slot of the
// context's table pool across validator-set changes (null: the tables are in validator order)
__device__ __forceinline__ uint32_t tab_slot(const VerifyArgs& a, uint32_t v) { return a.tslot ? a.tslot[v] : v; }
// K1 is split in two launches so each phase gets its own register allocation (one fused
// kernel kept the signature words and digits live across SHA-512 and the table walk and
// needed 272 VGPRs = 1 wave/SIMD):
//   K1a txv_k_challenge   per vote: length / top-bit / s < L / decode checks, k = SHA-512(R||A||M) mod L
//                         -> k[8][n_pad] (32 B/vote, HBM) and the "go" flag in ok_out
//   K1b txv_k_scalarmult  per vote (validator-grouped list for w <= 12, arrival order above): [s]B + [k](-A), encode, compare with R

// Prechecks + challenge of vote i: false if the vote is rejected before the group equation
// (length, sig[63] & 0xE0, undecodable A, s >= L, SignBytes failure), else k = SHA-512(R||A||M)
// mod L and the S half of the signature.
__device__ __forceinline__ bool vote_challenge(const VerifyArgs& a, uint32_t i, uint32_t k_out[8], uint32_t s_out[8]) {
  const uint8_t fl = a.flags[i];
  const uint32_t v = a.val[i];
  uint32_t s[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) s[j] = a.sig[(size_t)j * a.n_pad + i];
  const bool bad = !(fl & TXV_FLAG_SIG64) || (fl & TXV_FLAG_BADMSG) || (s[15] & 0xE0000000u) || !a.decode_ok[v] ||
                   !sc_lt_L(s + 8);
  if (bad) return false;
  const uint32_t* pw = a.pubs_le + (size_t)v * 8;
  uint64_t pre[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    pre[j] = be64_from_le32(s[2 * j], s[2 * j + 1]);
    pre[4 + j] = be64_from_le32(pw[2 * j], pw[2 * j + 1]);
  }
  MsgView m{a.msg + i, a.n_pad, a.msg_words, a.msg_len[i]};
  uint32_t dig[16];
#if TXV_K1A_PREFETCH
  sha512_prefixed_pf(dig, pre, 8, m);
#else
  sha512_prefixed(dig, pre, 8, m);
#endif
  sc k = sc_reduce512(dig);
#pragma unroll
  for (int j = 0; j < 8; ++j) { k_out[j] = k.v[j]; s_out[j] = s[8 + j]; }
  return true;
}

// the same out of line (the fused K1b: its SHA-512 registers then do not add to the walk's)
__device__ __attribute__((noinline)) bool vote_challenge_call(const VerifyArgs& a, uint32_t i, uint32_t k_out[8],
                                                              uint32_t s_out[8]) {
  return vote_challenge(a, i, k_out, s_out);
}

// the scalar checks of vote i and its SHA-512 prefix (R || A as big-endian words); false when the
// vote fails them (then no challenge is needed)
__device__ __forceinline__ bool vote_checks(const VerifyArgs& a, uint32_t i, uint32_t s[16], uint64_t pre[8]) {
  const uint8_t fl = a.flags[i];
  const uint32_t v = a.val[i];
#pragma unroll
  for (int j = 0; j < 16; ++j) s[j] = a.sig[(size_t)j * a.n_pad + i];
  const bool bad = !(fl & TXV_FLAG_PENDING) || !(fl & TXV_FLAG_SIG64) || (fl & TXV_FLAG_BADMSG) ||
                   (s[15] & 0xE0000000u) || !a.decode_ok[v] || !sc_lt_L(s + 8);
  const uint32_t* pw = a.pubs_le + (size_t)v * 8;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    pre[j] = be64_from_le32(s[2 * j], s[2 * j + 1]);
    pre[4 + j] = be64_from_le32(pw[2 * j], pw[2 * j + 1]);
  }
  return !bad;
}

// K1a with two votes per lane (TXV_K1A_PAIR=1, experiment): lane t takes votes t and t + n/2 and
// runs their SHA-512 compressions interleaved (sha512_block2), so the dependent round chain of one
// has the other's as independent work; 2 waves/SIMD at ~2x the VGPRs
__global__ void __launch_bounds__(256, 2) txv_k_challenge2(VerifyArgs a) {
  const uint32_t half = (a.n + 1) / 2;
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= half) return;
  const uint32_t i0 = t, i1 = t + half;
  const bool has1 = i1 < a.n;
  uint32_t s0[16], s1[16];
  uint64_t p0[8], p1[8];
  const bool ok0 = vote_checks(a, i0, s0, p0);
  const bool ok1 = has1 && vote_checks(a, has1 ? i1 : i0, s1, p1);
  if (!ok0 && !ok1) {
    a.ok_out[i0] = 0;
    if (has1) a.ok_out[i1] = 0;
    return;
  }
  const uint32_t j1 = has1 ? i1 : i0;
  MsgView m0{a.msg + i0, a.n_pad, a.msg_words, a.msg_len[i0]};
  MsgView m1{a.msg + j1, a.n_pad, a.msg_words, a.msg_len[j1]};
  uint32_t d0[16], d1[16];
  sha512_prefixed2(d0, p0, m0, d1, p1, m1, 8);
  if (ok0) {
    const sc k = sc_reduce512(d0);
#pragma unroll
    for (int j = 0; j < 8; ++j) a.kbuf[(size_t)j * a.n_pad + i0] = k.v[j];
  }
  a.ok_out[i0] = ok0 ? 2 : 0;
  if (has1) {
    if (ok1) {
      const sc k = sc_reduce512(d1);
#pragma unroll
      for (int j = 0; j < 8; ++j) a.kbuf[(size_t)j * a.n_pad + i1] = k.v[j];
    }
    a.ok_out[i1] = ok1 ? 2 : 0;
  }
}

// K1a: challenges of every pending vote into kbuf
#ifndef TXV_K1A_WAVES
#define TXV_K1A_WAVES 4
#endif
#ifdef TXV_K1A_VGPRS
#define TXV_K1A_VGPR_ATTR __attribute__((amdgpu_num_vgpr(TXV_K1A_VGPRS)))
#else
#define TXV_K1A_VGPR_ATTR
#endif
__global__ void __launch_bounds__(256, TXV_K1A_WAVES) TXV_K1A_VGPR_ATTR txv_k_challenge(VerifyArgs a) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  if (!(a.flags[i] & TXV_FLAG_PENDING)) { a.ok_out[i] = 0; return; }   // K1b may walk every vote
  uint32_t k[8], s[8];
  if (!vote_challenge(a, i, k, s)) { a.ok_out[i] = 0; return; }
#pragma unroll
  for (int j = 0; j < 8; ++j) a.kbuf[(size_t)j * a.n_pad + i] = k[j];
  a.ok_out[i] = 2;   // passed the scalar checks; K1b decides
}

template <int W, typename PtrB>
__device__ __forceinline__ void scalarmult_loop(const VerifyArgs& a, PtrB btab, uint32_t first, uint32_t stride) {
  for (uint32_t idx = first; idx < a.n_work; idx += stride) {
    const uint32_t i = a.order ? a.order[idx] : idx;
    if (a.ok_out[i] != 2) continue;
    const uint32_t v = a.val[i];
    uint32_t s[8], k[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[j] = a.sig[(size_t)(8 + j) * a.n_pad + i]; k[j] = a.kbuf[(size_t)j * a.n_pad + i]; }
    const uint32_t* ta = a.atables + (size_t)tab_slot(a, v) * Tab<W>::kWords;
    ge_ext R = double_scalarmult_w<W>(btab, ta, s, k, true);
    uint32_t enc[8];
    ge_encode_zinv(enc, R.X, R.Y, verify_invert(R.Z));
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) diff |= enc[j] ^ a.sig[(size_t)j * a.n_pad + i];
    a.ok_out[i] = diff == 0;
  }
}

// W = 4: the 74 KB B table is staged in LDS (8 waves per 512-thread block share it)
template <int BLOCK>
__global__ void __launch_bounds__(BLOCK, 2 * BLOCK / 256) txv_k_scalarmult_w4(VerifyArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t btab[Tab<4>::kWords];
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.btable);
    uint4* dst = reinterpret_cast<uint4*>(btab);
    for (int i = threadIdx.x; i < Tab<4>::kWords / 4; i += BLOCK) dst[i] = src[i];
  }
  __syncthreads();
  scalarmult_loop<4>(a, (const uint32_t*)btab, blockIdx.x * BLOCK + threadIdx.x, gridDim.x * BLOCK);
}

// W >= 8: both tables are gathered from L2 / MALL / HBM (the B table is hot in every XCD's
// L2 at W = 8).  Each lane verifies two votes and shares ONE field inversion between them
// (Montgomery's trick: 1/(Z0 Z1) then 1/Z0 = Z1/(Z0 Z1), 1/Z1 = Z0/(Z0 Z1)), saving ~1
// inversion (~250 squarings) per vote pair.  The first vote's (X, Y, Z) waits in LDS
// (column-major, conflict-free) while the second is computed, so it costs no VGPRs.
template <int BLOCK, int W>
__global__ void __launch_bounds__(BLOCK, 2 * BLOCK / 256) txv_k_scalarmult_pair(VerifyArgs a) {
  __shared__ uint32_t park[24][BLOCK];
  // XCD-aware split (speed only): blocks b and b+8 share an XCD under round-robin dispatch,
  // so the blocks of one XCD walk one contiguous eighth of the validator-sorted work list.
  // At any moment an XCD then touches a handful of validators' 396 KB A tables, which fit
  // its 4 MB L2, instead of slices of all of them (MI355X_MICROARCH.md §Workgroup dispatch).
  const uint32_t n_pairs = (a.n_work + 1) / 2;
  const uint32_t groups = gridDim.x >= 8 ? 8u : 1u;
  const uint32_t grp = blockIdx.x % groups, blocks_in_grp = gridDim.x / groups + (grp < gridDim.x % groups);
  const uint32_t chunk = (n_pairs + groups - 1) / groups;
  const uint32_t lo = grp * chunk, hi = min(n_pairs, lo + chunk);
  const uint32_t stride = blocks_in_grp * BLOCK;
  for (uint32_t pr = lo + (blockIdx.x / groups) * BLOCK + threadIdx.x; pr < hi; pr += stride) {
    uint32_t vi[2];
    bool act[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t idx = 2 * pr + h;
      vi[h] = idx < a.n_work ? (a.order ? a.order[idx] : idx) : 0u;
      act[h] = idx < a.n_work && a.ok_out[vi[h]] == 2;
    }
    if (!act[0] && !act[1]) continue;
    ge_ext R;
    for (int h = 0; h < 2; ++h) {
      const uint32_t i = vi[h];
      if (act[h]) {
        const uint32_t v = a.val[i];
        uint32_t s[8], k[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[j] = a.sig[(size_t)(8 + j) * a.n_pad + i]; k[j] = a.kbuf[(size_t)j * a.n_pad + i]; }
        R = double_scalarmult_w<W>(a.btable, a.atables + (size_t)tab_slot(a, v) * Tab<W>::kWords, s, k, true);
      } else {
        R = ge_identity();
      }
      if (h == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          park[j][threadIdx.x] = R.X.v[j];
          park[8 + j][threadIdx.x] = R.Y.v[j];
          park[16 + j][threadIdx.x] = R.Z.v[j];
        }
      }
    }
    fe X0, Y0, Z0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      X0.v[j] = park[j][threadIdx.x];
      Y0.v[j] = park[8 + j][threadIdx.x];
      Z0.v[j] = park[16 + j][threadIdx.x];
    }
    const fe inv = verify_invert(fe_mul(Z0, R.Z));
    uint32_t enc[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 0) ge_encode_zinv(enc, X0, Y0, fe_mul(inv, R.Z));
      else ge_encode_zinv(enc, R.X, R.Y, fe_mul(inv, Z0));
      if (act[h]) {
        uint32_t diff = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) diff |= enc[j] ^ a.sig[(size_t)j * a.n_pad + vi[h]];
        a.ok_out[vi[h]] = diff == 0;
      }
    }
  }
}

// ---------------------------------------------------------------- K1b table walk, prefetched
// The walk's 24 table entries are random 128-byte lines in tens of GB of tables: every one is an
// HBM miss, and per-lane loads of them cost the memory pipeline one line request per 16 bytes
// (8 per entry; measured, tools/microbench/gather_calib.hip: 16M entries 2.00 ms as 8 x 16-byte
// loads per lane, 0.78 ms loaded cooperatively).  So the wave loads its 64 entries together:
// load i (i < 8) fetches entries 8i .. 8i+7, 8 lanes x 16 bytes per entry (one whole line per 8
// lanes), global -> LDS (global_load_lds_dwordx4, no VGPRs; the entry's address comes from its
// lane by ds_bpermute).  The LDS image is lane-linear (load i, lane l at i * 1 KiB + 16 l); lane
// l loads piece ((l & 7) + e) & 7 of entry e = 8i + (l >> 3), which makes the pieces a reader
// lane wants land in distinct banks (8 consecutive readers -> 8 distinct 16-byte slots of a
// 256-byte row).  Entry t + 1 is issued once entry t has been read out, so it has a whole
// addition (x the other waves) to arrive.  LDS per wave 8 KiB; 64 KiB per 512-thread block.
// Schedule: B0 A0 B1 A1 ... (B positions first exhausted at W_B > W_A).
#ifndef TXV_K1B_PREFETCH
#define TXV_K1B_PREFETCH 1
#endif

// TXV_K1B_NO_GATHER=1 (experiment builds only, tools/microbench/walk_rate): issue no gathers, the
// walk reads whatever the LDS buffers hold -- the walk's time without its table traffic
#ifndef TXV_K1B_NO_GATHER
#define TXV_K1B_NO_GATHER 0
#endif
// the wave's 64 entries (entry index e_l of lane l, 128-byte units from base) -> buf
__device__ __forceinline__ void entries_to_lds(const uint32_t* base, uint32_t e_l, uint4* buf) {
  if (TXV_K1B_NO_GATHER) return;
  const int lane = threadIdx.x & 63;
  // all 8 permutes first (one LDS round trip instead of one per load: the compiler waits for
  // outstanding LDS operations before each LDS-DMA issue)
  uint32_t e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) e[i] = (uint32_t)__builtin_amdgcn_ds_bpermute((8 * i + (lane >> 3)) << 2, (int)e_l);
  TXV_SCHED_FENCE();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t piece = (uint32_t)((lane & 7) + 8 * i + (lane >> 3)) & 7u;
    const uint32_t* g = base + (size_t)e[i] * kEntryWords + piece * 4u;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)(buf + 64 * i), 16, 0, 0);
  }
}

// piece j of this lane's entry in the image entries_to_lds wrote
__device__ __forceinline__ const uint4* entry_piece(const uint4* buf, int j) {
  const int e = threadIdx.x & 63;
  return buf + 64 * (e >> 3) + 8 * (e & 7) + ((j - e) & 7);
}

// one field of the lane's entry; role 0 = qp, 1 = qm (swapped for -Q by the piece choice),
// 2 = qd.  Words 0..9 = pieces 0, 1, 2.xy; 12..21 = pieces 3, 4, 5.xy; qd = 5.zw, 6, 7.
__device__ __forceinline__ fe10 entry_field_lds(const uint4* buf, bool neg, int role) {
  fe10 r;
  if (role == 2) {
    const uint2 d0 = reinterpret_cast<const uint2*>(entry_piece(buf, 5))[1];
    const uint4 d1 = *entry_piece(buf, 6), d2 = *entry_piece(buf, 7);
    r.v[0] = d0.x; r.v[1] = d0.y; r.v[2] = d1.x; r.v[3] = d1.y;
    r.v[4] = d1.z; r.v[5] = d1.w; r.v[6] = d2.x; r.v[7] = d2.y; r.v[8] = d2.z; r.v[9] = d2.w;
    return r;
  }
  const int j0 = (neg != (role == 1)) ? 3 : 0;
  const uint4 p0 = *entry_piece(buf, j0), p1 = *entry_piece(buf, j0 + 1);
  const uint2 p2 = *reinterpret_cast<const uint2*>(entry_piece(buf, j0 + 2));
  r.v[0] = p0.x; r.v[1] = p0.y; r.v[2] = p0.z; r.v[3] = p0.w;
  r.v[4] = p1.x; r.v[5] = p1.y; r.v[6] = p1.z; r.v[7] = p1.w; r.v[8] = p2.x; r.v[9] = p2.y;
  return r;
}

// tb: the B table; ta: the validators' tables, va = this lane's validator (entries of validator v
// start at entry v * positions * entries)
template <int WB, int WA, int PD>
__device__ __forceinline__ ge_ext double_scalarmult_pf(const uint32_t* tb, const uint32_t* ta, uint32_t va,
                                                       const uint32_t s_in[8], const uint32_t k_in[8], uint4* buf) {
  static_assert(WB >= WA, "B window must be at least the A window");
  static_assert(PD == 1 || PD == 2, "prefetch depth");
  constexpr int nB = Tab<WB>::kPositions, nA = Tab<WA>::kPositions, nT = nB + nA;
  uint32_t s[8], k[8], cs = 0, ck = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) { s[i] = s_in[i]; k[i] = k_in[i]; }
  // entry t of the schedule: its digit (consumed from s or k in order), table lines -> LDS
  // buffer t % PD
  auto issue = [&](int t) -> bool {
    const bool isB = t < 2 * nB && !(t & 1);
    const int pos = t < 2 * nB ? (t >> 1) : t - nB;
    uint4* b = buf + (PD == 2 ? (t & 1) * 512 : 0);
    if (isB) {
      const int d = next_digit<WB>(s, cs);
      entries_to_lds(tb, (uint32_t)(pos * Tab<WB>::kEntries + (d < 0 ? -d : d)), b);
      return d < 0;
    }
    const int d = table_digit<WA>(k, ck, pos);
    entries_to_lds(ta, (uint32_t)(va * (uint32_t)(Tab<WA>::kWords / kEntryWords) + pos * Tab<WA>::kEntries + (d < 0 ? -d : d)), b);
    return d > 0;                                   // [k](-A): a positive digit subtracts
  };
  ge10_ext P;
  bool neg = issue(0), neg2 = false;
  if (PD == 2) neg2 = issue(1);
#pragma unroll 1
  for (int t = 0; t < nT - 1; ++t) {
    // entry t has landed in LDS (with PD = 2 entry t + 1's 8 loads may stay in flight)
    if (PD == 2 && t + 1 < nT) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const bool neg_t = neg;
    const uint4* bt = buf + (PD == 2 ? (t & 1) * 512 : 0);
    auto next = [&]() {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");      // read out before the next DMA lands
      if (PD == 2) {
        neg = neg2;
        if (t + 2 < nT) neg2 = issue(t + 2);
      } else if (t + 1 < nT) {
        neg = issue(t + 1);
      }
    };
    if (t) {
      P = ge10_madd_rd(P, [&](int role) { return entry_field_lds(bt, neg_t, role); }, neg_t, next);
    } else {
      const fe10 qp = entry_field_lds(bt, neg_t, 0), qm = entry_field_lds(bt, neg_t, 1);
      next();
      P = ge10_from_entry(qp, qm);
    }
  }
  {   // the last addition: nothing left to prefetch, and its T is never read
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint4* bt = buf + (PD == 2 ? ((nT - 1) & 1) * 512 : 0);
    const bool neg_t = neg;
    P = ge10_madd_rd<false>(P, [&](int role) { return entry_field_lds(bt, neg_t, role); }, neg_t, [] {});
  }
  ge_ext R;
  R.X = fe_from_fe10(P.X);
  R.Y = fe_from_fe10(P.Y);
  R.Z = fe_from_fe10(P.Z);
  R.T = fe_zero();
  return R;
}

// The same walk with the entry fields staged in VGPRs (TXV_K1B_REGSTAGE, the default): addition
// t starts with entry t's three fields already in registers; entry t+1's are read out of LDS
// right after addition t's first three products consumed entry t's (the registers are free
// then), so the LDS read latency hides behind the last four products instead of stalling in
// front of each field's first use; once they are read the buffer takes entry t+3's gather.
// Two LDS buffers per wave as in double_scalarmult_pf<.., .., 2>: entry t+1 lands during
// addition t-1, t+2 during addition t.
template <int WB, int WA>
__device__ __forceinline__ ge_ext double_scalarmult_rs(const uint32_t* tb, const uint32_t* ta, uint32_t va,
                                                       const uint32_t s_in[8], const uint32_t k_in[8], uint4* buf) {
  static_assert(WB >= WA, "B window must be at least the A window");
  constexpr int nB = Tab<WB>::kPositions, nA = Tab<WA>::kPositions, nT = nB + nA;
  static_assert(nT >= 4, "schedule too short");
  uint32_t s[8], k[8], cs = 0, ck = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) { s[i] = s_in[i]; k[i] = k_in[i]; }
  auto issue = [&](int t) -> bool {           // entry t's digit and gather into buffer t % 2
    const bool isB = t < 2 * nB && !(t & 1);
    const int pos = t < 2 * nB ? (t >> 1) : t - nB;
    uint4* b = buf + (t & 1) * 512;
    if (isB) {
      const int d = next_digit<WB>(s, cs);
      entries_to_lds(tb, (uint32_t)(pos * Tab<WB>::kEntries + (d < 0 ? -d : d)), b);
      return d < 0;
    }
    const int d = table_digit<WA>(k, ck, pos);
    entries_to_lds(ta, (uint32_t)(va * (uint32_t)(Tab<WA>::kWords / kEntryWords) + pos * Tab<WA>::kEntries + (d < 0 ? -d : d)), b);
    return d > 0;                                   // [k](-A): a positive digit subtracts
  };
  const bool n0 = issue(0), n1a = issue(1);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");     // entry 0 landed
  fe10 qp = entry_field_lds(buf, n0, 0), qm = entry_field_lds(buf, n0, 1), qd;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bool nq2 = issue(2);
  ge10_ext P = ge10_from_entry(qp, qm);
  TXV_SCHED_FENCE();
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");     // entry 1 landed
  qp = entry_field_lds(buf + 512, n1a, 0);
  qm = entry_field_lds(buf + 512, n1a, 1);
  qd = entry_field_lds(buf + 512, n1a, 2);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bool ncur = n1a, nq1 = nq2;
  nq2 = issue(3);
  TXV_SCHED_FENCE();
#pragma unroll 1
  for (int t = 1; t < nT; ++t) {
    // VGPRs: entry t; LDS: entry t+1 (buffer (t+1) % 2) and t+2 (buffer t % 2), both gathers
    // possibly in flight
    const bool more = t + 1 < nT;
    const fe10 C = fe10_cneg(fe10_mul(P.T, qd), ncur);
    TXV_SCHED_FENCE();
    const fe10 A = fe10_mul(fe10_sub(P.Y, P.X), qm);
    TXV_SCHED_FENCE();
    const fe10 B = fe10_mul(fe10_add(P.Y, P.X), qp);
    TXV_SCHED_FENCE();
    if (more) {
      if (t + 2 < nT) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // entry t+1 landed
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint4* bn = buf + ((t + 1) & 1) * 512;
      qp = entry_field_lds(bn, nq1, 0);
      qm = entry_field_lds(bn, nq1, 1);
      qd = entry_field_lds(bn, nq1, 2);
    }
    TXV_SCHED_FENCE();
    const fe10 E = fe10_sub(B, A), H = fe10_add(B, A);
    const fe10 G = fe10_add(P.Z, C), F = fe10_sub(P.Z, C);
    ge10_ext r;
    r.X = fe10_mul(F, E);
    TXV_SCHED_FENCE();
    if (more) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");      // entry t+1 read out of its buffer
      ncur = nq1;
      nq1 = nq2;
      if (t + 3 < nT) nq2 = issue(t + 3);
    }
    TXV_SCHED_FENCE();
    r.Y = fe10_mul(H, G);
    TXV_SCHED_FENCE();
    r.Z = fe10_mul(F, G);
    TXV_SCHED_FENCE();
    r.T = more ? fe10_mul(H, E) : fe10_zero();           // the last addition's T is never read
    TXV_SCHED_FENCE();
    P = r;
  }
  ge_ext R;
  R.X = fe_from_fe10(P.X);
  R.Y = fe_from_fe10(P.Y);
  R.Z = fe_from_fe10(P.Z);
  R.T = fe_zero();
  return R;
}

#ifndef TXV_K1B_REGSTAGE
#define TXV_K1B_REGSTAGE 1
#endif
template <int WB, int WA, int PD>
__device__ __forceinline__ ge_ext k1b_walk(const uint32_t* tb, const uint32_t* ta, uint32_t va, const uint32_t s[8],
                                           const uint32_t k[8], uint4* buf) {
  if constexpr (TXV_K1B_REGSTAGE && PD == 2) return double_scalarmult_rs<WB, WA>(tb, ta, va, s, k, buf);
  else return double_scalarmult_pf<WB, WA, PD>(tb, ta, va, s, k, buf);
}

// W >= 8, V votes per lane sharing ONE field inversion (Montgomery's trick over the V
// results: P_h = Z_0 ... Z_h; 1/Z_h = P_{h-1} / P_{V-1} walking back).  The first V-1
// results wait in a global scratch buffer (wave-interleaved: coalesced, L2-resident,
// 128 B per parked vote each way), so the register budget of the scalar multiply is
// unchanged.  V = 4 saves 3/4 of an inversion (~190 squarings) per vote versus V = 1 and
// fills 4 waves/SIMD in one round for a 1M-vote batch on 256 CUs.
// TXV_PARK_LAST: the last vote's (X, Y, Z) is parked too, so only P is live in VGPRs across the
// inversion (the divstep state needs ~40 VGPRs of the 128-VGPR / 4-wave budget)
#ifndef TXV_PARK_LAST
#define TXV_PARK_LAST 1
#endif
// V = 8 is launched for batches that give 2 waves per SIMD (launch_lane_votes), so its register
// budget is 256 VGPRs (2 waves/SIMD); V = 4 too (at 128 VGPRs / 4 waves it spilled ~138 VGPRs:
// 1.57 vs 0.60 ms for a 65k-vote batch, profiles/r02/small_batch)
#ifndef TXV_V4_WAVES
#define TXV_V4_WAVES 2
#endif
// Experiment builds only (time attribution inside K1b; wrong verdicts): TXV_EXP_NO_TAIL=1 skips
// the shared inversion and the encodings (the walks' results still go to the park buffer),
// TXV_EXP_NO_WALK=1 replaces each walk by a point made of the scalar words (the tail alone)
#ifndef TXV_EXP_NO_TAIL
#define TXV_EXP_NO_TAIL 0
#endif
#ifndef TXV_EXP_NO_WALK
#define TXV_EXP_NO_WALK 0
#endif
#ifdef TXV_K1B_VGPRS
#define TXV_K1B_VGPR_ATTR __attribute__((amdgpu_num_vgpr(TXV_K1B_VGPRS)))
#else
#define TXV_K1B_VGPR_ATTR
#endif
template <int BLOCK, int WB, int WA, int V>
__global__ void __launch_bounds__(BLOCK, V == 8 ? 2 : TXV_V4_WAVES * BLOCK / 512) TXV_K1B_VGPR_ATTR txv_k_scalarmult_multi(VerifyArgs a) {
  // lane group g = 64 w + l takes the work-list entries 64 V w + 64 h + l (h < V): the lanes of
  // a wave read 64 consecutive entries per vote slot, so the vote-column reads (sig, kbuf) of an
  // arrival-ordered list are two lines per column per wave
  const uint32_t n_grp = (a.n_work + 64u * V - 1u) / (64u * V) * 64u;
  // XCD-aware split as in the pair kernel: the blocks of one XCD walk one contiguous
  // eighth of the work list (with a validator-sorted list its A tables stay in that XCD's L2);
  // the eighths are whole waves' worth of groups
  const uint32_t groups = gridDim.x >= 8 ? 8u : 1u;
  const uint32_t grp = blockIdx.x % groups, blocks_in_grp = gridDim.x / groups + (grp < gridDim.x % groups);
  const uint32_t chunk = ((n_grp + groups - 1) / groups + 63u) & ~63u;
  const uint32_t lo = grp * chunk, hi = min(n_grp, lo + chunk);
  const uint32_t stride = blocks_in_grp * BLOCK;
  // park layout: [wave][slot h][word][64 lanes]: a wave's stores of one word are one
  // contiguous 256-byte line and every offset is a compile-time immediate
  const uint32_t gwave = (blockIdx.x * BLOCK + threadIdx.x) >> 6;
  uint32_t* park = a.park + (size_t)gwave * (V - 1 + TXV_PARK_LAST) * TXV_PARK_WORDS * 64 + (threadIdx.x & 63);
#if TXV_K1B_PREFETCH
  // V = 8 runs 2 waves/SIMD (one 512-thread block per CU): two 8 KiB entry buffers per wave
  // (prefetch 2 additions ahead, 128 KiB); V = 4 runs two blocks per CU: one buffer (64 KiB)
  constexpr int PD = V == 8 ? 2 : 1;
  __shared__ uint4 pf[BLOCK / 64][PD * 8 * 64];
  // the wave's buffer from a wave-uniform (scalar) index: the LDS-DMA destination goes to M0
  uint4* wbuf = pf[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
#endif
  for (uint32_t g = lo + (blockIdx.x / groups) * BLOCK + threadIdx.x; g < hi; g += stride) {
    uint32_t act = 0;
#pragma unroll
    for (int h = 0; h < V; ++h) {
      const uint32_t idx = (g & ~63u) * V + 64u * h + (g & 63u);
      if (idx < a.n_work && a.ok_out[a.order ? a.order[idx] : idx] == 2) act |= 1u << h;
    }
#if TXV_K1B_PREFETCH
    // the cooperative walk needs every lane of the wave (g < hi is wave-uniform: lo, hi and the
    // wave's first g are multiples of 64): skip only when the whole wave is idle; idle lanes walk
    // the digit-0 (identity) entries of validator 0
    if (__builtin_amdgcn_ballot_w64(act != 0) == 0) continue;
#else
    if (!act) continue;
#endif
    ge_ext R;
    fe P;
#pragma unroll 1
    for (int h = 0; h < V; ++h) {
#if TXV_K1B_PREFETCH
      {
        const bool on = act >> h & 1u;
        const uint32_t idx = (g & ~63u) * V + 64u * h + (g & 63u);
        const uint32_t i = on ? (a.order ? a.order[idx] : idx) : 0u;
        uint32_t s[8], k[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] = on ? a.sig[(size_t)(8 + j) * a.n_pad + i] : 0u;
          k[j] = on ? a.kbuf[(size_t)j * a.n_pad + i] : 0u;
        }
#if TXV_EXP_NO_WALK
        (void)wbuf;
#pragma unroll
        for (int j = 0; j < 8; ++j) { R.X.v[j] = s[j] | 1u; R.Y.v[j] = k[j] | 2u; R.Z.v[j] = s[j] ^ k[j] ^ 5u; R.T.v[j] = 0; }
#else
        R = k1b_walk<WB, WA, PD>(a.btable, a.atables, on ? tab_slot(a, a.val[i]) : 0u, s, k, wbuf);
#endif
      }
#else
      if (act >> h & 1u) {
        const uint32_t idx = (g & ~63u) * V + 64u * h + (g & 63u);
        const uint32_t i = a.order ? a.order[idx] : idx;
        uint32_t s[8], k[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[j] = a.sig[(size_t)(8 + j) * a.n_pad + i]; k[j] = a.kbuf[(size_t)j * a.n_pad + i]; }
        R = double_scalarmult_w2<WB, WA>(a.btable, a.atables + (size_t)tab_slot(a, a.val[i]) * Tab<WA>::kWords, s, k, true);
      } else {
        R = ge_identity();
      }
#endif
      P = h ? fe_mul(P, R.Z) : R.Z;
      if (h < V - 1 || TXV_PARK_LAST) {
        uint32_t* slot = park + h * TXV_PARK_WORDS * 64;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          slot[j * 64] = R.X.v[j];
          slot[(8 + j) * 64] = R.Y.v[j];
          slot[(16 + j) * 64] = P.v[j];
          slot[(24 + j) * 64] = R.Z.v[j];
        }
      }
    }
#if TXV_EXP_NO_TAIL
    if (act & 1u) a.ok_out[(g & ~63u) * V + (g & 63u)] = P.v[0] == 0x12345u;
    continue;
#endif
    fe inv = verify_invert(P);
#pragma unroll 1
    for (int h = V - 1; h >= 0; --h) {
      fe X, Y, Z, zi;
      if (h == V - 1 && !TXV_PARK_LAST) {
        X = R.X; Y = R.Y; Z = R.Z;
      } else {
        const uint32_t* slot = park + h * TXV_PARK_WORDS * 64;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          X.v[j] = slot[j * 64];
          Y.v[j] = slot[(8 + j) * 64];
          Z.v[j] = slot[(24 + j) * 64];
        }
      }
      if (h) {
        const uint32_t* prev = park + (h - 1) * TXV_PARK_WORDS * 64;
        fe Pp;
#pragma unroll
        for (int j = 0; j < 8; ++j) Pp.v[j] = prev[(16 + j) * 64];
        zi = fe_mul(inv, Pp);          // 1/Z_h = P_{h-1} / P_h
        inv = fe_mul(inv, Z);          // 1/P_{h-1}
      } else {
        zi = inv;
      }
      if (act >> h & 1u) {
        const uint32_t idx = (g & ~63u) * V + 64u * h + (g & 63u);
        const uint32_t i = a.order ? a.order[idx] : idx;
        uint32_t enc[8];
        ge_encode_zinv(enc, X, Y, zi);
        uint32_t diff = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) diff |= enc[j] ^ a.sig[(size_t)j * a.n_pad + i];
        a.ok_out[i] = diff == 0;
      }
    }
  }
}

// The same multi-vote K1b with dynamic work (TXV_K1B_DYNAMIC, the default at V = 8): K1b is ONE
// round of waves (2 per SIMD for a 1M-vote batch), so with a static split its time is that of the
// slowest CU -- a CU whose block was dispatched late (a TxFlow kernel of the neighbouring batch
// still held its slots) or that shares its issue slots with one finishes last.  Here every wave
// takes its work in chunks of 64 work entries (one vote slot per lane) from the counter of its
// XCD's eighth of the work list, and from the other eighths once its own is drained: up to V
// chunks share one inversion, and a wave keeps taking chunks (further inversions) while any are
// left.  Each slot parks its lane's vote index beside the point (park word 32).
#ifndef TXV_K1B_DYNAMIC
#define TXV_K1B_DYNAMIC 1
#endif
// TXV_K1B_DYN_WAVES (experiment): waves per SIMD of the work-stealing K1b; 3 needs <= 168 VGPRs and
// one 8 KiB entry buffer per wave (prefetch one addition ahead) to fit the 160 KiB of LDS
#ifndef TXV_K1B_DYN_WAVES
#define TXV_K1B_DYN_WAVES 2
#endif
template <int BLOCK, int WB, int WA, int V, int WAVES, bool FUSED>
__device__ __forceinline__ void k1b_dyn_body(const VerifyArgs& a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t n_chunks = (a.n_work + 63u) / 64u;
  const uint32_t xg = gridDim.x >= 8 ? 8u : 1u, myx = blockIdx.x % xg;
  const uint32_t per = (n_chunks + xg - 1u) / xg;
  const uint32_t gwave = (blockIdx.x * BLOCK + threadIdx.x) >> 6;
  uint32_t* park = a.park + (size_t)gwave * V * TXV_PARK_WORDS * 64 + lane;
  constexpr int PD = WAVES >= 3 ? 1 : 2;
  __shared__ uint4 pf[BLOCK / 64][PD * 8 * 64];
  uint4* wbuf = pf[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
  uint32_t src = 0;                      // ranges tried: (myx + src) % xg
  // the next chunk for this wave (wave-uniform), or 0xFFFFFFFFu when every range is drained
  auto next_chunk = [&]() -> uint32_t {
    while (src < xg) {
      const uint32_t x = (myx + src) % xg;
      const uint32_t end = min(n_chunks, (x + 1u) * per);
      uint32_t c = 0;
      if (lane == 0) c = atomicAdd(a.wctr + 16u * x, 1u);
      c = x * per + __builtin_amdgcn_readfirstlane(c);
      if (c < end) return c;
      ++src;
    }
    return 0xFFFFFFFFu;
  };
  for (;;) {
    ge_ext R;
    fe P;
    uint32_t h = 0;
#pragma unroll 1
    for (; h < (uint32_t)V; ++h) {
      const uint32_t c = next_chunk();
      if (c == 0xFFFFFFFFu) break;
      const uint32_t idx = 64u * c + lane;
      const uint32_t i = idx < a.n_work ? (a.order ? a.order[idx] : idx) : 0u;
      bool on;
      uint32_t s[8], k[8];
      if constexpr (FUSED) {
        // K1a's work for this chunk here (arrival order, every vote of the batch): the SHA-512 of
        // one wave interleaves with the other wave's walk on the SIMD
        on = idx < a.n_work && (a.flags[i] & TXV_FLAG_PENDING) && vote_challenge_call(a, i, k, s);
        if (idx < a.n_work && !on) a.ok_out[i] = 0;
        if (!on) {
#pragma unroll
          for (int j = 0; j < 8; ++j) { s[j] = 0u; k[j] = 0u; }
        }
      } else {
        on = idx < a.n_work && a.ok_out[i] == 2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] = on ? a.sig[(size_t)(8 + j) * a.n_pad + i] : 0u;
          k[j] = on ? a.kbuf[(size_t)j * a.n_pad + i] : 0u;
        }
      }
      // idle lanes walk the digit-0 (identity) entries of validator 0: the cooperative gathers
      // need every lane of the wave
      R = k1b_walk<WB, WA, PD>(a.btable, a.atables, on ? tab_slot(a, a.val[i]) : 0u, s, k, wbuf);
      P = h ? fe_mul(P, R.Z) : R.Z;
      uint32_t* slot = park + h * TXV_PARK_WORDS * 64;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        slot[j * 64] = R.X.v[j];
        slot[(8 + j) * 64] = R.Y.v[j];
        slot[(16 + j) * 64] = P.v[j];
        slot[(24 + j) * 64] = R.Z.v[j];
      }
      slot[32 * 64] = on ? i + 1u : 0u;
    }
    if (h == 0) break;
    fe inv = verify_invert(P);
#pragma unroll 1
    for (int hh = (int)h - 1; hh >= 0; --hh) {
      const uint32_t* slot = park + hh * TXV_PARK_WORDS * 64;
      fe X, Y, Z, zi;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        X.v[j] = slot[j * 64];
        Y.v[j] = slot[(8 + j) * 64];
        Z.v[j] = slot[(24 + j) * 64];
      }
      const uint32_t i1 = slot[32 * 64];
      if (hh) {
        const uint32_t* prev = park + (hh - 1) * TXV_PARK_WORDS * 64;
        fe Pp;
#pragma unroll
        for (int j = 0; j < 8; ++j) Pp.v[j] = prev[(16 + j) * 64];
        zi = fe_mul(inv, Pp);          // 1/Z_h = P_{h-1} / P_h
        inv = fe_mul(inv, Z);          // 1/P_{h-1}
      } else {
        zi = inv;
      }
      if (i1) {
        const uint32_t i = i1 - 1u;
        uint32_t enc[8];
        ge_encode_zinv(enc, X, Y, zi);
        uint32_t diff = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) diff |= enc[j] ^ a.sig[(size_t)j * a.n_pad + i];
        a.ok_out[i] = diff == 0;
      }
    }
    if (h < (uint32_t)V) break;
  }
}

template <int BLOCK, int WB, int WA, int V, int WAVES = 2>
__global__ void __launch_bounds__(BLOCK, WAVES) TXV_K1B_VGPR_ATTR txv_k_scalarmult_dyn(VerifyArgs a) {
  k1b_dyn_body<BLOCK, WB, WA, V, WAVES, false>(a);
}
// TXV_K1B_FUSED=1: K1a's work inside the chunks, capped at the unfused kernel's register budget so
// the TxFlow kernels of the neighbouring batches still find VGPRs beside two K1b waves
#ifndef TXV_K1B_FUSED_VGPRS
#define TXV_K1B_FUSED_VGPRS 200
#endif
template <int BLOCK, int WB, int WA>
__global__ void __launch_bounds__(BLOCK, 2) __attribute__((amdgpu_num_vgpr(TXV_K1B_FUSED_VGPRS)))
txv_k_scalarmult_dyn_fused(VerifyArgs a) {
  k1b_dyn_body<BLOCK, WB, WA, 8, 2, true>(a);
}

// Split mode (lane_votes = 1): the inversion leaves the scalar-multiply kernel.  Under SIMD a
// wave pays the full inversion chain (254 S + 11 M wave instructions) however many of its
// lanes' votes it covers, so its per-vote share only falls with more votes per LANE; inside
// K1b that costs occupancy (V = 8 halves the waves of a 1M batch).  K1b-points therefore
// stores R' = (X, Y, Z) per work entry, column-major by work index (coalesced, 96 B per vote),
// and K1c gives each lane G entries: Montgomery's trick over G (3 multiplies per vote + one
// inversion per G votes instead of per 4) followed by the canonical encoding and the compare
// against the signature's R (x/crypto ed25519.Verify's final bytewise check).
template <int BLOCK, int WB, int WA>
__global__ void __launch_bounds__(BLOCK, 2 * BLOCK / 256) txv_k_scalarmult_points(VerifyArgs a) {
  // XCD-aware split as in the multi kernel: the blocks of one XCD walk a contiguous eighth
  const uint32_t n_grp = (a.n_work + 63u) & ~63u;
  const uint32_t groups = gridDim.x >= 8 ? 8u : 1u;
  const uint32_t grp = blockIdx.x % groups, blocks_in_grp = gridDim.x / groups + (grp < gridDim.x % groups);
  const uint32_t chunk = ((n_grp + groups - 1) / groups + 63u) & ~63u;
  const uint32_t lo = grp * chunk, hi = min(n_grp, lo + chunk);
  const uint32_t stride = blocks_in_grp * BLOCK;
  const size_t np = a.n_pad;
#pragma unroll 1
  for (uint32_t idx = lo + (blockIdx.x / groups) * BLOCK + threadIdx.x; idx < hi; idx += stride) {
    if (idx >= a.n_work) continue;
    const uint32_t i = a.order ? a.order[idx] : idx;
    if (a.ok_out[i] != 2) continue;
    uint32_t s[8], k[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[j] = a.sig[(size_t)(8 + j) * np + i]; k[j] = a.kbuf[(size_t)j * np + i]; }
    const ge_ext R = double_scalarmult_w2<WB, WA>(a.btable, a.atables + (size_t)tab_slot(a, a.val[i]) * Tab<WA>::kWords, s, k, true);
    uint32_t* o = a.rpts + idx;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __builtin_nontemporal_store(R.X.v[j], o + (size_t)j * np);
      __builtin_nontemporal_store(R.Y.v[j], o + (size_t)(8 + j) * np);
      o[(size_t)(16 + j) * np] = R.Z.v[j];
    }
  }
}

// ---------------------------------------------------------------- K1b split (small batches)
// C5's 64k-vote batches leave a one-vote-per-lane walk with 1024 waves (one per SIMD) and its
// 26 dependent additions as the critical path.  Here FOUR lanes share a vote: the schedule of its
// nT = nB + nA table entries (B positions 0..nB-1, then A positions) is cut in four runs of
// ceil(nT / 4) entries, each lane walks its run with the cooperative LDS-DMA gathers of the big
// K1b (per-lane entry addresses: a wave's lanes mix B and A runs), and the lane quad combines its
// four partial sums with two full additions over DPP quad permutes ((0,1)(2,3), then (0,2)(1,3));
// every lane of the quad ends with [s]B + [k](-A), and lane 0 stores R' for K1c (the batched
// inversion + encoding + compare).  4x the waves and ~1/3 of the dependent chain for 5 % more
// multiplies (4 starting entries and 3 x 9-multiply additions instead of 3 mixed additions).
__device__ __forceinline__ void entries_to_lds_p(const uint32_t* p_l, uint4* buf) {
  if (TXV_K1B_NO_GATHER) return;
  const int lane = threadIdx.x & 63;
  const uint64_t addr = (uint64_t)p_l;
  uint32_t lo[8], hi[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int src = (8 * i + (lane >> 3)) << 2;
    lo[i] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)addr);
    hi[i] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(addr >> 32));
  }
  TXV_SCHED_FENCE();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t piece = (uint32_t)((lane & 7) + 8 * i + (lane >> 3)) & 7u;
    const uint32_t* g = reinterpret_cast<const uint32_t*>(((uint64_t)hi[i] << 32) | lo[i]) + piece * 4u;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)(buf + 64 * i), 16, 0, 0);
  }
}

template <int CTRL>
__device__ __forceinline__ fe10 fe10_dpp(const fe10& x) {
  fe10 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)x.v[i], CTRL, 0xF, 0xF, false);
  return r;
}
__device__ __forceinline__ fe10 fe10_sel(bool c, const fe10& x, const fe10& y) {
  fe10 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = c ? x.v[i] : y.v[i];
  return r;
}
__device__ __forceinline__ fe10 fe10_small(uint32_t k) { fe10 r = fe10_zero(); r.v[0] = k; return r; }

// The lane quad's two combining additions (ge.h ge10_add, add-2008-hwcd-3: A = (Y1-X1)(Y2-X2),
// B = (Y1+X1)(Y2+X2), C = 2d T1 T2, D = 2 Z1 Z2, then X3 = EF, Y3 = GH, Z3 = FG, T3 = EH) with
// their products spread over the lanes that compute the same sum -- one multiply instruction
// stream whose operands are chosen per lane -- and the results exchanged by DPP:
// level 1 (pairs (0,1), (2,3)): even lanes A, T1T2, C; odd lanes B, Z1Z2, D; then even X3, Y3,
//   odd Z3, T3: 5 multiplies per lane instead of 9; both lanes of a pair end with the pair's sum
// level 2 ((0,2), (1,3)): lane q one of A, B, T1T2, Z1Z2, lanes 2 / 3 then C / D, every lane
//   reads A..D by quad broadcast; lane q then computes X3 / Y3 / Z3 (q = 0 / 1 / 2): 3 multiplies
//   per lane instead of 9; lane q holds coordinate q of the vote's R' (T3 is not needed)
// Operand bounds as in ge10_add (multiplying by the constant 2 gives D carried).
__device__ __forceinline__ ge10_ext ge10_quad_level1(const ge10_ext& p, uint32_t q) {
  const bool ev = (q & 1u) == 0;
  // one permute per product: a lane sends what its partner needs (the partner of an even lane is
  // odd and vice versa), so the permuted operand is dpp(select of the other parity's choice)
  fe10 r1, r3;
  {
    const fe10 ymx = fe10_sub(p.Y, p.X), ypx = fe10_add(p.Y, p.X);
    r1 = fe10_mul(fe10_sel(ev, ymx, ypx), fe10_dpp<0xB1>(fe10_sel(ev, ypx, ymx)));   // even A, odd B
  }
  TXV_SCHED_FENCE();
  {
    const fe10 r2 = fe10_mul(fe10_sel(ev, p.T, p.Z), fe10_dpp<0xB1>(fe10_sel(ev, p.Z, p.T)));   // T1T2 / Z1Z2
    TXV_SCHED_FENCE();
    r3 = fe10_mul(r2, ev ? fe10_from_fe(fe_const_d2()) : fe10_small(2));   // even C, odd D
  }
  TXV_SCHED_FENCE();
  fe10 E, F, G, H;
  {
    const fe10 o1 = fe10_dpp<0xB1>(r1), o3 = fe10_dpp<0xB1>(r3);
    const fe10 A = fe10_sel(ev, r1, o1), B = fe10_sel(ev, o1, r1), C = fe10_sel(ev, r3, o3), D = fe10_sel(ev, o3, r3);
    E = fe10_sub(B, A); H = fe10_add(B, A); G = fe10_add(D, C); F = fe10_sub(D, C);
  }
  TXV_SCHED_FENCE();
  const fe10 s1 = fe10_mul(F, fe10_sel(ev, E, G));               // even X3 = FE, odd Z3 = FG
  TXV_SCHED_FENCE();
  const fe10 s2 = fe10_mul(H, fe10_sel(ev, G, E));               // even Y3 = HG, odd T3 = HE
  TXV_SCHED_FENCE();
  ge10_ext r;
  {
    const fe10 t1 = fe10_dpp<0xB1>(s1);
    r.X = fe10_sel(ev, s1, t1);
    r.Z = fe10_sel(ev, t1, s1);
  }
  {
    const fe10 t2 = fe10_dpp<0xB1>(s2);
    r.Y = fe10_sel(ev, s2, t2);
    r.T = fe10_sel(ev, t2, s2);
  }
  return r;
}

// level 2: returns coordinate q of the quad's sum (X, Y, Z for q = 0, 1, 2; lane 3: junk)
__device__ __forceinline__ fe10 ge10_quad_level2(const ge10_ext& p, uint32_t q) {
  fe10 r1;
  {
    const fe10 ymx = fe10_sub(p.Y, p.X), ypx = fe10_add(p.Y, p.X);
    // lane q computes A / B / T1T2 / Z1Z2 with partner q ^ 2, which sends T / Z / ymx / ypx to 0 / 1 / 2 / 3
    const fe10 f = fe10_sel(q < 2, fe10_sel(q == 0, ymx, ypx), fe10_sel(q == 2, p.T, p.Z));
    const fe10 h = fe10_sel(q < 2, fe10_sel(q == 0, p.T, p.Z), fe10_sel(q == 2, ymx, ypx));
    r1 = fe10_mul(f, fe10_dpp<0x4E>(h));
  }
  TXV_SCHED_FENCE();
  const fe10 r2 = fe10_mul(r1, q == 2 ? fe10_from_fe(fe_const_d2()) : fe10_small(2));   // lane 2 C, lane 3 D
  TXV_SCHED_FENCE();
  fe10 E, F, G, H;
  {
    const fe10 A = fe10_dpp<0x00>(r1), B = fe10_dpp<0x55>(r1), C = fe10_dpp<0xAA>(r2), D = fe10_dpp<0xFF>(r2);
    E = fe10_sub(B, A); H = fe10_add(B, A); G = fe10_add(D, C); F = fe10_sub(D, C);
  }
  // q = 0: X3 = F E, 1: Y3 = H G, 2: Z3 = F G
  return fe10_mul(fe10_sel(q & 1u, H, F), fe10_sel(q == 0, E, G));
}

#ifndef TXV_SPLIT_WAVES
#define TXV_SPLIT_WAVES 3
#endif
template <int WB, int WA>
__global__ void __launch_bounds__(256, TXV_SPLIT_WAVES) txv_k_scalarmult_split(VerifyArgs a) {
  constexpr int nB = Tab<WB>::kPositions, nA = Tab<WA>::kPositions, nT = nB + nA, per = (nT + 3) / 4;
  __shared__ uint4 pf[4][8 * 64];   // one 8 KiB gather buffer per wave (prefetch one entry ahead)
  uint4* wbuf = pf[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
  const uint32_t lane = threadIdx.x & 63, q = lane & 3;
  const uint32_t n_waves = (a.n_work + 15u) / 16u;   // 16 votes per wave
  const uint32_t stride = gridDim.x * 4u;
  for (uint32_t w = blockIdx.x * 4u + (threadIdx.x >> 6); w < n_waves; w += stride) {   // wave-uniform
    const uint32_t idx = w * 16u + (lane >> 2);
    const uint32_t i = idx < a.n_work ? (a.order ? a.order[idx] : idx) : 0u;
    const bool on = idx < a.n_work && a.ok_out[i] == 2;
    uint32_t s[8], k[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] = on ? a.sig[(size_t)(8 + j) * a.n_pad + i] : 0u;
      k[j] = on ? a.kbuf[(size_t)j * a.n_pad + i] : 0u;
    }
    const uint32_t va = on ? tab_slot(a, a.val[i]) : 0u;
    // every entry of this lane's run up front as (table, entry index), so the scalars are dead
    // before the walk starts: all signed digits of s and k by direct window extraction (carries
    // rippled in order, as next_digit), then run entry j of lane q = schedule entry q * per + j,
    // one of four candidates chosen by q
    uint32_t eidx[per];
    uint32_t negm = 0, am = 0;           // per run entry: negate, A table
    {
      int dB[nB], dA[nA];
      signed_digits<WB, nB>(s, dB);
      signed_digits<WA, nA>(k, dA);
#pragma unroll
      for (int j = 0; j < per; ++j) {
        uint32_t ec[4], nc = 0, ac = 0;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int t = qq * per + j;
          if (t < nB) {
            ec[qq] = (uint32_t)t * Tab<WB>::kEntries + (uint32_t)(dB[t] < 0 ? -dB[t] : dB[t]);
            nc |= (dB[t] < 0 ? 1u : 0u) << qq;
          } else if (t < nT) {
            const int d = dA[t - nB];
            ec[qq] = va * (uint32_t)(Tab<WA>::kWords / kEntryWords) + (uint32_t)(t - nB) * (uint32_t)Tab<WA>::kEntries + (uint32_t)(d < 0 ? -d : d);
            nc |= (d > 0 ? 1u : 0u) << qq;   // [k](-A): a positive digit subtracts
            ac |= 1u << qq;
          } else {
            ec[qq] = 0;                      // beyond the schedule: B position 0, digit 0 = identity
          }
        }
        eidx[j] = q == 0 ? ec[0] : q == 1 ? ec[1] : q == 2 ? ec[2] : ec[3];
        negm |= ((nc >> q) & 1u) << j;
        am |= ((ac >> q) & 1u) << j;
      }
    }
    auto entry_ptr = [&](int j) -> const uint32_t* {
      uint32_t e = eidx[0];
#pragma unroll
      for (int jj = 1; jj < per; ++jj) e = (jj == j) ? eidx[jj] : e;   // j is wave-uniform
      return ((am >> j) & 1u ? a.atables : a.btable) + (size_t)e * kEntryWords;
    };
    entries_to_lds_p(entry_ptr(0), wbuf);
    ge10_ext P;
#pragma unroll 1
    for (int j = 0; j < per; ++j) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // entry j landed in LDS
      const bool nj = (negm >> j) & 1u;
      auto rd = [&](int role) { return entry_field_lds(wbuf, nj, role); };
      auto next = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read out before the next DMA lands
        if (j + 1 < per) entries_to_lds_p(entry_ptr(j + 1), wbuf);
      };
      if (j == 0) {
        const fe10 qp = rd(0), qm = rd(1);
        next();
        P = ge10_from_entry(qp, qm);
      } else {
        P = ge10_madd_rd<true>(P, rd, nj, next);
      }
    }
    P = ge10_quad_level1(P, q);                 // lanes 0, 1: P0 + P1; lanes 2, 3: P2 + P3
    const fe10 coord = ge10_quad_level2(P, q);  // lane q < 3: coordinate q of R' = sum of the four
    if (q < 3 && on) {                          // lane q stores coordinate q (rpts words 8q..8q+7)
      const fe c = fe_from_fe10(coord);
      uint32_t* o = a.rpts + idx + (size_t)(8 * q) * a.n_pad;
      const size_t np = a.n_pad;
#pragma unroll
      for (int j = 0; j < 8; ++j) __builtin_nontemporal_store(c.v[j], o + (size_t)j * np);
    }
  }
}

// K1c: lane t takes the work entries (t & ~63) G + 64 h + (t & 63), h < G (a wave reads 64
// consecutive entries per slot).  Pass 1 stores each active entry's exclusive prefix product
// E_h = prod of the earlier active Z (words 24..31, skipped for the first); pass 2 walks back
// from 1/P: 1/Z_h = E_h / (E_h Z_h), then 1/(E_h) = (1/(E_h Z_h)) Z_h.
template <int G>
__global__ void __launch_bounds__(64) txv_k_batch_encode(VerifyArgs a) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  const uint32_t base = (t & ~63u) * G + (t & 63u);
  const size_t np = a.n_pad;
  uint32_t act = 0;
  fe P;
#pragma unroll 1
  for (int h = 0; h < G; ++h) {
    const uint32_t idx = base + 64u * h;
    if (idx >= a.n_work) break;
    const uint32_t i = a.order ? a.order[idx] : idx;
    if (a.ok_out[i] != 2) continue;
    uint32_t* e = a.rpts + idx;
    fe Z;
#pragma unroll
    for (int j = 0; j < 8; ++j) Z.v[j] = e[(size_t)(16 + j) * np];
    if (act) {
#pragma unroll
      for (int j = 0; j < 8; ++j) e[(size_t)(24 + j) * np] = P.v[j];
      P = fe_mul(P, Z);
    } else {
      P = Z;
    }
    act |= 1u << h;
  }
  if (!act) return;
  const int first = __builtin_ctz(act);
  fe inv = verify_invert(P);
#pragma unroll 1
  for (int h = G - 1; h >= first; --h) {
    if (!(act >> h & 1u)) continue;
    const uint32_t idx = base + 64u * h;
    const uint32_t i = a.order ? a.order[idx] : idx;
    const uint32_t* e = a.rpts + idx;
    fe X, Y, zi;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      X.v[j] = __builtin_nontemporal_load(e + (size_t)j * np);
      Y.v[j] = __builtin_nontemporal_load(e + (size_t)(8 + j) * np);
    }
    if (h > first) {
      fe Z, E;
#pragma unroll
      for (int j = 0; j < 8; ++j) { Z.v[j] = e[(size_t)(16 + j) * np]; E.v[j] = e[(size_t)(24 + j) * np]; }
      zi = fe_mul(inv, E);
      inv = fe_mul(inv, Z);
    } else {
      zi = inv;
    }
    uint32_t enc[8];
    ge_encode_zinv(enc, X, Y, zi);
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) diff |= enc[j] ^ a.sig[(size_t)j * np + i];
    a.ok_out[i] = diff == 0;
  }
}

// ---------------------------------------------------------------- load generator
// keygen: seed (32 B) -> expanded secret scalar a (mod L), prefix, public key encoding
__global__ void __launch_bounds__(64) txv_k_keygen(const uint32_t* __restrict__ seeds_le, uint32_t n,
                                                   const uint32_t* __restrict__ btable,
                                                   uint32_t* __restrict__ scal_out,   // n x 8 (a mod L)
                                                   uint32_t* __restrict__ araw_out,   // n x 8 (clamped a)
                                                   uint32_t* __restrict__ prefix_out, // n x 8 (LE words)
                                                   uint32_t* __restrict__ pub_out) {  // n x 8 (LE words)
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  uint64_t pre[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) pre[j] = be64_from_le32(seeds_le[i * 8 + 2 * j], seeds_le[i * 8 + 2 * j + 1]);
  MsgView none{nullptr, 0, 0, 0};
  uint32_t h[16];
  sha512_prefixed(h, pre, 4, none);
  h[0] &= 0xfffffff8u; h[7] &= 0x7fffffffu; h[7] |= 0x40000000u;
  uint32_t x[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) x[j] = j < 8 ? h[j] : 0u;
  sc a = sc_reduce512(x);
  uint32_t zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  ge_ext P = double_scalarmult_fixed(btable, btable, a.v, zero, false);
  uint32_t enc[8];
  ge_encode(enc, P);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    scal_out[i * 8 + j] = a.v[j];
    araw_out[i * 8 + j] = h[j];
    prefix_out[i * 8 + j] = h[8 + j];
    pub_out[i * 8 + j] = enc[j];
  }
}

// sign: S = (r + k*a) mod L with r = SHA-512(prefix || M), R = [r]B, k = SHA-512(R || A || M)
__global__ void __launch_bounds__(64) txv_k_sign(SignArgs a) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t v = a.val[i];
  MsgView m{a.msg + i, a.n_pad, a.msg_words, a.msg_len[i]};
  uint64_t pre[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) pre[j] = be64_from_le32(a.prefix[v * 8 + 2 * j], a.prefix[v * 8 + 2 * j + 1]);
  uint32_t h[16];
  sha512_prefixed(h, pre, 4, m);
  sc r = sc_reduce512(h);
  uint32_t zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  ge_ext R = double_scalarmult_fixed(a.btable, a.btable, r.v, zero, false);
  uint32_t Rw[8];
  ge_encode(Rw, R);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    pre[j] = be64_from_le32(Rw[2 * j], Rw[2 * j + 1]);
    pre[4 + j] = be64_from_le32(a.pub[v * 8 + 2 * j], a.pub[v * 8 + 2 * j + 1]);
  }
  sha512_prefixed(h, pre, 8, m);
  sc k = sc_reduce512(h);
  // k * a + r  (a = clamped raw scalar; reduction of the 512-bit sum mod L)
  uint32_t t[16];
  {
    uint64_t acc = 0; uint32_t ovf = 0;
#pragma unroll
    for (int c = 0; c < 15; ++c) {
#pragma unroll
      for (int j = (c > 7 ? c - 7 : 0); j <= (c < 7 ? c : 7); ++j) mac(acc, ovf, k.v[j], a.araw[v * 8 + c - j]);
      t[c] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)ovf << 32);
      ovf = 0;
    }
    t[15] = (uint32_t)acc;
    uint64_t cc;
    add_cc(t[0], cc, t[0], r.v[0]);
#pragma unroll
    for (int j = 1; j < 16; ++j) addc_cc(t[j], cc, t[j], j < 8 ? r.v[j] : 0u, cc);
  }
  sc S = sc_reduce512(t);
  // optional corruption hook for the adversarial generator is applied on the host
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a.sig[(size_t)j * a.n_pad + i] = Rw[j];
    a.sig[(size_t)(8 + j) * a.n_pad + i] = S.v[j];
  }
}

// ---------------------------------------------------------------- field self-test
// op 0: a*b  1: a^2  2: a+b  3: a-b  4: canon(a)  5: invert(a)  6: sc_reduce512(a||b)
__global__ void txv_k_fe_selftest(const uint32_t* a, const uint32_t* b, uint32_t* out, uint32_t n, int op) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe x, y;
#pragma unroll
  for (int j = 0; j < 8; ++j) { x.v[j] = a[i * 8 + j]; y.v[j] = b[i * 8 + j]; }
  fe r;
  switch (op) {
    case 0: r = fe_mul(x, y); break;
    case 1: r = fe_sq(x); break;
    case 2: r = fe_add(x, y); break;
    case 3: r = fe_sub(x, y); break;
    case 4: r = fe_canon(x); break;
    case 5: r = fe_invert(x); break;
    default: {
      uint32_t t[16];
#pragma unroll
      for (int j = 0; j < 8; ++j) { t[j] = x.v[j]; t[8 + j] = y.v[j]; }
      sc s = sc_reduce512(t);
#pragma unroll
      for (int j = 0; j < 8; ++j) r.v[j] = s.v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) out[i * 8 + j] = r.v[j];
}

// ---------------------------------------------------------------- host launchers
extern "C" {

}  // extern "C"

template <int W>
static void launch_build(const uint32_t* pubs_le, uint32_t n_points, uint32_t* tables, uint8_t* decode_ok,
                         uint32_t* addr_words, const uint32_t* out_slot, hipStream_t st) {
  const uint64_t lanes = (uint64_t)n_points * Tab<W>::kBuildLanes;
  hipLaunchKernelGGL(txv_k_build_tables<W>, dim3((uint32_t)((lanes + 63) / 64)), dim3(64), 0, st, pubs_le, n_points,
                     tables, decode_ok, addr_words, out_slot);
}

// K1c's votes per lane: the largest G whose launch still gives every SIMD of the chip about a
// quarter wave (1024 SIMDs on MI355X), so the inversion's share per vote falls as the batch grows.
// K1c runs beside the other batches' kernels in a pipeline, so it need not fill the SIMDs itself:
// at C5's 64k-vote batches G = 4 (256 waves) took K1b + K1c from 0.159-0.163 to 0.154 ms in the
// pipeline and the latency to commit from 3.0-3.3 to 2.5-2.9 ms against G = 1 (one wave per SIMD)
// (round 6, same boxes).  TXV_K1C_G overrides it (experiments)
static int k1c_votes_per_lane(uint32_t n_work) {
  static const int forced = [] {
    const char* e = getenv("TXV_K1C_G");
    const int g = e ? atoi(e) : 0;
    return (g == 1 || g == 2 || g == 4 || g == 8 || g == 16 || g == 32) ? g : 0;
  }();
  if (forced) return forced;
  for (int g : {32, 16, 8, 4, 2})
    if ((uint64_t)n_work >= (uint64_t)g * 64 * 256) return g;
  return 1;
}

static hipError_t launch_batch_encode(const VerifyArgs* args, hipStream_t st) {
  const int g = k1c_votes_per_lane(args->n_work);
  const uint32_t grid = (uint32_t)(((uint64_t)args->n_work + 64u * g - 1) / (64u * g));
  switch (g) {
    case 1: hipLaunchKernelGGL(txv_k_batch_encode<1>, dim3(grid), dim3(64), 0, st, *args); break;
    case 2: hipLaunchKernelGGL(txv_k_batch_encode<2>, dim3(grid), dim3(64), 0, st, *args); break;
    case 4: hipLaunchKernelGGL(txv_k_batch_encode<4>, dim3(grid), dim3(64), 0, st, *args); break;
    case 8: hipLaunchKernelGGL(txv_k_batch_encode<8>, dim3(grid), dim3(64), 0, st, *args); break;
    case 16: hipLaunchKernelGGL(txv_k_batch_encode<16>, dim3(grid), dim3(64), 0, st, *args); break;
    default: hipLaunchKernelGGL(txv_k_batch_encode<32>, dim3(grid), dim3(64), 0, st, *args); break;
  }
  return hipSuccess;
}

// V = 2: the LDS-parked pair kernel (WB = WA only); V = 4: parked in args->park;
// V = 1: split mode (points kernel, then K1c)
template <int B, int WB, int WA>
static hipError_t launch_multi(const VerifyArgs* args, uint32_t grid, hipStream_t st) {
  if (args->lane_votes == 1) {
    if (!args->rpts) return hipErrorInvalidValue;
    if constexpr (WB >= 24) {
      // TXV_K1B_SPLIT=0 (experiments): the one-vote-per-lane points kernel instead
      static const bool split = !(getenv("TXV_K1B_SPLIT") && atoi(getenv("TXV_K1B_SPLIT")) == 0);
      if (split) {
        const uint32_t waves = (args->n_work + 15u) / 16u;
        const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((waves + 3u) / 4u, std::max<uint32_t>(args->n_cus, 1u) * TXV_SPLIT_WAVES));
        hipLaunchKernelGGL((txv_k_scalarmult_split<WB, WA>), dim3(blocks), dim3(256), 0, st, *args);
        return launch_batch_encode(args, st);
      }
    }
    hipLaunchKernelGGL((txv_k_scalarmult_points<B, WB, WA>), dim3(grid), dim3(B), 0, st, *args);
    return launch_batch_encode(args, st);
  } else if (args->lane_votes == 4) {
    hipLaunchKernelGGL((txv_k_scalarmult_multi<B, WB, WA, 4>), dim3(grid), dim3(B), 0, st, *args);
  } else if (args->lane_votes == 8) {
    if constexpr (WB >= 24) {
      if (TXV_K1B_DYNAMIC && args->wctr) {
        const hipError_t e = hipMemsetAsync(args->wctr, 0, 8 * 16 * sizeof(uint32_t), st);
        if (e != hipSuccess) return e;
        if constexpr (TXV_K1B_DYN_WAVES >= 3) {
          // persistent: every resident slot (256-thread blocks, TXV_K1B_DYN_WAVES per SIMD)
          // TXV_K1B_DYN_BLOCKS = blocks per CU x 100 (default: every slot); fewer leave SIMDs with
          // room for the neighbouring batches' TxFlow kernels
          // (grid capped at the park buffer's capacity: one V-slot park per wave)
          static const int per100 = getenv("TXV_K1B_DYN_BLOCKS") ? atoi(getenv("TXV_K1B_DYN_BLOCKS")) : 100 * TXV_K1B_DYN_WAVES;
          const uint32_t want = std::max<uint32_t>(8, args->n_cus * (uint32_t)std::max(per100, 1) / 100u);
          const uint32_t grid3 = std::min<uint32_t>(want, args->park_waves / 4u);
          if (!grid3) return hipErrorInvalidValue;
          hipLaunchKernelGGL((txv_k_scalarmult_dyn<256, WB, WA, 8, TXV_K1B_DYN_WAVES>),
                             dim3(grid3), dim3(256), 0, st, *args);
        } else if (args->fused_k1a) {
          hipLaunchKernelGGL((txv_k_scalarmult_dyn_fused<B, WB, WA>), dim3(grid), dim3(B), 0, st, *args);
        } else {
          hipLaunchKernelGGL((txv_k_scalarmult_dyn<B, WB, WA, 8>), dim3(grid), dim3(B), 0, st, *args);
        }
      } else {
        hipLaunchKernelGGL((txv_k_scalarmult_multi<B, WB, WA, 8>), dim3(grid), dim3(B), 0, st, *args);
      }
    } else {
      return hipErrorInvalidValue;
    }
  } else if (args->lane_votes == 2 && WB == WA) {
    hipLaunchKernelGGL((txv_k_scalarmult_pair<B, WA>), dim3(grid), dim3(B), 0, st, *args);
  } else {
    return hipErrorInvalidValue;
  }
  return hipSuccess;
}

extern "C" {

hipError_t txv_launch_build_tables_at(int w, const uint32_t* pubs_le, uint32_t n_points, const uint32_t* out_slot,
                                      uint32_t* tables, uint8_t* decode_ok, uint32_t* addr_words, hipStream_t st) {
  if (!n_points) return hipSuccess;
  switch (w) {
    case 4: launch_build<4>(pubs_le, n_points, tables, decode_ok, addr_words, out_slot, st); break;
    case 8: launch_build<8>(pubs_le, n_points, tables, decode_ok, addr_words, out_slot, st); break;
    case 10: launch_build<10>(pubs_le, n_points, tables, decode_ok, addr_words, out_slot, st); break;
    case 12: launch_build<12>(pubs_le, n_points, tables, decode_ok, addr_words, out_slot, st); break;
    case 14: launch_build<14>(pubs_le, n_points, tables, decode_ok, addr_words, out_slot, st); break;
    case 16: launch_build<16>(pubs_le, n_points, tables, decode_ok, addr_words, out_slot, st); break;
    case 18: launch_build<18>(pubs_le, n_points, tables, decode_ok, addr_words, out_slot, st); break;
    case 20: launch_build<20>(pubs_le, n_points, tables, decode_ok, addr_words, out_slot, st); break;
    case 21: launch_build<21>(pubs_le, n_points, tables, decode_ok, addr_words, out_slot, st); break;
    case 22: launch_build<22>(pubs_le, n_points, tables, decode_ok, addr_words, out_slot, st); break;
    case 24: launch_build<24>(pubs_le, n_points, tables, decode_ok, addr_words, out_slot, st); break;
    case 26: launch_build<26>(pubs_le, n_points, tables, decode_ok, addr_words, out_slot, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t txv_launch_build_tables(int w, const uint32_t* pubs_le, uint32_t n_points, uint32_t* tables,
                                   uint8_t* decode_ok, uint32_t* addr_words, hipStream_t st) {
  return txv_launch_build_tables_at(w, pubs_le, n_points, nullptr, tables, decode_ok, addr_words, st);
}

// (wb, wa): base-point and validator windows; supported pairs are (w, w) for every table
// window, the radix-2^24 base table over wa = 12..20, the radix-2^26 one (43 GB: 10 positions
// instead of 11) over wa = 16..21 (21: the 12-position long-top layout, Tab<21>), and wb in
// {20, 22} over wa = 16
bool txv_verify_windows_supported(int wb, int wa) {
  if (wb == wa) return wa == 4 || wa == 8 || wa == 10 || wa == 12 || wa == 14 || wa == 16;
  if (wb == 24) return wa == 12 || wa == 14 || wa == 16 || wa == 18 || wa == 20;
  if (wb == 26) return wa == 16 || wa == 18 || wa == 20 || wa == 21;
  return wa == 16 && (wb == 20 || wb == 22);
}

bool txv_k1b_fusable(int wb, const VerifyArgs* args) {
  return TXV_K1B_DYNAMIC && TXV_K1B_DYN_WAVES < 3 && wb >= 24 && args->lane_votes == 8 && args->wctr && !args->order;
}

// K1a alone (the AddVote pipeline runs it on another stream than K1b, beside the previous
// batch's K1b: K1b leaves ~116 VGPRs per SIMD free, room for one K1a wave)
hipError_t txv_launch_challenge(const VerifyArgs* args, hipStream_t st) {
  if (!args->n) return hipSuccess;
  static const bool pair = getenv("TXV_K1A_PAIR") && atoi(getenv("TXV_K1A_PAIR")) == 1;
  if (pair) {
    const uint32_t half = (args->n + 1) / 2;
    hipLaunchKernelGGL(txv_k_challenge2, dim3((half + 255) / 256), dim3(256), 0, st, *args);
  } else {
    hipLaunchKernelGGL(txv_k_challenge, dim3((args->n + 255) / 256), dim3(256), 0, st, *args);
  }
  return hipGetLastError();
}

hipError_t txv_launch_verify(int wb, int wa, const VerifyArgs* args, uint32_t grid, hipStream_t st) {
  if (!args->n) return hipSuccess;
  if (!txv_verify_windows_supported(wb, wa)) return hipErrorInvalidValue;
  // K1a stays a separate launch: fused into the 4-vote kernel (128-VGPR budget) the SHA-512
  // phase spilled and every wave hit its memory stalls at the same time (2.29 vs 2.12 ms)
  hipError_t e0 = txv_launch_challenge(args, st);
  if (e0 != hipSuccess) return e0;
  return txv_launch_scalarmult(wb, wa, args, grid, st);
}

// K1b (+ K1c in split mode) alone, after K1a wrote kbuf and the verdict flags
hipError_t txv_launch_scalarmult(int wb, int wa, const VerifyArgs* args, uint32_t grid, hipStream_t st) {
  if (!args->n) return hipSuccess;
  if (!txv_verify_windows_supported(wb, wa)) return hipErrorInvalidValue;
  if (args->n_work) {
    constexpr int B = TXV_VERIFY_BLOCK;
    hipError_t e = hipSuccess;
    switch (wb * 100 + wa) {
      case 404: hipLaunchKernelGGL(txv_k_scalarmult_w4<B>, dim3(grid), dim3(B), 0, st, *args); break;
      case 808: e = launch_multi<B, 8, 8>(args, grid, st); break;
      case 1010: e = launch_multi<B, 10, 10>(args, grid, st); break;
      case 1212: e = launch_multi<B, 12, 12>(args, grid, st); break;
      case 1414: e = launch_multi<B, 14, 14>(args, grid, st); break;
      case 1616: e = launch_multi<B, 16, 16>(args, grid, st); break;
      case 2016: e = launch_multi<B, 20, 16>(args, grid, st); break;
      case 2216: e = launch_multi<B, 22, 16>(args, grid, st); break;
      case 2412: e = launch_multi<B, 24, 12>(args, grid, st); break;
      case 2414: e = launch_multi<B, 24, 14>(args, grid, st); break;
      case 2416: e = launch_multi<B, 24, 16>(args, grid, st); break;
      case 2418: e = launch_multi<B, 24, 18>(args, grid, st); break;
      case 2420: e = launch_multi<B, 24, 20>(args, grid, st); break;
      case 2616: e = launch_multi<B, 26, 16>(args, grid, st); break;
      case 2618: e = launch_multi<B, 26, 18>(args, grid, st); break;
      case 2620: e = launch_multi<B, 26, 20>(args, grid, st); break;
      case 2621: e = launch_multi<B, 26, 21>(args, grid, st); break;
      default: return hipErrorInvalidValue;
    }
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

hipError_t txv_launch_keygen(const uint32_t* seeds_le, uint32_t n, const uint32_t* btable, uint32_t* scal,
                             uint32_t* araw, uint32_t* prefix, uint32_t* pub, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_keygen, dim3((n + 63) / 64), dim3(64), 0, st, seeds_le, n, btable, scal, araw,
                     prefix, pub);
  return hipGetLastError();
}

hipError_t txv_launch_sign(const SignArgs* args, hipStream_t st) {
  if (!args->n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_sign, dim3((args->n + 63) / 64), dim3(64), 0, st, *args);
  return hipGetLastError();
}

hipError_t txv_launch_fe_selftest(const uint32_t* a, const uint32_t* b, uint32_t* out, uint32_t n, int op,
                                  hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_fe_selftest, dim3((n + 63) / 64), dim3(64), 0, st, a, b, out, n, op);
  return hipGetLastError();
}

}  // extern "C"

// ---------------------------------------------------------------- integer-VALU peak probe
// Measures the chip's issue rate of the two ops a field multiply is made of, so bench.py
// prices roofline.peak on the box it runs on (P must be measured).
template <int OP>
__global__ void __launch_bounds__(256) txv_k_valu_probe(uint32_t* out, uint32_t seed, int iters) {
  uint32_t a[8];
  uint64_t m[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { a[i] = seed + threadIdx.x + i; m[i] = a[i]; }
  const uint32_t b = seed * 3u + 1u, c = seed ^ 0x9e3779b9u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      else asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(m[i]) : "v"(b), "v"(c) : "s0", "s1");
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= a[i] ^ (uint32_t)m[i] ^ (uint32_t)(m[i] >> 32);
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

extern "C" hipError_t txv_launch_valu_probe(int op, uint32_t* out, uint32_t blocks, int iters, hipStream_t st) {
  if (op == 0) hipLaunchKernelGGL(txv_k_valu_probe<0>, dim3(blocks), dim3(256), 0, st, out, 7u, iters);
  else hipLaunchKernelGGL(txv_k_valu_probe<1>, dim3(blocks), dim3(256), 0, st, out, 7u, iters);
  return hipGetLastError();
}
