// kernels_tally.hip — the stake tally of TxFlow.addVote / TxVoteSet.AddVote as a
// data-parallel pass over one batch ("parallel restatement").
//
// Sequential semantics being reproduced (types/vote_set.go:92-166, txflow/service.go:192-234):
// votes of one (tx, validator) group are decided in arrival order; a vote is
//   DUPLICATE / NONDETERMINISTIC if the group already holds an accepted vote (signature
//     bytes equal / different) — decided BEFORE verification (and before SignBytes);
//   INVALID_SIGNATURE (or the SignBytes error) if it fails Verify: not stored, so a later
//     vote of the group may still be added;
//   ADDED otherwise: sum += power, maj23 |= sum >= Total*2/3 + 1.
//
// Set-major form (K2a, one wave per touched TxVoteSet): the host stages the batch's pending
// votes grouped by (set, validator) with arrival order kept inside each group (two stable
// counting sorts).  A wave walks its set's votes 64 at a time:
//   * an inclusive segmented min-scan (segments = validator groups, value = position if the
//     vote verified) gives every vote the first verified position F of its group so far:
//     F == none -> INVALID_SIGNATURE, F == own position -> ADDED, F earlier -> compare
//     signature bytes with the vote at F (DUPLICATE / NONDETERMINISTIC);
//   * a group whose validator already has an accepted vote from an earlier batch compares
//     against the arena row of that vote instead;
//   * the ADDED votes (at most one per validator) are listed; the commit crossing (smallest
//     arrival index whose stake prefix reaches quorum) is found by binary lifting over the
//     arrival-index bits, one list pass + wave sum per bit; ADDED votes at or after it fire.
// K2b (arrival order, coalesced) writes the pre-check statuses and copies each ADDED vote's
// signature into arena row arena_base + i, so K2a's per-set traffic stays contiguous.
//
// HBM traffic per vote (algorithmic): tvote/tval 8, ok 1, status 1, acc_slot 4 (per set row,
// contiguous), sig 64 read + 64 arena write per ADDED vote ~ 142 B.
#include "txv_device.h"
#include "txv_tally.h"

#define TXV_ST_PENDING 0xFFu
#define TXV_ERR_SIGNBYTES_DEV 8u
#define TXV_INF 0xFFFFFFFFu

// tval packs the validator index with the per-vote flags the tally needs
#define TXV_TVAL_SIG64 0x80000000u
#define TXV_TVAL_BADMSG 0x40000000u
#define TXV_TVAL_MASK 0x3FFFFFFFu

__device__ __forceinline__ int64_t wave_sum64(int64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
__device__ __forceinline__ uint32_t wave_min32(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o, 64));
  return x;
}

// signature of vote i (column-major sig[16][n_pad]) equals 16 words at q?
__device__ __forceinline__ bool sig_equals_row(const TallyArgs& a, uint32_t i, const uint32_t* q) {
  uint32_t d = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) d |= a.sig[(size_t)j * a.n_pad + i] ^ q[j];
  return d == 0;
}
__device__ __forceinline__ bool sig_equals_vote(const TallyArgs& a, uint32_t i, uint32_t f) {
  uint32_t d = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) d |= a.sig[(size_t)j * a.n_pad + i] ^ a.sig[(size_t)j * a.n_pad + f];
  return d == 0;
}

// ADDED-vote list of a set kept in LDS when it has at most this many entries (every set of a
// <= 256-validator registry): the crossing search reads it ~20 times
constexpr uint32_t kListCap = 256;

__global__ void __launch_bounds__(256) txv_k_tally_sets(TallyArgs a) {
  __shared__ uint32_t l_vote[4][kListCap], l_val[4][kListCap];
  __shared__ int64_t l_pow[4][kListCap];
  const uint32_t t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t wv = threadIdx.x >> 6;
  if (t >= a.n_touched) return;
  const uint32_t set = a.touched[t];
  const uint32_t beg = a.toff[t], end = a.toff[t + 1];
  const size_t row = (size_t)set * a.n_vals;

  // pass 1: group resolution, chunk by chunk, carrying the open group across chunks
  uint32_t carry_val = TXV_INF, carry_first = TXV_INF;
  uint32_t k = 0;            // ADDED votes listed so far (wave-uniform)
  int64_t batch = 0;         // their stake (lane partials)
  for (uint32_t base = beg; base < end; base += 64) {
    const uint32_t p = base + lane;
    const bool valid = p < end;
    const uint32_t i = valid ? a.tvote[p] : 0u;
    const uint32_t tv = valid ? a.tval[p] : TXV_INF;
    const uint32_t v = tv & TXV_TVAL_MASK;
    const bool okv = valid && a.ok[i] == 1 && !(tv & TXV_TVAL_BADMSG);
    const uint32_t prev_v = (uint32_t)__shfl_up((int)v, 1, 64);
    bool head = lane == 0 ? (v != carry_val) : (v != prev_v);
    uint32_t x = okv ? p : TXV_INF;
    if (lane == 0 && !head) x = min(x, carry_first);
    if (!valid) head = true;
    // inclusive segmented min-scan over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
      const bool g = __shfl_up((int)head, d, 64) != 0;
      if (lane >= d && !head) { x = min(x, y); head = g; }
    }
    carry_val = (uint32_t)__shfl((int)v, 63, 64);
    carry_first = (uint32_t)__shfl((int)x, 63, 64);
    bool added = false;
    if (valid) {
      const uint32_t slot = a.acc_slot[row + v];
      uint8_t st;
      if (slot) {
        st = (tv & TXV_TVAL_SIG64) && sig_equals_row(a, i, a.arena + (size_t)(slot - 1) * 16)
                 ? TXV_DUPLICATE_DEV : TXV_ERR_NONDETERMINISTIC_DEV;
      } else if (x == TXV_INF) {
        st = (tv & TXV_TVAL_BADMSG) ? TXV_ERR_SIGNBYTES_DEV : TXV_ERR_INVALID_SIGNATURE_DEV;
      } else if (x == p) {
        added = true;
        st = TXV_ADDED_DEV;
      } else {
        st = (tv & TXV_TVAL_SIG64) && sig_equals_vote(a, i, a.tvote[x]) ? TXV_DUPLICATE_DEV
                                                                         : TXV_ERR_NONDETERMINISTIC_DEV;
      }
      if (!added) a.status[i] = st;
    }
    // list the ADDED votes (compacted in lane order) at beg + k ..
    const uint64_t m = __ballot(added);
    if (added) {
      const uint32_t e = beg + k + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      const int64_t pw = a.power[v];
      a.ent_vote[e] = i;
      a.ent_power[e] = pw;
      a.ent_val[e] = v;
      if (e - beg < kListCap) { l_vote[wv][e - beg] = i; l_pow[wv][e - beg] = pw; l_val[wv][e - beg] = v; }
      batch += pw;
    }
    k += (uint32_t)__popcll(m);
  }
  __threadfence_block();   // the list written above is read back by other lanes of the wave
  const bool in_lds = k <= kListCap;   // wave-uniform

  // pass 2: the commit crossing in arrival order
  const int64_t prior = a.set_sum[set];
  const int64_t total = prior + wave_sum64(batch);
  uint32_t cross = TXV_NO_CROSS;
  if (prior >= a.quorum) {
    cross = 0;                                   // already committed: every ADDED vote re-fires
  } else if (total >= a.quorum) {
    // crossing = the arrival index T at which the stake prefix (in arrival order) first reaches
    // quorum: with g(t) = stake of listed votes with arrival < t (monotone), T is the largest t
    // with prior + g(t) < quorum, found by binary lifting over the bits of t; each probe is one
    // pass over the list (k/64 coalesced, L1-resident loads per lane) and one wave sum, so the
    // cost is O(k log n) instead of a k x k prefix comparison
    const int64_t need = a.quorum - prior;
    uint32_t T = 0;
    for (int b = 31 - __builtin_clz(max(a.n, 2u) - 1u); b >= 0; --b) {
      const uint32_t cand = T | (1u << b);
      int64_t s = 0;
      if (in_lds) {
        for (uint32_t c = lane; c < k; c += 64)
          if (l_vote[wv][c] < cand) s += l_pow[wv][c];
      } else {
        for (uint32_t c = lane; c < k; c += 64)
          if (a.ent_vote[beg + c] < cand) s += a.ent_power[beg + c];
      }
      if (wave_sum64(s) < need) T = cand;
    }
    cross = T;
  }

  // pass 3: ADDED statuses (+ fired bit) and the accepted-vote rows
  for (uint32_t e = lane; e < k; e += 64) {
    const uint32_t ie = in_lds ? l_vote[wv][e] : a.ent_vote[beg + e];
    const uint32_t ve = in_lds ? l_val[wv][e] : a.ent_val[beg + e];
    const bool fire = cross != TXV_NO_CROSS && ie >= cross;
    a.status[ie] = TXV_ADDED_DEV | (fire ? 0x80u : 0u);
    a.acc_slot[row + ve] = a.arena_base + ie + 1u;
  }
  if (lane == 0) {
    a.set_sum[set] = total;
    const bool maj = total >= a.quorum;
    a.t_sum[t] = total;
    a.t_maj[t] = maj ? 1 : 0;
    a.t_cross[t] = (prior >= a.quorum) ? TXV_NO_CROSS : cross;   // event only on the transition
    if (maj) atomicOr(&a.commit_bitmap[set >> 5], 1u << (set & 31));
  }
}

// K2b: pre-check statuses, and the ADDED votes' signatures into their arena rows
__global__ void __launch_bounds__(256) txv_k_tally_finish(TallyArgs a) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint8_t pre = a.pre[i];
  if (pre != TXV_ST_PENDING) {
    a.status[i] = pre;
    a.status_host[i] = pre;
    return;
  }
  const uint8_t st = a.status[i];
  a.status_host[i] = st;
  if ((st & 0x7Fu) != TXV_ADDED_DEV) return;
  // whole 64-byte row per lane in four 16-byte stores
  uint4* dst = reinterpret_cast<uint4*>(a.arena + (size_t)(a.arena_base + i) * 16);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    dst[q] = make_uint4(a.sig[(size_t)(4 * q) * a.n_pad + i], a.sig[(size_t)(4 * q + 1) * a.n_pad + i],
                        a.sig[(size_t)(4 * q + 2) * a.n_pad + i], a.sig[(size_t)(4 * q + 3) * a.n_pad + i]);
}

// TxVoteSet.GetVotes / GetByAddress readers: per validator of one set, the accepted vote's
// arena row (0 = none) and its signature bytes
__global__ void __launch_bounds__(256) txv_k_set_votes(const uint32_t* __restrict__ acc_row, uint32_t n_vals,
                                                       const uint32_t* __restrict__ arena, uint32_t* __restrict__ rows,
                                                       uint32_t* __restrict__ sigs) {
  const uint32_t v = blockIdx.x * 256 + threadIdx.x;
  if (v >= n_vals) return;
  const uint32_t slot = acc_row[v];
  rows[v] = slot;
#pragma unroll
  for (int j = 0; j < 16; ++j) sigs[(size_t)v * 16 + j] = slot ? arena[(size_t)(slot - 1) * 16 + j] : 0u;
}

extern "C" hipError_t txv_launch_set_votes(const uint32_t* acc_row, uint32_t n_vals, const uint32_t* arena, uint32_t* rows,
                                           uint32_t* sigs, hipStream_t st) {
  if (!n_vals) return hipSuccess;
  hipLaunchKernelGGL(txv_k_set_votes, dim3((n_vals + 255) / 256), dim3(256), 0, st, acc_row, n_vals, arena, rows, sigs);
  return hipGetLastError();
}

extern "C" hipError_t txv_launch_tally(const TallyArgs* args, hipStream_t st) {
  if (!args->n) return hipSuccess;
  if (args->n_touched)
    hipLaunchKernelGGL(txv_k_tally_sets, dim3((args->n_touched + 3) / 4), dim3(256), 0, st, *args);
  hipLaunchKernelGGL(txv_k_tally_finish, dim3((args->n + 255) / 256), dim3(256), 0, st, *args);
  return hipGetLastError();
}
