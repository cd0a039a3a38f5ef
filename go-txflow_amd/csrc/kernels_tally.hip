// kernels_tally.hip — the stake tally of TxFlow.addVote / TxVoteSet.AddVote as a
// data-parallel pass over one batch ("parallel restatement").
//
// Sequential semantics being reproduced (types/vote_set.go:92-166, txflow/service.go:192-234):
// votes of one (tx, validator) group are decided in arrival order; a vote is
//   DUPLICATE / NONDETERMINISTIC if the group already holds an accepted vote (signature
//     bytes equal / different) — decided BEFORE verification;
//   INVALID_SIGNATURE if it fails Verify (not stored, so a later vote may still be added);
//   ADDED otherwise: sum += power, maj23 |= sum >= Total*2/3 + 1.
// Parallel form: f = the smallest arrival index in the group whose vote verifies (one
// 64-bit atomicMin per verified vote on an epoch-tagged key, so no per-batch clearing of
// the [set][validator] table is needed); votes before f keep their verify verdict, f is
// ADDED, later votes compare their signature with f's.  Per set, the commit crossing is the
// first arrival index at which prior_sum + (power of ADDED votes up to it) reaches quorum;
// it is found by one wave per touched set with a bisection over arrival index using
// cross-lane reductions (DPP-lowered __shfl_xor sums).
//
// HBM traffic per vote (algorithmic): set/val/flags/status/ok 4+4+1+1+1, slot 4, tag 8,
// power 8 (L2-resident) ~ 31 B; per ADDED vote +64 B arena write.
#include "txv_device.h"
#include "txv_tally.h"

#define TXV_ST_PENDING 0xFFu
#define TXV_ST_OPEN 0xFEu

__device__ __forceinline__ uint64_t tag_of(uint32_t epoch_hi, uint32_t seq) {
  return ((uint64_t)epoch_hi << 32) | seq;
}

// K2a: groups with an accepted vote from an earlier batch; first-verified candidates
__global__ void __launch_bounds__(256) txv_k_tally_mark(TallyArgs a) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint8_t pre = a.pre[i];
  if (pre != TXV_ST_PENDING) { a.status[i] = pre; return; }
  const uint64_t key = (uint64_t)a.set[i] * a.n_vals + a.val[i];
  const uint32_t slot = a.acc_slot[key];
  if (slot) {
    uint8_t st = TXV_ERR_NONDETERMINISTIC_DEV;
    if (a.flags[i] & TXV_FLAG_SIG64) {
      const uint32_t* acc = a.arena + (size_t)(slot - 1) * 16;
      uint32_t d = 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) d |= acc[j] ^ a.sig[(size_t)j * a.n_pad + i];
      if (!d) st = TXV_DUPLICATE_DEV;
    }
    a.status[i] = st;
    return;
  }
  a.status[i] = TXV_ST_OPEN;
  if (a.ok[i]) atomicMin((unsigned long long*)&a.first_tag[key], (unsigned long long)tag_of(a.epoch_hi, i));
}

// K2b: resolve open votes against the group's first verified vote of this batch
__global__ void __launch_bounds__(256) txv_k_tally_resolve(TallyArgs a) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  if (a.status[i] != TXV_ST_OPEN) return;
  const uint64_t key = (uint64_t)a.set[i] * a.n_vals + a.val[i];
  const uint64_t t = a.first_tag[key];
  uint8_t st;
  if ((uint32_t)(t >> 32) != a.epoch_hi || i < (uint32_t)t) {
    st = TXV_ERR_INVALID_SIGNATURE_DEV;           // failed Verify before (or without) an accepted vote
  } else if (i == (uint32_t)t) {
    st = TXV_ADDED_DEV;
    const uint32_t slot = atomicAdd(a.arena_count, 1u);
    if (slot < a.arena_cap) {
      // whole 64-byte line per lane in four 16-byte stores (4-byte scattered stores cost a
      // partial-line write each: ~480 B of HBM writes per vote measured)
      uint4* dst = reinterpret_cast<uint4*>(a.arena + (size_t)slot * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        dst[q] = make_uint4(a.sig[(size_t)(4 * q) * a.n_pad + i], a.sig[(size_t)(4 * q + 1) * a.n_pad + i],
                            a.sig[(size_t)(4 * q + 2) * a.n_pad + i], a.sig[(size_t)(4 * q + 3) * a.n_pad + i]);
      a.acc_slot[key] = slot + 1;
    } else {
      atomicOr(a.error_flags, TXV_DEVERR_ARENA_FULL);
    }
  } else {
    const uint32_t f = (uint32_t)t;
    st = TXV_ERR_NONDETERMINISTIC_DEV;
    if (a.flags[i] & TXV_FLAG_SIG64) {
      uint32_t d = 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) d |= a.sig[(size_t)j * a.n_pad + f] ^ a.sig[(size_t)j * a.n_pad + i];
      if (!d) st = TXV_DUPLICATE_DEV;
    }
  }
  a.status[i] = st;
}

__device__ __forceinline__ int64_t wave_sum64(int64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// K2c: one wave per touched set: batch power, crossing index, sum/maj23 update
__global__ void __launch_bounds__(256) txv_k_tally_sets(TallyArgs a) {
  const uint32_t t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= a.n_touched) return;
  const uint32_t set = a.touched[t];
  const uint64_t base = (uint64_t)set * a.n_vals;
  int64_t part = 0;
  for (uint32_t v = lane; v < a.n_vals; v += 64) {
    const uint64_t e = a.first_tag[base + v];
    if ((uint32_t)(e >> 32) == a.epoch_hi) part += a.power[v];
  }
  const int64_t batch = wave_sum64(part);
  const int64_t prior = a.set_sum[set];
  const int64_t total = prior + batch;
  uint32_t cross = TXV_NO_CROSS;
  if (prior >= a.quorum) {
    cross = 0;                                       // already committed: every ADDED vote re-fires
  } else if (total >= a.quorum) {
    // smallest s with prior + sum_{seq <= s} power >= quorum
    uint32_t lo = 0, hi = a.n - 1;
    while (lo < hi) {
      const uint32_t mid = lo + ((hi - lo) >> 1);
      int64_t p = 0;
      for (uint32_t v = lane; v < a.n_vals; v += 64) {
        const uint64_t e = a.first_tag[base + v];
        if ((uint32_t)(e >> 32) == a.epoch_hi && (uint32_t)e <= mid) p += a.power[v];
      }
      if (prior + wave_sum64(p) >= a.quorum) hi = mid; else lo = mid + 1;
    }
    cross = lo;
  }
  if (lane == 0) {
    a.set_sum[set] = total;
    const bool maj = total >= a.quorum;
    a.set_cross[set] = cross;
    a.t_sum[t] = total;
    a.t_maj[t] = maj ? 1 : 0;
    a.t_cross[t] = (prior >= a.quorum) ? TXV_NO_CROSS : cross;   // event only on the transition
    if (maj) atomicOr(&a.commit_bitmap[set >> 5], 1u << (set & 31));
  }
}

// K2d: commit side effects fire for ADDED votes at or after the set's crossing
__global__ void __launch_bounds__(256) txv_k_tally_fire(TallyArgs a) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  if (a.status[i] != TXV_ADDED_DEV) return;
  const uint32_t c = a.set_cross[a.set[i]];
  if (c != TXV_NO_CROSS && i >= c) a.status[i] = TXV_ADDED_DEV | 0x80u;
}

extern "C" hipError_t txv_launch_tally(const TallyArgs* args, hipStream_t st) {
  if (!args->n) return hipSuccess;
  const uint32_t g = (args->n + 255) / 256;
  hipLaunchKernelGGL(txv_k_tally_mark, dim3(g), dim3(256), 0, st, *args);
  hipLaunchKernelGGL(txv_k_tally_resolve, dim3(g), dim3(256), 0, st, *args);
  if (args->n_touched)
    hipLaunchKernelGGL(txv_k_tally_sets, dim3((args->n_touched + 3) / 4), dim3(256), 0, st, *args);
  hipLaunchKernelGGL(txv_k_tally_fire, dim3(g), dim3(256), 0, st, *args);
  return hipGetLastError();
}
