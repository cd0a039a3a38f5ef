// lookback.h — single-pass exclusive scans of 0/1 flags by decoupled look-back, shared by the
// pool engine (kernels_pool.hip) and the TxFlow event compaction (kernels_flow.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

constexpr uint32_t kLookbackTile = 1024;   // 256 threads x 4 rounds; item = tile * 1024 + 256 k + t

// Single-pass exclusive scans of 0/1 flags (decoupled look-back) fused into the kernels that
// produce the flags, instead of two hipcub launches per scan.  A block takes the next tile of
// kLookbackTile items by ticket, so every tile it waits for belongs to a block that is already running;
// it ranks its tile's flags (ballots), publishes the tile's aggregate, sums its predecessors'
// published words back to the first inclusive prefix, and publishes its own.  The words carry the
// batch's epoch: nothing is cleared between batches.
__device__ __forceinline__ uint64_t tile_word(uint32_t epoch, uint32_t flag, uint32_t v) {
  return ((uint64_t)(epoch & 0x3FFFFFFFu) << 34) | ((uint64_t)flag << 32) | v;
}
// exclusive prefix of tile `tile` (wave 0 of its block, every lane; the result in every lane):
// flag 1 = aggregate, 2 = inclusive.  The wave reads 64 predecessors' words at once and sums back
// to the nearest inclusive one (a single lane walking them one by one made the last tiles of a
// 128-tile chain wait ~100 dependent loads).  The value travels inside the 8-byte word, so relaxed
// agent-scope atomics on both sides carry it across XCDs (sc1 stores and loads): no release /
// acquire fence, which would write back or invalidate the whole XCD L2 per tile
// (MI355X_MICROARCH.md, inter-workgroup visibility).  A predecessor that never publishes (a broken
// invariant: a stale tag, a ticket left unreset by a failed launch) ends the wait after 2^22 spins
// with err_val or-ed into *err (a sticky device word the host learns of: the batch fails loudly
// instead of carrying a partial prefix), before this tile publishes its own word.
__device__ uint32_t tile_lookback(uint64_t* st, uint32_t tile, uint32_t epoch, uint32_t agg, uint32_t* err,
                                  uint32_t err_val) {
  const int lane = threadIdx.x & 63;
  const uint32_t ep = epoch & 0x3FFFFFFFu;
  if (tile == 0) {
    if (lane == 0) __hip_atomic_store(st, tile_word(epoch, 2, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0) __hip_atomic_store(st + tile, tile_word(epoch, 1, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t prefix = 0, spins = 0;
  for (int32_t j = (int32_t)tile - 1; j >= 0;) {
    const int32_t idx = j - lane;
    // before tile 0 nothing is counted: such lanes read as an inclusive 0
    const uint64_t w = idx >= 0 ? __hip_atomic_load(st + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                : tile_word(epoch, 2, 0);
    const uint32_t f = (uint32_t)(w >> 32) & 3u;
    const bool ok = (uint32_t)(w >> 34) == ep && f != 0;
    const uint64_t incm = __ballot(ok && f == 2), okm = __ballot(ok);
    const int first = incm ? __builtin_ctzll(incm) : 64;          // the nearest inclusive word
    const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
    if ((okm & need) != need) {
      // a predecessor's block is running (tickets are taken at block start): it publishes within
      // microseconds; the bound only keeps a broken invariant from hanging the queue
      if (++spins > (1u << 22)) {
        if (lane == 0 && err) {
          __hip_atomic_fetch_or(err, err_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __threadfence();
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    uint32_t v = lane <= first ? (uint32_t)w : 0u;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    prefix += v;
    if (first < 64) break;
    j -= 64;
  }
  if (lane == 0)
    __hip_atomic_store(st + tile, tile_word(epoch, 2, prefix + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return prefix;
}
// the next tile of chain `ch` for this block
__device__ __forceinline__ uint32_t take_tile(uint32_t* tk) {
  __shared__ uint32_t s_tile;
  if (threadIdx.x == 0) s_tile = atomicAdd(tk, 1u);
  __syncthreads();
  return s_tile;
}
// exclusive ranks of the 4 flags of each thread in item order, plus the tile's exclusive prefix;
// *incl (optional) = the inclusive count through this tile, in every thread
__device__ __forceinline__ void tile_scan(const bool f[4], uint32_t out[4], uint64_t* st, uint32_t tile, uint32_t epoch,
                                          uint32_t* err, uint32_t err_val, uint32_t* incl = nullptr) {
  __shared__ uint32_t cnt[4][4];
  __shared__ uint32_t s_prefix;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t m[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    m[k] = __ballot(f[k]);
    if (lane == 0) cnt[k][w] = (uint32_t)__popcll(m[k]);
  }
  __syncthreads();
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t run = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t before = 0, round = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      before += q < w ? cnt[k][q] : 0u;
      round += cnt[k][q];
    }
    out[k] = run + before + (uint32_t)__popcll(m[k] & below);
    run += round;
  }
  if (w == 0) {                                      // wave 0 looks back (run is block-uniform)
    const uint32_t pre = tile_lookback(st, tile, epoch, run, err, err_val);
    if (lane == 0) s_prefix = pre;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) out[k] += s_prefix;
  if (incl) *incl = s_prefix + run;
}

}  // namespace
