// kernels_route.hip — the owner rank's ingest route on the device: the votes a
// CheckTx batch admitted go to the rank owning their TxHash, in arrival order, each rank's votes
// packed into one contiguous buffer (route.h) that the node's RCCL scatter sends as it is.
//
// Reference path: Reactor.Receive (txvotepool/reactor.go:170-190) -> TxVotePool.CheckTxWithInfo
// (txvotepool/txvotepool.go:187-261) -> the TxFlow goroutine's TryAddVote
// (txflow/service.go:123-166).  TxVotePool is one order-dependent LRU with one Size cap, so CheckTx
// runs once for the node (the owner rank); TxFlow shards by transaction: a vote belongs to rank
// SHA-256(TxHash bytes)[0] mod G (txv_shard_of), every TxVoteSet on exactly one rank.
//
// Three launches over one batch (one lane per vote, a wave = 64 consecutive arrival indices):
//   count    admitted? (pool status TXV_POOL_OK), the vote's shard (SHA-256 of its TxHash), and per
//            wave and shard the vote count and TxHash bytes (ballots and wave sums), the longest
//            TxHash per shard (the receiver's SignBytes column bound)
//   scan     one block per shard: exclusive scans of those per-wave counts / bytes over the waves
//            (arrival order), the shard's totals, its buffer header and the 16 zero bytes behind
//            its TxHash arena, its meta entry in mapped host memory
//   scatter  each admitted vote's rank inside its shard = the wave's prefix + its rank among the
//            wave's lanes of that shard (ballot), its TxHash arena offset likewise (a masked wave
//            scan of the lengths); every column written at that position, the TxHash copied
// No atomics on shared words, no host round trip between the launches.
#include <algorithm>

#include "sha2.h"
#include "route.h"

namespace {


__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
// exclusive prefix sum over the wave's lanes
__device__ __forceinline__ uint32_t wave_excl(uint32_t v) {
  const int lane = threadIdx.x & 63;
  uint32_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x - v;
}

// a vote's TxHash length as routed: a nil vote carries none
__device__ __forceinline__ uint32_t routed_len(const RouteArgs& a, uint32_t i) {
  return (a.nil && a.nil[i]) ? 0u : a.th_len[i];
}

__global__ void __launch_bounds__(256) txv_k_route_count(RouteArgs a) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const uint32_t w = i >> 6;
  uint32_t r = 0xFFu, len = 0;
  if (i < a.n) {
    const bool adm = !a.status || a.status[i] == TXV_POOL_OK;
    if (adm) {
      len = routed_len(a, i);
      uint32_t st[8];
      txv::sha256_bytes(a.th + a.th_off[i], len, st);   // txv_shard_of: SHA-256(TxHash)[0] mod G
      r = (st[0] >> 24) % a.G;
    }
    a.shard[i] = (uint8_t)r;
  }
  if (w >= a.nw) return;   // (wave-uniform)
  for (uint32_t s = 0; s < a.G; ++s) {
    const bool mine = r == s;
    const uint64_t m = __ballot(mine);
    if (!m) {
      if ((threadIdx.x & 63) == 0) { a.wcnt[(size_t)w * a.G + s] = 0; a.wbytes[(size_t)w * a.G + s] = 0; }
      continue;
    }
    const uint32_t b = wave_sum(mine ? len : 0u), mx = wave_max(mine ? len : 0u);
    if ((threadIdx.x & 63) == 0) {
      a.wcnt[(size_t)w * a.G + s] = (uint32_t)__popcll(m);
      a.wbytes[(size_t)w * a.G + s] = b;
      if (mx) atomicMax(a.maxhl + s, mx);
    }
  }
}

// block s: exclusive scans of shard s's per-wave counts and bytes, 1024 waves per round
__global__ void __launch_bounds__(1024) txv_k_route_scan(RouteArgs a) {
  const uint32_t s = blockIdx.x;
  __shared__ uint32_t sc[16], sb[16];
  __shared__ uint32_t carry_c, carry_b;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) { carry_c = 0; carry_b = 0; }
  __syncthreads();
  for (uint32_t base = 0; base < a.nw; base += 1024) {
    const uint32_t w = base + threadIdx.x;
    const uint32_t c = w < a.nw ? a.wcnt[(size_t)w * a.G + s] : 0u;
    const uint32_t b = w < a.nw ? a.wbytes[(size_t)w * a.G + s] : 0u;
    const uint32_t ec = wave_excl(c), eb = wave_excl(b);
    if (lane == 63) { sc[wv] = ec + c; sb[wv] = eb + b; }
    __syncthreads();
    uint32_t pc = carry_c, pb = carry_b, tc = 0, tb = 0;
    for (int q = 0; q < 16; ++q) {
      if (q < wv) { pc += sc[q]; pb += sb[q]; }
      tc += sc[q];
      tb += sb[q];
    }
    if (w < a.nw) {
      a.wcnt[(size_t)w * a.G + s] = pc + ec;
      a.wbytes[(size_t)w * a.G + s] = pb + eb;
    }
    __syncthreads();
    if (threadIdx.x == 0) { carry_c += tc; carry_b += tb; }
    __syncthreads();
  }
  const uint64_t n = carry_c, ab = carry_b;
  uint64_t off[txv_route::kNCols];
  const uint64_t total = txv_route::layout(n, ab, a.flags, off);
  uint8_t* base = a.dst + (size_t)s * a.stride;
  if (threadIdx.x < 8) {
    const uint64_t hdr[8] = {txv_route::kMagic, n, ab, a.flags, a.maxhl[s], total, 0, 0};
    reinterpret_cast<uint64_t*>(base)[threadIdx.x] = hdr[threadIdx.x];
  }
  if (threadIdx.x < 16) base[off[txv_route::kArena] + ab + threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    a.tot[2 * s] = n;
    a.tot[2 * s + 1] = ab;
    txv_route_meta m;
    m.n = (uint32_t)n;
    m.max_txhash_len = a.maxhl[s];
    m.flags = a.flags;
    m.reserved = 0;
    m.arena_bytes = ab;
    m.bytes = total;
    a.meta[s] = m;
  }
}

__global__ void __launch_bounds__(256) txv_k_route_scatter(RouteArgs a) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const uint32_t w = i >> 6;
  if (w >= a.nw) return;   // (wave-uniform)
  const uint32_t r = i < a.n ? a.shard[i] : 0xFFu;
  const uint32_t len = r != 0xFFu ? routed_len(a, i) : 0u;
  const uint64_t below = (1ull << (threadIdx.x & 63)) - 1ull;
  uint32_t rank = 0, brank = 0;
  for (uint32_t s = 0; s < a.G; ++s) {
    const bool mine = r == s;
    const uint64_t m = __ballot(mine);
    if (!m) continue;
    const uint32_t e = wave_excl(mine ? len : 0u);
    if (mine) {
      rank = (uint32_t)__popcll(m & below);
      brank = e;
    }
  }
  if (r == 0xFFu) return;
  const uint64_t j = a.wcnt[(size_t)w * a.G + r] + rank;
  const uint64_t bo = a.wbytes[(size_t)w * a.G + r] + brank;
  uint64_t off[txv_route::kNCols];
  (void)txv_route::layout(a.tot[2 * r], a.tot[2 * r + 1], a.flags, off);
  uint8_t* base = a.dst + (size_t)r * a.stride;
  reinterpret_cast<int64_t*>(base + off[txv_route::kHeight])[j] = a.height[i];
  reinterpret_cast<int64_t*>(base + off[txv_route::kSec])[j] = a.ts_sec[i];
  reinterpret_cast<int32_t*>(base + off[txv_route::kNanos])[j] = a.ts_nanos[i];
  reinterpret_cast<uint32_t*>(base + off[txv_route::kOff])[j] = (uint32_t)bo;
  reinterpret_cast<uint32_t*>(base + off[txv_route::kLen])[j] = len;
  reinterpret_cast<uint32_t*>(base + off[txv_route::kAddrLen])[j] = a.addr_len[i];
  reinterpret_cast<uint32_t*>(base + off[txv_route::kSigLen])[j] = a.sig_len[i];
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.addr + (size_t)i * 20);
    uint32_t* d = reinterpret_cast<uint32_t*>(base + off[txv_route::kAddr] + j * 20);
#pragma unroll
    for (int q = 0; q < 5; ++q) d[q] = src[q];
  }
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.sig + (size_t)i * 64);
    uint4* d = reinterpret_cast<uint4*>(base + off[txv_route::kSig] + j * 64);
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = src[q];
  }
  if (a.flags & txv_route::kFlagTxKey) {
    uint4* d = reinterpret_cast<uint4*>(base + off[txv_route::kTxKey] + j * 32);
    if (a.txkey) {
      const uint4* src = reinterpret_cast<const uint4*>(a.txkey + (size_t)i * 32);
      d[0] = src[0];
      d[1] = src[1];
    } else {
      d[0] = make_uint4(0, 0, 0, 0);
      d[1] = make_uint4(0, 0, 0, 0);
    }
  }
  if (a.flags & txv_route::kFlagNil) base[off[txv_route::kNil] + j] = (a.nil && a.nil[i]) ? 1 : 0;
  const uint8_t* src = a.th + a.th_off[i];
  uint8_t* d = base + off[txv_route::kArena] + bo;
  for (uint32_t q = 0; q < len; ++q) d[q] = src[q];
}

}  // namespace

extern "C" hipError_t txv_launch_route(const RouteArgs* ap, hipStream_t st) {
  const RouteArgs& a = *ap;
  hipError_t e;
  if ((e = hipMemsetAsync(a.maxhl, 0, (size_t)a.G * 4, st))) return e;
  const dim3 g((std::max<uint32_t>(a.n, 1) + 255) / 256), b(256);
  hipLaunchKernelGGL(txv_k_route_count, g, b, 0, st, a);
  hipLaunchKernelGGL(txv_k_route_scan, dim3(a.G), dim3(1024), 0, st, a);
  hipLaunchKernelGGL(txv_k_route_scatter, g, b, 0, st, a);
  return hipGetLastError();
}
