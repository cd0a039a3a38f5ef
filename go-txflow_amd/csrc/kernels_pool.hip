// kernels_pool.hip — TxVotePool ingest on the GPU: txVoteKey(tx) = SHA-256(tx.Signature)
// (txvotepool/txvotepool.go:467-469), the key of the pool's LRU cache (mapTxCache.Push,
// :416-438) and of txsMap, for a whole batch.  One lane per vote; signatures of up to 64 bytes
// (every well-formed vote) are hashed here, longer ones on the host (they are rejected by
// Verify anyway but still occupy pool/cache entries, so their keys must be exact).
#include "sha2.h"
#include "txv_device.h"
#include "txv_hash.h"
#include "lookback.h"

using namespace txv;

// sig: [n][16] u32, the first 64 signature bytes little-endian-loaded; sig_len: [n];
// keys: [n][8] u32 holding the 32 digest bytes in memory order.  Lanes with sig_len > 64 skip.
__global__ void __launch_bounds__(256) txv_k_sig_keys(const uint32_t* __restrict__ sig,
                                                      const uint32_t* __restrict__ sig_len, uint32_t n,
                                                      uint32_t* __restrict__ keys) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t len = sig_len[i];
  if (len > 64) return;
  uint32_t m[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) m[j] = sig[(size_t)i * 16 + j];
  // big-endian message words, zero beyond len, then 0x80, length in bits at the end.
  // len <= 55 fits one block, 56..64 needs two.
  uint32_t st[8], w[16];
  sha256_init(st);
  const uint32_t nblk = len <= 55 ? 1u : 2u;
  for (uint32_t b = 0; b < nblk; ++b) {
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const uint32_t gw = 16u * b + (uint32_t)t;       // global word index (4 bytes each)
      uint32_t v = 0;
      if (gw < 16) {
        const uint32_t word = bswap32(m[gw]);
        const int valid = (int)len - 4 * (int)gw;      // message bytes inside this word
        if (valid >= 4) v = word;
        else if (valid > 0) v = word & (0xFFFFFFFFu << (8 * (4 - valid)));
      }
      if (gw == len / 4) v |= 0x80000000u >> (8 * (len & 3));
      if (gw == 16u * nblk - 1u) v = len * 8u;
      w[t] = v;
    }
    sha256_block(st, w);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) keys[(size_t)i * 8 + j] = bswap32(st[j]);
}

extern "C" hipError_t txv_launch_sig_keys(const uint32_t* sig, const uint32_t* sig_len, uint32_t n, uint32_t* keys,
                                          hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_sig_keys, dim3((n + 255) / 256), dim3(256), 0, st, sig, sig_len, n, keys);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// CheckTx decisions for a batch on the GPU (pool_dev.h; the host engine is runtime.cpp's
// pooldev_*).  The cache's order-dependent semantics are resolved by LRU stack distance, exactly
// as pool.cpp's batch_check does it on the host: S = the L0 cache entries front to back followed
// by the batch's pushes; the push of key k at position e hits iff k occurs earlier in S (last at
// p) and fewer than C distinct keys lie strictly between -- (e - p - 1) minus the pairs of
// consecutive occurrences of one key nested inside (p, e).  Previous occurrences come from a
// sort of the pushes by a 32-bit key slice (stable, so equal slices stay in arrival order; the
// full keys are compared inside a run), cached keys from the cache's index.
#include <hipcub/hipcub.hpp>
#include "pool_dev.h"
#include "../../include/txvote.h"

namespace {

constexpr uint64_t kNoPair = ~0ull;

__device__ __forceinline__ bool key_eq(const uint32_t* keys, uint32_t a, uint32_t b) {
  const uint4* x = reinterpret_cast<const uint4*>(keys + (size_t)a * 8);
  const uint4* y = reinterpret_cast<const uint4*>(keys + (size_t)b * 8);
  const uint4 x0 = x[0], x1 = x[1], y0 = y[0], y1 = y[1];
  return ((x0.x ^ y0.x) | (x0.y ^ y0.y) | (x0.z ^ y0.z) | (x0.w ^ y0.w) | (x1.x ^ y1.x) | (x1.y ^ y1.y) |
          (x1.z ^ y1.z) | (x1.w ^ y1.w)) == 0;
}
__device__ __forceinline__ bool key_eq2(const uint32_t* ka, uint32_t a, const uint32_t* kb, uint32_t b) {
  const uint4* x = reinterpret_cast<const uint4*>(ka + (size_t)a * 8);
  const uint4* y = reinterpret_cast<const uint4*>(kb + (size_t)b * 8);
  const uint4 x0 = x[0], x1 = x[1], y0 = y[0], y1 = y[1];
  return ((x0.x ^ y0.x) | (x0.y ^ y0.y) | (x0.z ^ y0.z) | (x0.w ^ y0.w) | (x1.x ^ y1.x) | (x1.y ^ y1.y) |
          (x1.z ^ y1.z) | (x1.w ^ y1.w)) == 0;
}
// Every placement of a key -- the cache index, the pool list's index, the sort slice that groups
// a batch's repeats -- goes through txv_hash::key32 under the engine's secret seed (a different
// derived seed each), never through a raw key slice: the keys are SHA-256 of peer-supplied
// signature bytes that CheckTx never verifies (txvotepool.go:467-469), so a peer could grind keys
// onto one home slot or one sort slice and make every probe or run scan of the batch quadratic.
constexpr uint64_t kSeedIdx = 0x243F6A8885A308D3ull, kSeedList = 0x13198A2E03707344ull, kSeedSort = 0xA4093822299F31D0ull;
__device__ __forceinline__ uint32_t idx_hash(const uint32_t* k, uint64_t seed) {
  return (uint32_t)txv_hash::key32(k, seed ^ kSeedIdx);
}

// position of key (keys + 8 * i) in the cache (ck / ci of length L), or -1
__device__ __forceinline__ int32_t cache_find(const uint32_t* ck, const uint32_t* ci, uint32_t icap,
                                              const uint32_t* keys, uint32_t i, uint64_t seed) {
  uint32_t s = idx_hash(keys + (size_t)i * 8, seed) & (icap - 1);
  for (uint32_t probe = 0; probe < icap; ++probe, s = (s + 1) & (icap - 1)) {
    const uint32_t v = ci[s];
    if (!v) return -1;
    if (key_eq2(ck, v - 1, keys, i)) return (int32_t)(v - 1);
  }
  return -1;
}

constexpr uint32_t kTile = kLookbackTile;
// the sort key: a 24-bit slice of the key's seeded hash (three radix passes; equal slices are told
// apart by the full key inside their run, and only repeats of one key or a chance collision share
// a run), the non-pushes on the value above every push's
constexpr uint32_t kSliceBits = 24, kSliceNone = (1u << kSliceBits) - 1;
__device__ __forceinline__ uint32_t sort_slice(const uint32_t* k, uint64_t seed) {
  return (uint32_t)(txv_hash::key32(k, seed ^ kSeedSort) >> (64 - kSliceBits));
}

// ---- the pool list in HBM (pool_dev.h PoolListArgs) ----
__device__ __forceinline__ uint32_t list_home(const uint32_t* k, uint64_t seed) {
  return (uint32_t)txv_hash::key32(k, seed ^ kSeedList);
}
__device__ __forceinline__ unsigned long long list_slot(uint32_t tag, uint32_t low) {
  return ((unsigned long long)tag << 32) | low;
}
__device__ __forceinline__ unsigned long long slot_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// entry e's key == k (entries are written by an earlier launch than any reader's)
__device__ __forceinline__ bool list_key_eq(const uint32_t* lk, uint32_t e, const uint32_t k[8]) {
  const uint4* x = reinterpret_cast<const uint4*>(lk + (size_t)e * 8);
  const uint4 x0 = x[0], x1 = x[1];
  return ((x0.x ^ k[0]) | (x0.y ^ k[1]) | (x0.z ^ k[2]) | (x0.w ^ k[3]) | (x1.x ^ k[4]) | (x1.y ^ k[5]) |
          (x1.z ^ k[6]) | (x1.w ^ k[7])) == 0;
}
// txsMap.Store(key, pos): insert, or -- the key indexed already (a vote admitted twice, the
// earlier one still in the list) -- the later position stays indexed, as the sequential Stores
// leave it; the other entry stays in the list, unindexed
__device__ void list_insert(unsigned long long* li, uint32_t imask, const uint32_t* lk, uint32_t pos, const uint32_t k[8],
                            uint64_t seed) {
  const uint32_t tg = k[3];
  const unsigned long long mine = list_slot(tg, pos + 1);
  uint32_t s = list_home(k, seed) & imask;
  for (uint32_t probe = 0; probe <= imask; ++probe, s = (s + 1) & imask) {
    unsigned long long v = slot_load(li + s);
    if (v == 0) {
      v = atomicCAS(li + s, 0ull, mine);
      if (v == 0) return;
    }
    if ((uint32_t)(v >> 32) != tg || (uint32_t)v == kListTomb || !list_key_eq(lk, (uint32_t)v - 1, k)) continue;
    for (;;) {
      if ((uint32_t)v - 1 > pos) return;
      const unsigned long long prev = atomicCAS(li + s, v, mine);
      if (prev == v) return;
      v = prev;                 // another insert of this key took the slot meanwhile
    }
  }
}
// the tile's (entries, bytes) into out[0..1] (one plain store pair per tile, summed on the host:
// no counter to zero before the launch, no atomic on a shared word)
__device__ __forceinline__ void list_partial(uint64_t* out, uint32_t hits, uint64_t bytes) {
  __shared__ uint64_t s_c[4], s_b[4];
  uint64_t c = hits;
  for (int o = 32; o > 0; o >>= 1) {
    bytes += __shfl_xor(bytes, o, 64);
    c += __shfl_xor(c, o, 64);
  }
  if ((threadIdx.x & 63) == 0) { s_c[threadIdx.x >> 6] = c; s_b[threadIdx.x >> 6] = bytes; }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = s_c[0] + s_c[1] + s_c[2] + s_c[3];
    out[1] = s_b[0] + s_b[1] + s_b[2] + s_b[3];
  }
}

// Update's removeTx(tx, e, false) (txvotepool.go:339-344) for committed key k if the index holds
// it: the slot becomes a tombstone, the entry dead (a key twice in the batch: removed once)
__device__ bool list_remove(const PoolListArgs& l, const uint32_t* key) {
  const uint4* src = reinterpret_cast<const uint4*>(key);
  const uint4 k0 = src[0], k1 = src[1];
  const uint32_t k[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
  const uint32_t tg = k[3];
  uint32_t s = list_home(k, l.seed) & l.imask;
  for (uint32_t probe = 0; probe <= l.imask; ++probe, s = (s + 1) & l.imask) {
    const unsigned long long v = slot_load(l.li + s);
    if (v == 0) return false;
    if ((uint32_t)(v >> 32) != tg || (uint32_t)v == kListTomb || !list_key_eq(l.lk, (uint32_t)v - 1, k)) continue;
    if (atomicCAS(l.li + s, v, list_slot(tg, kListTomb)) != v) return false;   // a twin of this key removed it
    l.lfl[(uint32_t)v - 1] = 0;
    return true;
  }
  return false;
}

// pushes, sort input, and aidx = exclusive scan of the pushes (the push's index in S after the
// cache); the ticket counters of pd_status's two scans are reset here.  With the pool list in HBM
// the tiles after the batch's remove Update's committed votes [0, n_force) from it
__global__ void __launch_bounds__(256) pd_init(PoolDevArgs a) {
  // the new cache's index, cleared for pd_newcache (this chain reads only the old one)
  if (a.C)
    for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < a.icap; s += gridDim.x * 256) a.ci_new[s] = 0;
  const uint32_t tile = take_tile(a.tk + 0);
  const uint32_t nt = (a.n + kTile - 1) / kTile;
  if (tile >= nt) {                                // (tickets reset by the previous batch: never)
    const uint32_t rt = tile - nt;
    if (!a.list_on || rt >= (a.n_force + kTile - 1) / kTile) return;
    uint32_t hits = 0;
    uint64_t bytes = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t i = rt * kTile + 256u * k + threadIdx.x;
      if (i < a.n_force && list_remove(a.l, a.keys + (size_t)i * 8)) {
        ++hits;
        bytes += a.sizes[i];      // the committed vote's Size(), as the host path subtracts it
      }
    }
    list_partial(a.res_rm + 2 * rt, hits, bytes);
    return;
  }
  if (tile == 0 && threadIdx.x == 0) {
    a.nfar[0] = 0;          // far pushes (appended by pd_link)
    a.tk[1] = 0;
    a.tk[2] = 0;
  }
  bool f[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = tile * kTile + 256u * k + threadIdx.x;
    f[k] = false;
    if (i >= a.n) continue;
    const bool forced = i < a.n_force;             // Update's committed votes: every one pushes
    const bool ok = forced || !a.valid || a.valid[i - a.n_force] == a.valid_ok;
    const bool p = forced || (ok && (int64_t)a.sizes[i] <= a.max_tx);
    f[k] = p;
    a.push[i] = p;
    // non-pushes sort into a run of their own at the end: a push's slice is clamped below it, so a
    // key whose slice is 0xFFFFFFFF never shares a run with them (pd_link scans its run backwards)
    a.hkey[i] = p ? min(sort_slice(a.keys + (size_t)i * 8, a.seed), kSliceNone - 1) : kSliceNone;
    a.hidx[i] = i;
    a.last[i] = p;          // cleared by pd_link for a push with a later push of its key
  }
  uint32_t r[4];
  tile_scan(f, r, a.tiles, tile, a.epoch, a.err, 1u);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = tile * kTile + 256u * k + threadIdx.x;
    if (i < a.n) a.aidx[i] = r[k];
  }
}

__device__ __forceinline__ uint32_t n_pushes(const PoolDevArgs& a) {
  return a.n ? a.aidx[a.n - 1] + a.push[a.n - 1] : 0u;
}

// per sorted position j, for vote i = sidx[j]: the nearest earlier push of the same key (runs of
// one slice are in arrival order; that push's last[] is cleared -- each push is the nearest later
// occurrence of at most one push, so no two writers), else the key's cache position; then the
// push's decision (batch_check step 2): miss, hit, or far (counted by pd_far), with its pair
// (previous occurrence, this push) in doubled S positions while evicting
__global__ void __launch_bounds__(256) pd_link(PoolDevArgs a) {
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= a.n) return;
  const uint32_t i = a.sidx[j];
  a.pst[i] = kNoPair;
  a.pend[i] = kNoPair;
  if (!a.push[i]) { a.dec[i] = 0; return; }
  const uint32_t h = a.skey[j];
  int32_t pj = -1, cr = -1;
  for (int32_t jj = (int32_t)j - 1; jj >= 0 && a.skey[jj] == h; --jj) {
    const uint32_t k = a.sidx[jj];
    if (a.push[k] && key_eq(a.keys, k, i)) {
      pj = (int32_t)k;
      a.last[k] = 0;
      break;
    }
  }
  const uint64_t C = a.C, L0 = a.C ? *a.clen : 0, na = n_pushes(a);
  if (pj < 0 && C && L0) {
    cr = cache_find(a.ck_old, a.ci_old, a.icap, a.keys, i, a.seed);
    if (cr >= 0) a.detached[cr] = 1;
  }
  const bool cache_on = C != 0, evict = cache_on && L0 + na > C;
  const uint64_t F = L0 < na ? L0 : na;                    // front entries this batch can evict
  const uint64_t e2 = 2 * (L0 + a.aidx[i]);
  uint8_t d = 1;
  uint64_t ps = kNoPair;
  if (pj >= 0) {
    d = !cache_on ? 1 : ((!evict || a.aidx[i] - a.aidx[pj] - 1 < C) ? 2 : 3);
    if (evict) ps = 2 * (L0 + a.aidx[pj]);
  } else if (cr >= 0) {
    const uint64_t r = (uint64_t)cr;
    const bool front = evict && r < F;
    d = (!front || L0 + a.aidx[i] - r - 1 < C) ? 2 : 3;
    if (evict) ps = front ? 2 * r : 2 * L0 - 1;
  }
  a.dec[i] = d;
  if (ps != kNoPair) {                      // the pair (previous occurrence, this push), by arrival index
    a.pst[i] = ps;
    a.pend[i] = e2;
  }
  if (d == 3) a.far[atomicAdd(a.nfar, 1u)] = i;
}

// The far pushes' nested-pair counts in O(log) per block of votes instead of a scan of every pair
// (a peer-controlled stream of replays at window ~C made the scan O(far x pairs)).
// A pair ends where its push stands in S, and pushes stand in S in arrival order, so the pairs
// ending before a far push at arrival index i are exactly the pairs of votes i' < i; what remains
// to count is how many of those start after the far push's previous occurrence.  Each block of
// kXBlock votes sorts its pairs' start positions here (hipcub block radix sort in LDS, votes
// without a pair as 0xFFFFFFFF at the end; xn = pairs in the block) ...
constexpr uint32_t kXBlock = 1024;
__global__ void __launch_bounds__(256) pd_xsort(PoolDevArgs a) {
  using Sort = hipcub::BlockRadixSort<uint32_t, 256, 4>;
  __shared__ typename Sort::TempStorage tmp;
  __shared__ uint32_t wcnt[4];
  const uint32_t base = blockIdx.x * kXBlock;
  uint32_t x[4];
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = base + threadIdx.x * 4 + k;
    const uint64_t p = i < a.n ? a.pst[i] : kNoPair;
    x[k] = p == kNoPair ? 0xFFFFFFFFu : (uint32_t)p;      // S positions are < 2^32 - 1 (host check)
    c += p != kNoPair;
  }
  Sort(tmp).Sort(x);
#pragma unroll
  for (int k = 0; k < 4; ++k) a.xs[base + threadIdx.x * 4 + k] = x[k];
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) wcnt[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) a.xn[blockIdx.x] = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
}

// ... and one wave per far push counts, over the sorted blocks before its own (one binary search
// each, a lane per block) and the votes of its own block before it (a scan), the pairs starting
// after fp: the pairs nested in (fp, fe); then its decision.
__global__ void __launch_bounds__(256) pd_far(PoolDevArgs a) {
  const uint32_t nf = a.nfar[0];
  const uint64_t C = a.C;
  const int lane = threadIdx.x & 63;
  const uint32_t gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  for (uint32_t f = gw; f < nf; f += nw) {
    const uint32_t i = a.far[f];
    const uint64_t fp = a.pst[i], fe = a.pend[i];          // a far push always has its pair (evicting)
    const uint32_t fp32 = (uint32_t)fp, bi = i / kXBlock;
    uint32_t cnt = 0;
    for (uint32_t bk = lane; bk < bi; bk += 64) {
      const uint32_t* xs = a.xs + (size_t)bk * kXBlock;
      uint32_t lo = 0, hi = a.xn[bk];                      // first sorted start > fp
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (xs[mid] <= fp32) lo = mid + 1; else hi = mid;
      }
      cnt += a.xn[bk] - lo;
    }
    for (uint32_t t = bi * kXBlock + lane; t < i; t += 64) {
      const uint64_t x = a.pst[t];
      cnt += x != kNoPair && x > fp;
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if (lane == 0) {
      const uint64_t window = (fe - fp) / 2 - 1;            // pushes strictly between (fp exact here)
      a.dec[i] = window - cnt < C ? 2 : 1;
    }
  }
}

// statuses (batch_check step 3, no cut: the host checked the caps) with lpos = exclusive scan of
// `last` (the first ceil(n / 1024) blocks), and the old entries' survival with spos = its
// exclusive scan (the other ceil(C / 1024) blocks): two look-back chains of their own
__global__ void __launch_bounds__(256) pd_status(PoolDevArgs a) {
  const uint32_t nt = (a.n + kTile - 1) / kTile;
  const bool old = blockIdx.x >= nt;
  const uint32_t tile = take_tile(a.tk + (old ? 2 : 1));
  if (tile >= (old ? (a.C + kTile - 1) / kTile : nt)) return;   // (tickets reset by pd_init: never)
  bool f[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = tile * kTile + 256u * k + threadIdx.x;
    f[k] = false;
    if (!old) {
      if (i >= a.n) continue;
      uint8_t st;
      if (i >= a.n_force && a.valid && a.valid[i - a.n_force] != a.valid_ok) st = TXV_POOL_NOT_CHECKED;
      else {
        const uint8_t d = a.dec[i];
        st = d == 0 ? TXV_POOL_ERR_TOO_LARGE : d == 2 ? TXV_POOL_ERR_IN_CACHE
           : (!a.sizes[i] && a.wal) ? TXV_POOL_ERR_ENCODING : TXV_POOL_OK;
      }
      a.status[i] = st;
      if (i >= a.n_force) {
        a.status_out[i - a.n_force] = st;                     // mapped host memory: no copy back
        if (a.status_copy) a.status_copy[i - a.n_force] = st;
      }
      f[k] = a.last[i] != 0;
    } else {
      if (i >= a.C) continue;
      f[k] = i < *a.clen && !a.detached[i];
      a.surv[i] = f[k];
    }
  }
  uint32_t r[4];
  tile_scan(f, r, old ? a.tiles + 2 * (size_t)nt : a.tiles + nt, tile, a.epoch, a.err, 1u);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = tile * kTile + 256u * k + threadIdx.x;
    if (!old && i < a.n) a.lpos[i] = r[k];
    if (old && i < a.C) a.spos[i] = r[k];
  }
  if (old || !a.list_on) return;   // (block-uniform) the pool list's appends: a third chain
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = tile * kTile + 256u * k + threadIdx.x;
    f[k] = i < a.n && i >= a.n_force && a.status[i] == TXV_POOL_OK;   // written by this thread above
  }
  tile_scan(f, r, a.tiles + 2 * (size_t)nt + (a.C + kTile - 1) / kTile, tile, a.epoch, a.err, 1u);
  // addTx (txvotepool.go:265-270), in arrival order: txs.PushBack at tail + rank (txsMap.Store
  // follows in pd_newcache, a launch of its own: a duplicate's key compare reads an entry another
  // block wrote, which only a launch boundary makes visible across XCDs without a fence per vote)
  const uint32_t tail = *a.l.tail_in;
  uint32_t hits = 0;
  uint64_t bytes = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = tile * kTile + 256u * k + threadIdx.x;
    if (i >= a.n) continue;
    a.okpos[i] = r[k];
    if (f[k]) {
      const uint32_t pos = tail + r[k];
      const uint4* src = reinterpret_cast<const uint4*>(a.keys + (size_t)i * 8);
      uint4* dst = reinterpret_cast<uint4*>(a.l.lk + (size_t)pos * 8);
      dst[0] = src[0];
      dst[1] = src[1];
      a.l.lsz[pos] = a.sizes[i];
      a.l.lfl[pos] = 1;
      ++hits;
      bytes += a.sizes[i];
    }
    if (i == a.n - 1) *a.l.tail_out = tail + r[k] + (f[k] ? 1u : 0u);
  }
  list_partial(a.res + 2 * tile, hits, bytes);
}

// txsMap.Store for appended vote i (its entry written by pd_status, an earlier launch)
__device__ __forceinline__ void list_index_vote(const PoolDevArgs& a, uint32_t i) {
  if (i < a.n_force || i >= a.n || a.status[i] != TXV_POOL_OK) return;
  const uint32_t pos = *a.l.tail_in + a.okpos[i];
  const uint4* src = reinterpret_cast<const uint4*>(a.keys + (size_t)i * 8);
  const uint4 k0 = src[0], k1 = src[1];
  const uint32_t k[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
  list_insert(a.l.li, a.l.imask, a.l.lk, pos, k, a.l.seed);
}

__device__ __forceinline__ void cache_put(const PoolDevArgs& a, uint32_t q, const uint4* s) {
  const uint4 x0 = s[0], x1 = s[1];
  uint4* d = reinterpret_cast<uint4*>(a.ck_new + (size_t)q * 8);
  d[0] = x0;
  d[1] = x1;
  const uint32_t k[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
  uint32_t h = idx_hash(k, a.seed) & (a.icap - 1);
  while (atomicCAS(&a.ci_new[h], 0u, q + 1u) != 0u) h = (h + 1) & (a.icap - 1);
}

// the new cache = the last keep_old surviving old entries in order, then the last keepU of the
// batch's U distinct pushed keys (each at its last push) in push order: the C most recent distinct
// keys of S (batch_check step 4), each indexed as it is written (the index was cleared by
// pd_init); the new length; detached[] cleared for the next batch; pd_init's ticket counter reset;
// and, with the pool list in HBM, txsMap.Store for the batch's appended votes
__global__ void __launch_bounds__(256) pd_newcache(PoolDevArgs a) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  const uint32_t U = a.n ? a.lpos[a.n - 1] + a.last[a.n - 1] : 0u;
  const uint32_t L1 = a.spos[a.C - 1] + a.surv[a.C - 1];
  const uint32_t keepU = U < a.C ? U : a.C;
  const uint32_t keep_old = L1 < a.C - keepU ? L1 : a.C - keepU;
  if (t < a.C && a.surv[t]) {
    const int64_t q = (int64_t)a.spos[t] - (int64_t)(L1 - keep_old);
    if (q >= 0) cache_put(a, (uint32_t)q, reinterpret_cast<const uint4*>(a.ck_old + (size_t)t * 8));
  }
  if (t < a.n && a.last[t]) {
    const int64_t u = (int64_t)a.lpos[t] - (int64_t)(U - keepU);
    if (u >= 0) cache_put(a, keep_old + (uint32_t)u, reinterpret_cast<const uint4*>(a.keys + (size_t)t * 8));
  }
  if (t < a.C) a.detached[t] = 0;   // (read by pd_link / pd_status: earlier launches)
  if (t == 0) {
    a.clen[0] = keep_old + keepU;
    a.tk[0] = 0;
    if (const uint32_t e = *a.err) *a.err_host = e;   // (the scans ran in earlier launches)
  }
  if (a.list_on) list_index_vote(a, t);
}

// nopTxCache: the list's index stores and pd_init's ticket counter reset
__global__ void __launch_bounds__(256) pd_finish_nocache(PoolDevArgs a) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t == 0) {
    a.tk[0] = 0;
    if (const uint32_t e = *a.err) *a.err_host = e;
  }
  if (a.list_on) list_index_vote(a, t);
}

// an index over keys [L][8] (a cache uploaded from the host)
__global__ void __launch_bounds__(256) pd_index_only(const uint32_t* ck, uint32_t L, uint32_t* ci, uint32_t icap,
                                                     uint64_t seed) {
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  if (q >= L) return;
  uint32_t s = idx_hash(ck + (size_t)q * 8, seed) & (icap - 1);
  while (atomicCAS(&ci[s], 0u, q + 1u) != 0u) s = (s + 1) & (icap - 1);
}

// compaction (the list's positions ran out): the live entries, in order, into the other buffer
// (npos = exclusive scan of the old alive flags over [0, ocap)); the new flags written over the
// whole new buffer; the new tail
__global__ void __launch_bounds__(256) pl_move(const uint32_t* lk, const uint32_t* lsz, const uint8_t* lfl,
                                               const uint32_t* npos, uint32_t ocap, uint32_t* nk, uint32_t* nsz,
                                               uint8_t* nfl, uint32_t ncap, uint32_t* tail_out) {
  const uint32_t o = blockIdx.x * 256 + threadIdx.x;
  const uint32_t live = npos[ocap - 1] + (lfl[ocap - 1] ? 1u : 0u);
  if (o < ocap && lfl[o]) {
    const uint32_t q = npos[o];
    const uint4* s = reinterpret_cast<const uint4*>(lk + (size_t)o * 8);
    uint4* d = reinterpret_cast<uint4*>(nk + (size_t)q * 8);
    d[0] = s[0];
    d[1] = s[1];
    nsz[q] = lsz[o];
  }
  if (o < ncap) nfl[o] = o < live ? 1 : 0;
  if (o == 0) *tail_out = live;
}
// the index over the moved entries: every indexed (non-tombstone) slot of the old index again at
// its entry's new position (tombstones dropped; no key is compared: the keys are distinct)
__global__ void __launch_bounds__(256) pl_reindex(const unsigned long long* oi, uint32_t oicap, const uint32_t* npos,
                                                  const uint32_t* nk, unsigned long long* ni, uint32_t nmask, uint64_t seed) {
  const uint32_t s = blockIdx.x * 256 + threadIdx.x;
  if (s >= oicap) return;
  const unsigned long long v = oi[s];
  if (v == 0 || (uint32_t)v == kListTomb) return;
  const uint32_t q = npos[(uint32_t)v - 1];
  const uint32_t* k = nk + (size_t)q * 8;
  uint32_t t = list_home(k, seed) & nmask;
  const unsigned long long mine = list_slot((uint32_t)(v >> 32), q + 1);
  while (atomicCAS(ni + t, 0ull, mine) != 0ull) t = (t + 1) & nmask;
}
// the index of a list uploaded from the host: the positions marked in ins (each key once)
__global__ void __launch_bounds__(256) pl_index_up(const uint32_t* lk, const uint8_t* ins, uint32_t L,
                                                   unsigned long long* li, uint32_t imask, uint64_t seed) {
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  if (q >= L || !ins[q]) return;
  const uint32_t* k = lk + (size_t)q * 8;
  uint32_t t = list_home(k, seed) & imask;
  const unsigned long long mine = list_slot(k[3], q + 1);
  while (atomicCAS(li + t, 0ull, mine) != 0ull) t = (t + 1) & imask;
}
struct AliveU32 {
  __host__ __device__ uint32_t operator()(uint8_t f) const { return f ? 1u : 0u; }
};

}  // namespace

// hipcub temporary storage for a batch of n votes and a cache of C entries (scans of n and C,
// the pair sort of n)
extern "C" size_t txv_pooldev_tmp_bytes(uint32_t n, uint32_t C) {
  size_t c = 0;
  uint32_t* u = nullptr;
  (void)C;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, c, u, u, u, u, (int)std::max<uint32_t>(n, 1));
  return c;
}

// a CheckTx batch's statuses as a TxFlow nil column (txv_submit_checked): the votes the pool did
// not admit never reach AddVote's state (types/vote_set.go:93)
__global__ void __launch_bounds__(256) txv_k_nil_from_status(const uint8_t* __restrict__ st, uint32_t n,
                                                             uint8_t* __restrict__ nil, uint32_t or_nil) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint8_t rej = st[i] != TXV_POOL_OK ? 1 : 0;
  nil[i] = or_nil ? (uint8_t)(nil[i] | rej) : rej;
}

extern "C" hipError_t txv_launch_nil_from_status(const uint8_t* st, uint32_t n, uint8_t* nil, uint32_t or_nil,
                                                 hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_nil_from_status, dim3((n + 255) / 256), dim3(256), 0, s, st, n, nil, or_nil);
  return hipGetLastError();
}

// the whole decision + cache update chain for one batch on stream st (a.n > 0; a.C > 0 or 0)
extern "C" hipError_t txv_pooldev_run(const PoolDevArgs* ap, hipStream_t st) {
  const PoolDevArgs& a = *ap;
  const uint32_t n = a.n;
  if (!n) return hipSuccess;
  const dim3 gn((n + 255) / 256), b(256);
  hipError_t e;
  size_t tb = a.tmp_bytes;
  const uint32_t nt = (n + kTile - 1) / kTile, ntc = (a.C + kTile - 1) / kTile;
  const uint32_t nrt = a.list_on ? (a.n_force + kTile - 1) / kTile : 0u;   // pd_init's removal tiles
  hipLaunchKernelGGL(pd_init, dim3(nt + nrt), b, 0, st, a);
  if ((e = hipcub::DeviceRadixSort::SortPairs(a.tmp, tb, a.hkey, a.skey, a.hidx, a.sidx, (int)n, 0, kSliceBits, st)))
    return e;
  hipLaunchKernelGGL(pd_link, gn, b, 0, st, a);
  // an Update batch (every vote pushes: max_tx = INT64_MAX) needs the new cache, not statuses:
  // its far pushes' decisions are skipped
  if (a.C && a.max_tx != INT64_MAX) {
    hipLaunchKernelGGL(pd_xsort, dim3((n + kXBlock - 1) / kXBlock), b, 0, st, a);
    hipLaunchKernelGGL(pd_far, dim3(std::min<uint32_t>(1024, (n + 3) / 4)), b, 0, st, a);
  }
  const uint32_t span = std::max(n, a.C);
  hipLaunchKernelGGL(pd_status, dim3(nt + ntc), b, 0, st, a);
  if (!a.C) hipLaunchKernelGGL(pd_finish_nocache, gn, b, 0, st, a);
  else hipLaunchKernelGGL(pd_newcache, dim3((span + 255) / 256), b, 0, st, a);
  return hipGetLastError();
}

// the index of a cache uploaded from the host (keys already at ck, its length at clen[0])
extern "C" hipError_t txv_pooldev_index(const uint32_t* ck, uint32_t L, uint32_t* ci, uint32_t icap, uint64_t seed,
                                        hipStream_t st) {
  hipError_t e;
  if ((e = hipMemsetAsync(ci, 0, (size_t)icap * 4, st))) return e;
  if (L) hipLaunchKernelGGL(pd_index_only, dim3((L + 255) / 256), dim3(256), 0, st, ck, L, ci, icap, seed);
  return hipGetLastError();
}

// hipcub temporary storage of the compaction's scan over cap positions
extern "C" size_t txv_poollist_tmp_bytes(uint32_t cap) {
  size_t c = 0;
  uint32_t* u = nullptr;
  hipcub::TransformInputIterator<uint32_t, AliveU32, const uint8_t*> it(nullptr, AliveU32());
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, it, u, (int)std::max<uint32_t>(cap, 1));
  return c;
}

// the compaction: old buffer (ocap positions, index oicap slots) -> new buffer (ncap, nicap);
// npos [ocap] scratch, tmp hipcub storage
extern "C" hipError_t txv_poollist_compact(const uint32_t* lk, const uint32_t* lsz, const uint8_t* lfl,
                                           const unsigned long long* li, uint32_t ocap, uint32_t oicap, uint32_t* nk,
                                           uint32_t* nsz, uint8_t* nfl, unsigned long long* ni, uint32_t ncap,
                                           uint32_t nicap, uint32_t* npos, void* tmp, size_t tmp_bytes,
                                           uint32_t* tail_out, uint64_t seed, hipStream_t st) {
  hipError_t e;
  hipcub::TransformInputIterator<uint32_t, AliveU32, const uint8_t*> it(lfl, AliveU32());
  if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, it, npos, (int)ocap, st))) return e;
  const uint32_t span = std::max(ocap, ncap);
  hipLaunchKernelGGL(pl_move, dim3((span + 255) / 256), dim3(256), 0, st, lk, lsz, lfl, npos, ocap, nk, nsz, nfl, ncap,
                     tail_out);
  if ((e = hipMemsetAsync(ni, 0, (size_t)nicap * 8, st))) return e;
  hipLaunchKernelGGL(pl_reindex, dim3((oicap + 255) / 256), dim3(256), 0, st, li, oicap, npos, nk, ni, nicap - 1, seed);
  return hipGetLastError();
}

// a list of L entries uploaded from the host (keys / sizes at lk / lsz): flags, index
extern "C" hipError_t txv_poollist_upload_index(const uint32_t* lk, const uint8_t* ins, uint32_t L,
                                                unsigned long long* li, uint32_t icap, uint64_t seed, hipStream_t st) {
  hipError_t e;
  if ((e = hipMemsetAsync(li, 0, (size_t)icap * 8, st))) return e;
  if (L) hipLaunchKernelGGL(pl_index_up, dim3((L + 255) / 256), dim3(256), 0, st, lk, ins, L, li, icap - 1, seed);
  return hipGetLastError();
}
