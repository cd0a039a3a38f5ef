// route.h — the layout of one rank's ingest-route buffer (include/txvote.h txv_route_admitted),
// shared by the device packer (kernels_route.hip), the host packer and view (runtime.cpp) and the
// receiving rank's staging (txv_submit_routed), so every side agrees on every byte.
//
// [header: 8 x u64] then, each at a 16-byte aligned offset:
//   height i64[n], ts_sec i64[n], ts_nanos i32[n], txhash_off u32[n], txhash_len u32[n],
//   addr_len u32[n], sig_len u32[n], addr u8[20 n], sig u8[64 n], txkey u8[32 n] (TXV_ROUTE_TXKEY),
//   is_nil u8[n] (TXV_ROUTE_NIL), TxHash arena u8[arena_bytes] + 16 zero bytes (the device reads
//   keys 8 bytes at a time)
// header words: magic, n, arena_bytes, flags, max_txhash_len, total bytes, 0, 0
#pragma once
#include <stdint.h>

#include "../../include/txvote.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define TXV_ROUTE_HD __host__ __device__ __forceinline__
#else
#define TXV_ROUTE_HD inline
#endif

namespace txv_route {

constexpr uint64_t kMagic = 0x3130525654585654ull;   // "TVXTVR01"
enum Col { kHeight, kSec, kNanos, kOff, kLen, kAddrLen, kSigLen, kAddr, kSig, kTxKey, kNil, kArena, kNCols };
constexpr uint32_t kFlagTxKey = 0x1u, kFlagNil = 0x2u;   // = TXV_ROUTE_TXKEY / TXV_ROUTE_NIL

TXV_ROUTE_HD uint64_t align16(uint64_t x) { return (x + 15) & ~15ull; }

// column offsets of a buffer holding n votes and arena_bytes of TxHash; returns the total size
TXV_ROUTE_HD uint64_t layout(uint64_t n, uint64_t arena_bytes, uint32_t flags, uint64_t off[kNCols]) {
  const uint64_t w[kNCols] = {8, 8, 4, 4, 4, 4, 4, 20, 64, (flags & kFlagTxKey) ? 32u : 0u, (flags & kFlagNil) ? 1u : 0u, 0};
  uint64_t o = 64;
  for (int c = 0; c < kArena; ++c) {
    off[c] = o;
    o = align16(o + w[c] * n);
  }
  off[kArena] = o;
  return align16(o + arena_bytes + 16);
}

}  // namespace txv_route

// arguments of the three route launches (kernels_route.hip txv_launch_route)
struct RouteArgs {
  uint32_t n, G, nw;                 // votes, shards, waves (ceil(n / 64))
  const int64_t* height;
  const int64_t* ts_sec;
  const int32_t* ts_nanos;
  const uint32_t* th_off;
  const uint32_t* th_len;
  const uint8_t* th;                 // TxHash arena
  const uint8_t* addr;               // [n][20]
  const uint32_t* addr_len;
  const uint8_t* sig;                // [n][64]
  const uint32_t* sig_len;
  const uint8_t* txkey;              // [n][32] or null
  const uint8_t* nil;                // [n] or null
  const uint8_t* status;             // [n] pool statuses, or null: every vote admitted
  uint32_t flags;                    // txv_route flags of the output (txkey / nil columns present)
  uint8_t* shard;                    // [n] scratch: the vote's shard, 0xFF = not admitted
  uint32_t* wcnt;                    // [nw][G] per-wave counts, then their exclusive scan
  uint32_t* wbytes;                  // [nw][G] per-wave TxHash bytes, then their exclusive scan
  uint32_t* maxhl;                   // [G] longest TxHash per shard (zeroed before count)
  uint64_t* tot;                     // [G][2] votes, arena bytes per shard
  uint8_t* dst;                      // rank r's buffer at dst + r * stride
  uint64_t stride;
  txv_route_meta* meta;              // [G] mapped host memory
};

#if defined(__HIPCC__)
extern "C" hipError_t txv_launch_route(const RouteArgs* a, hipStream_t st);
#endif
