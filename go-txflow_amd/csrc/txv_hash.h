// txv_hash.h — the seeded 64-bit byte-string hash of the TxHash -> TxVoteSet table, shared by
// the device (kernels_flow.hip) and the host (reader lookups, host_pack.hpp's AddrTable), so
// both sides place a key in the same slot.  Only the table's probe length depends on it: every
// hit is confirmed by comparing the full key bytes.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define TXV_HASH_HD __host__ __device__ __forceinline__
#else
#define TXV_HASH_HD inline
#endif

namespace txv_hash {

TXV_HASH_HD uint64_t mix64(uint64_t x) {
  x ^= x >> 32; x *= 0xd6e8feb86659fd93ULL; x ^= x >> 32; x *= 0xd6e8feb86659fd93ULL; x ^= x >> 32;
  return x;
}

// hash of n bytes whose little-endian 8-byte chunk at byte i (i % 8 == 0) is get(i); bytes
// of the last chunk beyond n are masked off here
template <class Get>
TXV_HASH_HD uint64_t hash_chunks(uint32_t n, uint64_t seed, Get get) {
  uint64_t h = seed ^ (0x9e3779b97f4a7c15ULL * (uint64_t)(n + 1));
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8) h = mix64(h ^ get(i)) + 0x9e3779b97f4a7c15ULL;
  if (i < n) {
    const uint64_t t = get(i) & ((1ull << (8 * (n - i))) - 1ull);
    h = mix64(h ^ t ^ ((uint64_t)(n - i) << 56));
  }
  return mix64(h) | 1ull;   // never 0
}

// seeded hash of a 32-byte TxVotePool key (SHA-256(Signature), as 8 words in memory order).  The
// keys are peer-chosen (a peer can grind signatures until their keys share any fixed slice), so
// every table or sort over them places a key by this hash under a secret per-process / per-engine
// seed: the four 64-bit words folded (rotated apart, so a key differing in any byte folds apart)
// and one mix64, a bijection of the fold xor the seed.  Two keys land together for every seed only
// if their folds are equal -- 64 bits of SHA-256 output to match: pairs cost ~2^32 hashes, but k
// keys with one fold ~2^(64 (k-1) / k) (runs of ten: 2^57), so a run or a probe cluster stays a
// handful of keys whatever a peer grinds -- and the single mix keeps the host CheckTx loop at its
// unseeded speed (five mixes over the words made it 3-5x slower).
TXV_HASH_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
TXV_HASH_HD uint64_t key32(const uint32_t* k, uint64_t seed) {
  const uint64_t w0 = (uint64_t)k[0] | ((uint64_t)k[1] << 32), w1 = (uint64_t)k[2] | ((uint64_t)k[3] << 32);
  const uint64_t w2 = (uint64_t)k[4] | ((uint64_t)k[5] << 32), w3 = (uint64_t)k[6] | ((uint64_t)k[7] << 32);
  return mix64(w0 ^ rotl64(w1, 16) ^ rotl64(w2, 32) ^ rotl64(w3, 48) ^ seed);
}

}  // namespace txv_hash
