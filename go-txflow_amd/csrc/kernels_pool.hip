// kernels_pool.hip — TxVotePool ingest on the GPU: txVoteKey(tx) = SHA-256(tx.Signature)
// (txvotepool/txvotepool.go:467-469), the key of the pool's LRU cache (mapTxCache.Push,
// :416-438) and of txsMap, for a whole batch.  One lane per vote; signatures of up to 64 bytes
// (every well-formed vote) are hashed here, longer ones on the host (they are rejected by
// Verify anyway but still occupy pool/cache entries, so their keys must be exact).
#include "sha2.h"
#include "txv_device.h"

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
