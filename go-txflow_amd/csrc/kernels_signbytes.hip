// kernels_signbytes.hip — TxVote.SignBytes built on the GPU, straight into
// the column-major SHA-512 message layout K1a reads.
//
//   SignBytes = cdc.MarshalBinaryLengthPrefixed(CanonicalizeTxVote(chainID, vote))
//   (types/tx_vote.go:83-89, CanonicalTxVote :177-183, CanonicalizeTxVote :185-192; go-amino
//   v0.15.1-0.20190603130624-25d5598ed22b, external; byte layout SURVEY.md Appendix B):
//     uvarint(len(body)) || body,  body =
//       [0x09 Height as 8 LE bytes]                       (omitted when Height == 0)
//       [0x12 uvarint(len) TxHash]                        (omitted when empty)
//        0x1a 0x20 + 32 zero bytes                        (TxKey: never copied by CanonicalizeTxVote)
//       [0x22 uvarint(len) [0x08 uvarint(sec)] [0x10 uvarint(nanos)]]   (omitted at the Unix epoch)
//       [0x2a uvarint(len) ChainID]                       (omitted when empty)
//
// The length (which also decides the amino time-range error, TXV_FLAG_BADMSG) comes from the
// route kernel (kernels_flow.hip) or the signer's host pass; the bytes are produced here, one
// lane per vote, from the raw fields and the TxHash arena, as big-endian 64-bit words
// msg[w][n_pad] (zero beyond the length, so K1a needs no masking), 8 bytes per append step.
#include "txv_device.h"

namespace {

// little-endian 8 bytes at any byte address (reads up to 12 bytes from p rounded down to 4;
// the TxHash arena and the chain id carry >= 16 bytes of padding)
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t s = (uint32_t)(a & 3u);
  const uint32_t w0 = q[0], w1 = q[1], w2 = q[2];
  return ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, s) << 32) | __builtin_amdgcn_alignbyte(w1, w0, s);
}

// Streaming big-endian word writer over one lane's column, appending up to 8 bytes per step:
// acc holds the `fill` (< 8) pending bytes right-aligned, a full word goes out as soon as it
// completes.  Byte strings are appended 8 bytes at a time (one unaligned load + bswap).
struct WordSink {
  uint64_t* col;      // &msg[0][i]
  uint32_t stride;    // n_pad
  uint64_t acc = 0;
  uint32_t fill = 0;
  uint32_t word = 0;
  __device__ __forceinline__ void emit(uint64_t w) {
    col[(size_t)word * stride] = w;
    ++word;
  }
  // k (1..8) bytes, right-aligned big-endian in be (the first byte most significant)
  __device__ __forceinline__ void put(uint64_t be, uint32_t k) {
    const uint32_t total = fill + k;
    if (total < 8) {
      acc = (acc << (8 * k)) | be;
      fill = total;
      return;
    }
    const uint32_t rest = total - 8;
    emit((fill ? acc << (8 * (8 - fill)) : 0ull) | (be >> (8 * rest)));
    acc = rest ? be & ((1ull << (8 * rest)) - 1ull) : 0ull;
    fill = rest;
  }
  __device__ __forceinline__ void uvarint(uint64_t v) {
    uint64_t be = 0;
    uint32_t k = 0;
    while (v >= 0x80u) {
      be = (be << 8) | ((v & 0x7Fu) | 0x80u);
      v >>= 7;
      if (++k == 8) { put(be, 8); be = 0; k = 0; }
    }
    put((be << 8) | v, k + 1);
  }
  __device__ __forceinline__ void bytes(const uint8_t* p, uint32_t n) {
    for (uint32_t k = 0; k < n; k += 8) {
      const uint32_t m = n - k < 8 ? n - k : 8;
      put(__builtin_bswap64(ld64u(p + k)) >> (8 * (8 - m)), m);
    }
  }
  __device__ __forceinline__ void finish(uint32_t words) {
    if (fill) emit(acc << (8 * (8 - fill)));
    for (; word < words;) emit(0);
  }
};

__device__ __forceinline__ uint32_t uvarint_len(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80u) { v >>= 7; ++n; }
  return n;
}

}  // namespace

__global__ void __launch_bounds__(256) txv_k_signbytes(SignBytesArgs a) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n_pad) return;
  WordSink w{a.msg + i, a.n_pad};
  // with no length column (the TxFlow path, beside the route kernel) every non-nil vote is
  // encoded; K1a reads the words only for votes the route kernel left pending
  const uint32_t len = i >= a.n ? 0u : (a.msg_len ? a.msg_len[i] : (a.nil && a.nil[i] ? 0u : 1u));
  if (len) {
    const int64_t height = a.height[i];
    const int64_t sec = a.ts_sec[i];
    const int32_t nanos = a.ts_nanos[i];
    const uint32_t hl = a.txhash_len[i];
    const uint32_t tl = (sec != 0 ? 1u + uvarint_len((uint64_t)sec) : 0u) +
                        (nanos != 0 ? 1u + uvarint_len((uint64_t)(uint32_t)nanos) : 0u);
    const uint32_t body = (height != 0 ? 9u : 0u) + (hl ? 1u + uvarint_len(hl) + hl : 0u) + 34u +
                          (tl ? 1u + uvarint_len(tl) + tl : 0u) +
                          (a.chain_len ? 1u + uvarint_len(a.chain_len) + a.chain_len : 0u);
    w.uvarint(body);
    if (height != 0) {
      w.put(0x09, 1);
      w.put(__builtin_bswap64((uint64_t)height), 8);
    }
    if (hl) {
      w.put(0x12, 1);
      w.uvarint(hl);
      w.bytes(a.txhash + a.txhash_off[i], hl);
    }
    w.put(0x1a20, 2);                        // TxKey: never copied by CanonicalizeTxVote
    w.put(0, 8); w.put(0, 8); w.put(0, 8); w.put(0, 8);
    if (tl) {
      w.put(0x22, 1);
      w.uvarint(tl);
      if (sec != 0) { w.put(0x08, 1); w.uvarint((uint64_t)sec); }
      if (nanos != 0) { w.put(0x10, 1); w.uvarint((uint64_t)(uint32_t)nanos); }
    }
    if (a.chain_len) {
      w.put(0x2a, 1);
      w.uvarint(a.chain_len);
      w.bytes(a.chain, a.chain_len);
    }
  }
  w.finish(a.msg_words);
}

extern "C" hipError_t txv_launch_signbytes(const SignBytesArgs* args, hipStream_t st) {
  if (!args->n_pad) return hipSuccess;
  hipLaunchKernelGGL(txv_k_signbytes, dim3((args->n_pad + 255) / 256), dim3(256), 0, st, *args);
  return hipGetLastError();
}
