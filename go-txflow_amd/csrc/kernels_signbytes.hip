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
// The host keeps only what is order- or error-dependent: the length (which also decides the
// amino time-range error, TXV_FLAG_BADMSG) is computed in its parallel phase A; the bytes are
// produced here, one lane per vote, from the raw fields and the caller's TxHash arena, as
// big-endian 64-bit words msg[w][n_pad] (zero beyond the length, so K1a needs no masking).
// H2D per vote drops from ~148 B of message words to 28 B of fields (+ the shared TxHash arena).
#include "txv_device.h"

namespace {

// streaming big-endian word writer over one lane's column
struct WordSink {
  uint64_t* col;      // &msg[0][i]
  uint32_t stride;    // n_pad
  uint64_t acc = 0;
  uint32_t fill = 0;  // bytes in acc
  uint32_t word = 0;  // next word index
  __device__ void put(uint32_t b) {
    acc = (acc << 8) | (b & 0xFFu);
    if (++fill == 8) {
      col[(size_t)word * stride] = acc;
      ++word; acc = 0; fill = 0;
    }
  }
  __device__ void uvarint(uint64_t v) {
    while (v >= 0x80u) { put((uint32_t)(v | 0x80u)); v >>= 7; }
    put((uint32_t)v);
  }
  __device__ void finish(uint32_t words) {
    if (fill) {
      col[(size_t)word * stride] = acc << (8 * (8 - fill));
      ++word;
    }
    for (; word < words; ++word) col[(size_t)word * stride] = 0;
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
  const uint32_t len = i < a.n ? a.msg_len[i] : 0u;
  if (len) {
    const int64_t height = a.height[i];
    const int64_t sec = a.ts_sec[i];
    const int32_t nanos = a.ts_nanos[i];
    const uint32_t hl = a.txhash_len[i];
    const uint8_t* th = a.txhash + a.txhash_off[i];
    const uint32_t tl = (sec != 0 ? 1u + uvarint_len((uint64_t)sec) : 0u) +
                        (nanos != 0 ? 1u + uvarint_len((uint64_t)(uint32_t)nanos) : 0u);
    const uint32_t body = (height != 0 ? 9u : 0u) + (hl ? 1u + uvarint_len(hl) + hl : 0u) + 34u +
                          (tl ? 1u + uvarint_len(tl) + tl : 0u) +
                          (a.chain_len ? 1u + uvarint_len(a.chain_len) + a.chain_len : 0u);
    w.uvarint(body);
    if (height != 0) {
      w.put(0x09);
      for (int b = 0; b < 8; ++b) w.put((uint32_t)((uint64_t)height >> (8 * b)));
    }
    if (hl) {
      w.put(0x12);
      w.uvarint(hl);
      for (uint32_t b = 0; b < hl; ++b) w.put(th[b]);
    }
    w.put(0x1a); w.put(0x20);
    for (int b = 0; b < 32; ++b) w.put(0);
    if (tl) {
      w.put(0x22);
      w.uvarint(tl);
      if (sec != 0) { w.put(0x08); w.uvarint((uint64_t)sec); }
      if (nanos != 0) { w.put(0x10); w.uvarint((uint64_t)(uint32_t)nanos); }
    }
    if (a.chain_len) {
      w.put(0x2a);
      w.uvarint(a.chain_len);
      for (uint32_t b = 0; b < a.chain_len; ++b) w.put(a.chain[b]);
    }
  }
  w.finish(a.msg_words);
}

extern "C" hipError_t txv_launch_signbytes(const SignBytesArgs* args, hipStream_t st) {
  if (!args->n_pad) return hipSuccess;
  hipLaunchKernelGGL(txv_k_signbytes, dim3((args->n_pad + 255) / 256), dim3(256), 0, st, *args);
  return hipGetLastError();
}
