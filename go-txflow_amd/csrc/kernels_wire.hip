// kernels_wire.hip — Reactor.Receive's decodeMsg on the GPU: amino
// UnmarshalBinaryBare of TxVoteMessage wire bytes (txvotepool/reactor.go:170-190, 273-291) straight
// into the txv_votes column layout, one lane per message.
//
// The rules are go-amino v0.15.1 (external) as restated in oracle/wire.c's header: interface
// prefix (4 bytes) or disfix (0x00 + 3 + 4 bytes), TxVoteMessage{Tx} bare, TxVote's six fields in
// order with absent-field defaults, strictly increasing extra fields skipped by typ3, Go
// binary.Uvarint overflow rules, the time body's partial consumption and the nested-struct advance
// of UvarintSize(len) + consumed.
//
// Memory: a 256-message block stages the byte span its messages cover into LDS with 16-byte
// coalesced loads (56 KB: ~280 bytes per message on average), then every lane parses its message
// from LDS: the parse is a chain of dependent byte reads (keys, varints), which LDS serves at a
// fraction of the L2 latency.  Blocks whose span does not fit (long messages) parse from global
// memory.  The 32-byte TxKey, 20-byte address and 64-byte signature are copied into their output
// rows dword by dword with alignbit (unaligned source), zero beyond the field length; TxHash bytes
// and long signatures are not copied: the outputs carry their offsets into the wire buffer.
#include "txv_device.h"
#include "wire_dev.h"

using namespace txv::wire;

namespace {

constexpr uint32_t kWireBlock = 256;
constexpr uint32_t kWireLds = 56 * 1024;

}  // namespace

__global__ void __launch_bounds__(kWireBlock) txv_k_decode_msgs(WireArgs a) {
  __shared__ uint32_t lds_w[kWireLds / 4 + 4];
  __shared__ unsigned long long span_lo, span_hi;
  const uint32_t i = blockIdx.x * kWireBlock + threadIdx.x;
  const bool live = i < a.n;
  const uint64_t off = live ? a.off[i] : 0;
  const uint32_t len = live ? a.len[i] : 0;
  const bool parse = live && len > 0 && len <= a.max_msg_bytes;
  if (threadIdx.x == 0) { span_lo = ~0ull; span_hi = 0; }
  __syncthreads();
  if (parse) {
    atomicMin(&span_lo, (unsigned long long)off);
    atomicMax(&span_hi, (unsigned long long)(off + len));
  }
  __syncthreads();
  const uint64_t lo = span_lo & ~15ull, hi = span_hi;
  const bool staged = hi > lo && hi - lo <= kWireLds;
  if (staged) {   // 16-byte coalesced loads of [lo, hi rounded up); the device buffer is padded
    const uint32_t nvec = (uint32_t)((hi - lo + 15) >> 4);
    const uint4* src = reinterpret_cast<const uint4*>(a.wire + lo);
    uint4* dst = reinterpret_cast<uint4*>(lds_w);
    for (uint32_t v = threadIdx.x; v < nvec; v += kWireBlock) dst[v] = src[v];
  }
  __syncthreads();
  if (!live) return;

  Parsed o{};
  uint32_t st = 1;   // TXV_WIRE_TOO_LARGE
  if (len == 0) st = 3;
  else if (parse) {
    if (staged) {
      const uint8_t* b = reinterpret_cast<const uint8_t*>(lds_w) + (uint32_t)(off - lo);
      st = parse_msg(b, len, a.disamb, a.prefix, o);
    } else {
      st = parse_msg(a.wire + off, len, a.disamb, a.prefix, o);
    }
  }
  if (st != 0) o = Parsed{};

  uint32_t key[8], addr[5], sig[16];
  const uint32_t sig_n = o.sig_len < 64 ? o.sig_len : 64u, addr_n = o.addr_len < 20 ? o.addr_len : 20u;
  if (staged) {
    const uint32_t base = (uint32_t)(off - lo);
    copy_row<8>(lds_w, base + o.key_off, o.has_key ? 32u : 0u, key);
    copy_row<5>(lds_w, base + o.addr_off, addr_n, addr);
    copy_row<16>(lds_w, base + o.sig_off, sig_n, sig);
  } else {
    const uint32_t* gw = reinterpret_cast<const uint32_t*>(a.wire);
    const uint64_t base = off;
    // global rows: re-base the word pointer at the message's aligned start
    const uint32_t* mw = gw + (base >> 2);
    const uint32_t b3 = (uint32_t)(base & 3u);
    copy_row<8>(mw, b3 + o.key_off, o.has_key ? 32u : 0u, key);
    copy_row<5>(mw, b3 + o.addr_off, addr_n, addr);
    copy_row<16>(mw, b3 + o.sig_off, sig_n, sig);
  }
  a.status[i] = (uint8_t)st;
  a.height[i] = o.height;
  a.ts_sec[i] = o.sec;
  a.ts_nanos[i] = o.nanos;
  const uint32_t moff = (uint32_t)off;   // wire_bytes < 2^32 (host check)
  a.txhash_off[i] = st == 0 ? moff + o.th_off : 0u;
  a.txhash_len[i] = o.th_len;
  a.addr_len[i] = o.addr_len;
  a.sig_off[i] = st == 0 ? moff + o.sig_off : 0u;
  a.sig_len[i] = o.sig_len;
#pragma unroll
  for (int j = 0; j < 8; ++j) a.txkey[(size_t)i * 8 + j] = key[j];
#pragma unroll
  for (int j = 0; j < 5; ++j) a.addr[(size_t)i * 5 + j] = addr[j];
#pragma unroll
  for (int j = 0; j < 16; ++j) a.sig[(size_t)i * 16 + j] = sig[j];
}

extern "C" hipError_t txv_launch_decode_msgs(const WireArgs* a, hipStream_t st) {
  if (!a->n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_decode_msgs, dim3((a->n + kWireBlock - 1) / kWireBlock), dim3(kWireBlock), 0, st, *a);
  return hipGetLastError();
}
