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

#ifndef TXV_WIRE_BLOCK
#define TXV_WIRE_BLOCK 128
#endif
constexpr uint32_t kWireBlock = TXV_WIRE_BLOCK;        // messages per block
constexpr uint32_t kWireLds = kWireBlock * 224;        // staged bytes per block

}  // namespace

__global__ void __launch_bounds__(kWireBlock) txv_k_decode_msgs(WireArgs a) {
  __shared__ uint32_t lds_w[kWireLds / 4 + 24];   // + slack for the row reads
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
  if (staged) {   // 16-byte coalesced loads of [lo, hi rounded up); the device buffer is padded.
    // All of a lane's loads are issued before the first LDS store so they are in flight together.
    const uint32_t nvec = (uint32_t)((hi - lo + 15) >> 4);
    const uint4* src = reinterpret_cast<const uint4*>(a.wire + lo);
    uint4* dst = reinterpret_cast<uint4*>(lds_w);
    constexpr uint32_t kPer = (kWireLds / 16 + kWireBlock - 1) / kWireBlock;
    uint4 r[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      const uint32_t v = threadIdx.x + k * kWireBlock;
      r[k] = src[v < nvec ? v : nvec - 1];   // clamped: unconditional, all in flight
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      const uint32_t v = threadIdx.x + k * kWireBlock;
      if (v < nvec) dst[v] = r[k];
    }
  }
  __syncthreads();

  Parsed o{};
  uint32_t st = 1;   // TXV_WIRE_TOO_LARGE
  if (len == 0) st = 3;
  else if (parse) {
    // canonical layout: branch-free fast path; everything else: the general parser
#ifdef TXV_WIRE_NOPARSE   // experiment: memory structure only
    const bool fast = true;
    o.sig_len = 64; o.sig_off = (uint32_t)(off & 7u); o.addr_len = 20; o.has_key = true;
#else
    const bool fast = staged ? fast_msg(lds_w, (uint32_t)(off - lo), len, a.prefix, o)
                             : fast_msg(reinterpret_cast<const uint32_t*>(a.wire) + (off >> 2), (uint32_t)(off & 3u),
                                        len, a.prefix, o);
#endif
    if (fast) {
      st = 0;
    } else {
      o = Parsed{};
      if (staged) {
        const uint8_t* b = reinterpret_cast<const uint8_t*>(lds_w) + (uint32_t)(off - lo);
        st = parse_msg(b, len, a.disamb, a.prefix, o);
      } else {
        st = parse_msg(a.wire + off, len, a.disamb, a.prefix, o);
      }
    }
  }
  if (st != 0) o = Parsed{};

  // rows: only fields that exist are read (reads run up to 4 * (W + 1) bytes past a field's aligned
  // start: LDS slack / 128 bytes of padding behind the wire buffer)
  uint32_t key[8] = {}, addr[5] = {}, sig[16] = {};
  const uint32_t sig_n = o.sig_len < 64 ? o.sig_len : 64u, addr_n = o.addr_len < 20 ? o.addr_len : 20u;
  if (st == 0) {
    if (staged) {
      const uint32_t base = (uint32_t)(off - lo);
      if (o.has_key) copy_row<8>(lds_w, base + o.key_off, 32u, key);
      if (addr_n) copy_row<5>(lds_w, base + o.addr_off, addr_n, addr);
      if (sig_n) copy_row<16>(lds_w, base + o.sig_off, sig_n, sig);
    } else {   // word pointer re-based at the message's aligned start
      const uint32_t* mw = reinterpret_cast<const uint32_t*>(a.wire) + (off >> 2);
      const uint32_t b3 = (uint32_t)(off & 3u);
      if (o.has_key) copy_row<8>(mw, b3 + o.key_off, 32u, key);
      if (addr_n) copy_row<5>(mw, b3 + o.addr_off, addr_n, addr);
      if (sig_n) copy_row<16>(mw, b3 + o.sig_off, sig_n, sig);
    }
  }
  // one 160-byte record per message, transposed through LDS so the block writes its records as one
  // contiguous stream of 16-byte stores (instead of one word per lane per 32/20/64-byte row)
  constexpr uint32_t R = TXV_WIRE_REC_WORDS + 1;   // odd stride: conflict-free record writes
  static_assert(kWireBlock * R <= kWireLds / 4, "record stage does not fit the LDS buffer");
  __syncthreads();                                  // every lane is done reading the staged messages
  uint32_t* row = lds_w + threadIdx.x * R;
  const uint32_t moff = (uint32_t)off;              // wire_bytes < 2^32 (host check)
  row[0] = st;
  row[1] = (uint32_t)(uint64_t)o.height; row[2] = (uint32_t)((uint64_t)o.height >> 32);
  row[3] = (uint32_t)(uint64_t)o.sec; row[4] = (uint32_t)((uint64_t)o.sec >> 32);
  row[5] = (uint32_t)o.nanos;
  row[6] = st == 0 ? moff + o.th_off : 0u;
  row[7] = o.th_len;
  row[8] = o.addr_len;
  row[9] = st == 0 ? moff + o.sig_off : 0u;
  row[10] = o.sig_len;
#pragma unroll
  for (int j = 0; j < 8; ++j) row[11 + j] = key[j];
#pragma unroll
  for (int j = 0; j < 5; ++j) row[19 + j] = addr[j];
#pragma unroll
  for (int j = 0; j < 16; ++j) row[24 + j] = sig[j];
  __syncthreads();
  const uint32_t i0 = blockIdx.x * kWireBlock;
  const uint32_t nb = a.n - i0 < kWireBlock ? a.n - i0 : kWireBlock;   // messages of this block
  constexpr uint32_t C = TXV_WIRE_REC_WORDS / 4;                        // 16-byte chunks per record
  uint4* dst = reinterpret_cast<uint4*>(a.rec + (size_t)i0 * TXV_WIRE_REC_WORDS);
  for (uint32_t c = threadIdx.x; c < nb * C; c += kWireBlock) {
    const uint32_t* r = lds_w + (c / C) * R + 4 * (c % C);
    dst[c] = make_uint4(r[0], r[1], r[2], r[3]);
  }
}

extern "C" hipError_t txv_launch_decode_msgs(const WireArgs* a, hipStream_t st) {
  if (!a->n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_decode_msgs, dim3((a->n + kWireBlock - 1) / kWireBlock), dim3(kWireBlock), 0, st, *a);
  return hipGetLastError();
}
