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
#include "amino.hpp"
#include "sha2.h"
#include "txv_device.h"
#include "wire_dev.h"
#include "../../include/txvote.h"

using namespace txv::wire;

namespace {

constexpr uint32_t kWireBlock = TXV_WIRE_BLOCK;        // messages per chunk = threads per block
constexpr uint32_t kWireLds = kWireBlock * 224;        // staged bytes per chunk
constexpr uint32_t kPer = (kWireLds / 16 + kWireBlock - 1) / kWireBlock;   // 16-byte loads per lane
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // native vector: stays in VGPRs

// the next chunk's inputs, loaded one iteration ahead (registers = the second stage buffer)
struct Prefetch {
  u32x4 r[kPer];
  uint64_t off, lo;
  uint32_t len, nvec;
  bool staged;
};

// compile-time indices (template recursion, not a loop) so the register array is never demoted
// to scratch while it is live across the chunk loop
template <uint32_t K>
__device__ __forceinline__ void load_vecs(u32x4 (&r)[kPer], const u32x4* src, uint32_t nv) {
  const uint32_t v = threadIdx.x + K * kWireBlock;
  r[K] = __builtin_nontemporal_load(src + (v < nv ? v : nv - 1));   // streamed once: bypass-friendly
  if constexpr (K + 1 < kPer) load_vecs<K + 1>(r, src, nv);
}
template <uint32_t K>
__device__ __forceinline__ void store_vecs(const u32x4 (&r)[kPer], u32x4* dst, uint32_t nv) {
  const uint32_t v = threadIdx.x + K * kWireBlock;
  if (v < nv) dst[v] = r[K];
  if constexpr (K + 1 < kPer) store_vecs<K + 1>(r, dst, nv);
}

__device__ __forceinline__ void prefetch(const WireArgs& a, uint32_t c, Prefetch& p) {
  const uint64_t lo = a.span[2 * c], hi = a.span[2 * c + 1];   // host: [16-aligned lo, hi) of the chunk
  p.lo = lo;
  p.staged = hi > lo && hi - lo <= kWireLds;
  p.nvec = p.staged ? (uint32_t)((hi - lo + 15) >> 4) : 0u;
  const uint32_t i = c * kWireBlock + threadIdx.x;
  p.off = i < a.n ? a.off[i] : 0;
  p.len = i < a.n ? a.len[i] : 0;
  // unconditional (clamped) loads: all of a lane's loads in flight together, p.r stays in VGPRs
  const u32x4* src = reinterpret_cast<const u32x4*>(a.wire + (p.staged ? lo : 0));
  load_vecs<0>(p.r, src, p.nvec ? p.nvec : 1u);
}

}  // namespace

// Persistent blocks walk chunks c = blockIdx.x, + gridDim.x, ...: the loads of chunk c + gridDim.x
// are issued before chunk c is parsed, so HBM reads overlap the parse and the record stores.
__global__ void __launch_bounds__(kWireBlock) __attribute__((amdgpu_waves_per_eu(1, 3))) txv_k_decode_msgs(WireArgs a) {
  __shared__ uint32_t lds_w[kWireLds / 4 + 24];   // + slack for the row / window reads
  Prefetch p;
  prefetch(a, blockIdx.x, p);   // grid <= n_chunks
  for (uint32_t c = blockIdx.x; c < a.n_chunks; c += gridDim.x) {
    const uint32_t i = c * kWireBlock + threadIdx.x;
    const bool live = i < a.n;
    const uint64_t off = p.off, lo = p.lo;
    const uint32_t len = p.len;
    const bool staged = p.staged;
    __syncthreads();                                 // the previous chunk's records are out of LDS
    if (staged) store_vecs<0>(p.r, reinterpret_cast<u32x4*>(lds_w), p.nvec);
    __syncthreads();
    // next chunk (the last iteration re-loads the final chunk: unconditional keeps p in registers)
    prefetch(a, c + gridDim.x < a.n_chunks ? c + gridDim.x : a.n_chunks - 1, p);

    const bool parse = live && len > 0 && len <= a.max_msg_bytes;
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

    // rows: only fields that exist are read (reads run up to 4 * (W + 1) bytes past a field's
    // aligned start: LDS slack / 128 bytes of padding behind the wire buffer)
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
    // one 160-byte record per message, transposed through LDS so the block writes its records as
    // one contiguous stream of 16-byte stores
    constexpr uint32_t R = TXV_WIRE_REC_WORDS + 1;   // odd stride: conflict-free record writes
    static_assert(kWireBlock * R <= kWireLds / 4, "record stage does not fit the LDS buffer");
    __syncthreads();                                  // every lane is done reading the staged chunk
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
    const uint32_t i0 = c * kWireBlock;
    const uint32_t nb = a.n - i0 < kWireBlock ? a.n - i0 : kWireBlock;   // messages of this chunk
    constexpr uint32_t C = TXV_WIRE_REC_WORDS / 4;                        // 16-byte chunks per record
    u32x4* dst = reinterpret_cast<u32x4*>(a.rec + (size_t)i0 * TXV_WIRE_REC_WORDS);
    for (uint32_t q = threadIdx.x; q < nb * C; q += kWireBlock) {
      const uint32_t* r = lds_w + (q / C) * R + 4 * (q % C);
      const u32x4 val = {r[0], r[1], r[2], r[3]};
      __builtin_nontemporal_store(val, dst + q);   // written once, read by the host copy
    }
  }
}

// ------------------------------------------------------------------ device-resident ingest
// (txv_ingest_msgs: Reactor.Receive -> TxVotePool.CheckTxWithInfo -> TxFlow.TryAddVote without
// the decoded records leaving HBM)

// (txv::sha256_bytes, sha2.h: the wire buffer is padded behind its last message)

// Per decoded message (records of txv_k_decode_msgs): its wire status, and for the decoded ones
// txVoteKey = SHA-256(Signature) (txvotepool/txvotepool.go:467-469: the first 64 bytes come from
// the record, longer signatures are hashed from the wire buffer) and TxVote.Size()
// (types/tx_vote.go:144-150: 0 when amino rejects the time) -- everything the pool's
// order-dependent admission needs; the longest TxHash goes to max_hl (SignBytes column bound).
__global__ void __launch_bounds__(256) txv_k_rec_keys(const uint32_t* __restrict__ rec, const uint8_t* __restrict__ wire,
                                                      uint32_t n, uint8_t* __restrict__ status,
                                                      uint32_t* __restrict__ keys, uint32_t* __restrict__ sizes,
                                                      uint32_t* max_hl) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t* r = rec + (size_t)i * TXV_WIRE_REC_WORDS;
  const uint32_t stt = r[0];
  status[i] = (uint8_t)stt;
  if (stt != 0) return;
  const int64_t height = (int64_t)((uint64_t)r[1] | ((uint64_t)r[2] << 32));
  const int64_t sec = (int64_t)((uint64_t)r[3] | ((uint64_t)r[4] << 32));
  const uint32_t hl = r[7], al = r[8], sl = r[10];
  sizes[i] = (uint32_t)txv_host::txvote_size(height, hl, sec, (int32_t)r[5], al, sl);
  if (hl) atomicMax(max_hl, hl);
  uint32_t st[8];
  if (sl <= 64) {   // the record's signature words (little-endian, zero beyond sig_len)
    uint32_t w[16];
    txv::sha256_init(st);
    const uint32_t nblk = sl <= 55 ? 1u : 2u;
    for (uint32_t b = 0; b < nblk; ++b) {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const uint32_t gw = 16u * b + (uint32_t)t;
        uint32_t v = gw < 16 ? txv::bswap32(r[24 + gw]) : 0u;
        if (gw == sl / 4) v |= 0x80000000u >> (8 * (sl & 3));
        if (gw == 16u * nblk - 1u) v = sl * 8u;
        w[t] = v;
      }
      txv::sha256_block(st, w);
    }
  } else {
    txv::sha256_bytes(wire + r[9], sl, st);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) keys[(size_t)i * 8 + j] = txv::bswap32(st[j]);
}

// The admitted messages (pool OK, arrival order) -> the flow slot's raw TxVote columns, the
// layout txv_add_votes uploads (txv_flow.h FlowBatch): the TxHash offsets stay offsets into the
// wire buffer, which is the batch's TxHash arena.
__global__ void __launch_bounds__(256) txv_k_rec_to_flow(const uint32_t* __restrict__ rec,
                                                         const uint32_t* __restrict__ list, uint32_t n, FlowCols c) {
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const uint32_t* r = rec + (size_t)list[j] * TXV_WIRE_REC_WORDS;
  c.height[j] = (int64_t)((uint64_t)r[1] | ((uint64_t)r[2] << 32));
  c.ts_sec[j] = (int64_t)((uint64_t)r[3] | ((uint64_t)r[4] << 32));
  c.ts_nanos[j] = (int32_t)r[5];
  c.th_off[j] = r[6];
  c.th_len[j] = r[7];
  c.addr_len[j] = r[8];
  c.sig_len[j] = r[10];
  uint32_t* a = reinterpret_cast<uint32_t*>(c.addr + (size_t)j * 20);
#pragma unroll
  for (int q = 0; q < 5; ++q) a[q] = r[19 + q];
  uint4* sg = reinterpret_cast<uint4*>(c.sig + (size_t)j * 64);
#pragma unroll
  for (int q = 0; q < 4; ++q) sg[q] = make_uint4(r[24 + 4 * q], r[25 + 4 * q], r[26 + 4 * q], r[27 + 4 * q]);
  uint4* tk = reinterpret_cast<uint4*>(c.txkey + (size_t)j * 32);
  tk[0] = make_uint4(r[11], r[12], r[13], r[14]);
  tk[1] = make_uint4(r[15], r[16], r[17], r[18]);
}

// Every decoded message -> the flow slot's columns, the pool's rejections (and the messages that
// did not decode: TXV_POOL_NOT_CHECKED) as nil entries, which AddVote drops before any state
// (types/vote_set.go:93): the TxFlow chain of a wire batch is enqueued behind the pool's device
// decisions without their statuses making a host round trip first.
__global__ void __launch_bounds__(256) txv_k_rec_to_flow_nil(const uint32_t* __restrict__ rec,
                                                             const uint8_t* __restrict__ pool_status, uint32_t n,
                                                             FlowCols c, uint8_t* __restrict__ nil) {
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const uint32_t* r = rec + (size_t)j * TXV_WIRE_REC_WORDS;
  const bool ok = pool_status[j] == TXV_POOL_OK;
  nil[j] = ok ? 0 : 1;
  c.height[j] = ok ? (int64_t)((uint64_t)r[1] | ((uint64_t)r[2] << 32)) : 0;
  c.ts_sec[j] = ok ? (int64_t)((uint64_t)r[3] | ((uint64_t)r[4] << 32)) : 0;
  c.ts_nanos[j] = ok ? (int32_t)r[5] : 0;
  c.th_off[j] = ok ? r[6] : 0u;
  c.th_len[j] = ok ? r[7] : 0u;
  c.addr_len[j] = ok ? r[8] : 0u;
  c.sig_len[j] = ok ? r[10] : 0u;
  if (!ok) return;
  uint32_t* a = reinterpret_cast<uint32_t*>(c.addr + (size_t)j * 20);
#pragma unroll
  for (int q = 0; q < 5; ++q) a[q] = r[19 + q];
  uint4* sg = reinterpret_cast<uint4*>(c.sig + (size_t)j * 64);
#pragma unroll
  for (int q = 0; q < 4; ++q) sg[q] = make_uint4(r[24 + 4 * q], r[25 + 4 * q], r[26 + 4 * q], r[27 + 4 * q]);
  uint4* tk = reinterpret_cast<uint4*>(c.txkey + (size_t)j * 32);
  tk[0] = make_uint4(r[11], r[12], r[13], r[14]);
  tk[1] = make_uint4(r[15], r[16], r[17], r[18]);
}

extern "C" hipError_t txv_launch_rec_to_flow_nil(const uint32_t* rec, const uint8_t* pool_status, uint32_t n,
                                                 const FlowCols* c, uint8_t* nil, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_rec_to_flow_nil, dim3((n + 255) / 256), dim3(256), 0, st, rec, pool_status, n, *c, nil);
  return hipGetLastError();
}

extern "C" hipError_t txv_launch_rec_keys(const uint32_t* rec, const uint8_t* wire, uint32_t n, uint8_t* status,
                                          uint32_t* keys, uint32_t* sizes, uint32_t* max_hl, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_rec_keys, dim3((n + 255) / 256), dim3(256), 0, st, rec, wire, n, status, keys, sizes, max_hl);
  return hipGetLastError();
}

extern "C" hipError_t txv_launch_rec_to_flow(const uint32_t* rec, const uint32_t* list, uint32_t n, const FlowCols* c,
                                             hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_rec_to_flow, dim3((n + 255) / 256), dim3(256), 0, st, rec, list, n, *c);
  return hipGetLastError();
}

extern "C" hipError_t txv_launch_decode_msgs(const WireArgs* a, uint32_t grid, hipStream_t st) {
  if (!a->n) return hipSuccess;
  if (grid > a->n_chunks) grid = a->n_chunks;
  hipLaunchKernelGGL(txv_k_decode_msgs, dim3(grid), dim3(kWireBlock), 0, st, *a);
  return hipGetLastError();
}
