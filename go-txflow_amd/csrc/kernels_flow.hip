// kernels_flow.hip — TxFlow.addVote for a whole batch on the GPU, from the caller's raw
// TxVote columns to per-vote (added, err) codes, stake sums and commit events.
//
// Reference semantics (Fantom-foundation/go-txflow), per vote in
// arrival order:
//   txflow/service.go:200-209   TxVoteSets[vote.TxHash] created on first sight (any non-nil vote)
//   types/vote_set.go:93-106    nil -> ErrVoteNil; empty address; unknown validator
//                               (ValidatorSet.GetByAddress, tendermint, external)
//   types/vote_set.go:109-114   the set already holds an accepted vote of the validator: same
//                               signature bytes -> (false, nil), else ErrVoteNonDeterministicSignature
//                               -- decided BEFORE verification
//   types/vote_set.go:117-119   Verify fails -> ErrVoteInvalidSignature (not stored)
//   types/vote_set.go:143-166   ADDED: votes[addr] = vote, sum += power, maj23 |= sum >= quorum
//   txflow/service.go:215-216   commit side effects on every ADDED vote of a set with maj23
//
// The batch form (one launch chain per batch, everything keyed on the device):
//   prep     one lane per vote (verify stream): validator lookup (address hash table),
//            pre-checks, SignBytes length / amino time check, signature transpose into the
//            column-major layout the verify kernels read
//   key      one lane per vote (flow stream): find-or-insert of the TxHash into the set table;
//            a key seen for the first time records the smallest arrival index that carries it
//   new ids  a stream compaction over the arrival order of "first occurrence of a new key"
//            numbers the new sets exactly as the sequential loop would (first-seen order)
//   set ids  every vote reads its set id; the (set, validator) cells of pending votes are
//            cleared for the resolution below
//   (SignBytes + K1a/K1b verify run here, kernels_signbytes.hip / kernels_verify.hip)
//   min      every verified pending vote posts its arrival index to its cell (atomic min):
//            the cell then holds the FIRST verified vote of the (set, validator) group
//   resolve  each pending vote decides its code from its cell: earlier accepted vote ->
//            signature compare; first verified == itself -> ADDED (an arena row is taken by a
//            wave-aggregated atomic and written right there); first verified earlier ->
//            signature compare with it; none -> invalid signature
//   cross    one wave per set the batch ADDED votes to (the work list resolve compacted): its
//            ADDED votes are the stamped cells of its row; stake sum, and the arrival index at
//            which the prefix (in arrival order) of the stake first reaches quorum (a digit-by-
//            digit histogram search over the arrival index: LDS atomics, a DPP wave scan and a
//            ballot per 6 bits); the cells' accepted rows
//   out      final statuses (pre-check or tally; an ADDED vote at or after its set's crossing
//            fires) into mapped host memory, and the per-block counts of commit events
//   events   compaction of the crossing votes in arrival order -> commit events + batch summary
#include <algorithm>

#include "sha2.h"
#include "txv_device.h"
#include "txv_flow.h"
#include "lookback.h"

namespace {

constexpr int64_t kAminoMinSec = -62135596800LL;   // 0001-01-01T00:00:00Z
constexpr int64_t kAminoMaxSec = 253402300800LL;   // 10000-01-01T00:00:00Z (exclusive)
constexpr uint64_t kAddrSeed = 0x61646472ULL;      // host_pack.hpp AddrTable
constexpr uint32_t kScanItems = 1024;              // items per scan block (256 threads x 4)

// little-endian 4 / 8 bytes at any byte address (reads up to 12 bytes from p rounded down to 4)
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t s = (uint32_t)(a & 3u);
  const uint32_t w0 = q[0], w1 = q[1], w2 = q[2];
  return ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, s) << 32) | __builtin_amdgcn_alignbyte(w1, w0, s);
}

__device__ __forceinline__ bool key_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8)
    if (ld64u(a + i) != ld64u(b + i)) return false;
  if (i < n) {
    const uint64_t m = (1ull << (8 * (n - i))) - 1ull;
    if ((ld64u(a + i) ^ ld64u(b + i)) & m) return false;
  }
  return true;
}

// A key of at most 64 bytes in registers: 16 little-endian words (zero beyond the length),
// fetched with <= 5 16-byte loads from p rounded down to 16 (the arenas carry >= 16 bytes of
// padding) and realigned with v_alignbyte -- instead of 3 dword loads per 8 bytes
constexpr uint32_t kKeyRegBytes = 64;
struct KeyRegs {
  uint32_t w[16];
};
__device__ __forceinline__ void load_key(const uint8_t* p, uint32_t n, KeyRegs& k) {
  const uintptr_t a = (uintptr_t)p;
  const uint4* q = reinterpret_cast<const uint4*>(a & ~(uintptr_t)15);
  const uint32_t s = (uint32_t)(a & 15u);
  uint32_t raw[20];
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    const uint4 v = (16u * c < s + n) ? q[c] : make_uint4(0, 0, 0, 0);
    raw[4 * c] = v.x; raw[4 * c + 1] = v.y; raw[4 * c + 2] = v.z; raw[4 * c + 3] = v.w;
  }
  const uint32_t sb = s & 3u;
  // realign by whole words with a static copy per case (a computed index into raw[] would put
  // it in scratch), then by bytes with v_alignbyte
  uint32_t t[17];
  switch (s >> 2) {
#define TXV_SHIFT_CASE(W) \
    case W: { _Pragma("unroll") for (int j = 0; j < 17; ++j) t[j] = raw[j + W]; } break;
    TXV_SHIFT_CASE(0)
    TXV_SHIFT_CASE(1)
    TXV_SHIFT_CASE(2)
    default: { _Pragma("unroll") for (int j = 0; j < 16; ++j) t[j] = raw[j + 3]; t[16] = raw[19]; } break;
#undef TXV_SHIFT_CASE
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t x = __builtin_amdgcn_alignbyte(t[j + 1], t[j], sb);
    const int valid = (int)n - 4 * j;
    if (valid <= 0) x = 0;
    else if (valid < 4) x &= 0xFFFFFFFFu >> (8 * (4 - valid));
    k.w[j] = x;
  }
}
__device__ __forceinline__ uint64_t key_chunk(const KeyRegs& k, uint32_t i) {   // i % 8 == 0, i < 64
  uint64_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if ((uint32_t)j == i / 8) r = (uint64_t)k.w[2 * j] | ((uint64_t)k.w[2 * j + 1] << 32);
  return r;
}
// txv_hash::hash_chunks over the key in registers (bit-identical: the words beyond n are zero)
__device__ __forceinline__ uint64_t hash_regs(const KeyRegs& k, uint32_t n, uint64_t seed) {
  uint64_t h = seed ^ (0x9e3779b97f4a7c15ULL * (uint64_t)(n + 1));
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t i = 8u * j;
    const uint64_t c = (uint64_t)k.w[2 * j] | ((uint64_t)k.w[2 * j + 1] << 32);
    if (i + 8 <= n) h = txv_hash::mix64(h ^ c) + 0x9e3779b97f4a7c15ULL;
    else if (i < n) h = txv_hash::mix64(h ^ c ^ ((uint64_t)(n - i) << 56));
  }
  return txv_hash::mix64(h) | 1ull;
}

__device__ __forceinline__ bool key_eq_regs(const KeyRegs& a, const uint8_t* p, uint32_t n) {
  KeyRegs b;
  load_key(p, n, b);
  uint32_t d = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) d |= a.w[j] ^ b.w[j];
  return d == 0;
}

__device__ __forceinline__ uint32_t uvlen(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80u) { v >>= 7; ++n; }
  return n;
}

// len(SignBytes(chainID)) (types/tx_vote.go:83-89; layout kernels_signbytes.hip), or -1 when
// amino rejects the timestamp (out of [0001, 10000) years, or nanos out of range)
__device__ __forceinline__ int signbytes_len(int64_t height, uint32_t hl, int64_t sec, int32_t nanos, uint32_t cl) {
  if (sec != 0 && (sec < kAminoMinSec || sec >= kAminoMaxSec)) return -1;
  if (nanos != 0 && (nanos < 0 || nanos > 999999999)) return -1;
  const uint32_t tl = (sec != 0 ? 1u + uvlen((uint64_t)sec) : 0u) + (nanos != 0 ? 1u + uvlen((uint64_t)(uint32_t)nanos) : 0u);
  const uint32_t body = (height != 0 ? 9u : 0u) + (hl ? 1u + uvlen(hl) + hl : 0u) + 34u +
                        (tl ? 1u + uvlen(tl) + tl : 0u) + (cl ? 1u + uvlen(cl) + cl : 0u);
  return (int)(uvlen(body) + body);
}

// agent-coherent (sc1) 64-bit loads / stores of table words: the table is the one structure
// written and read inside the same launch, by lanes on different XCDs (private L2s)
__device__ __forceinline__ uint64_t ld_sc1(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t* w64(SetEntry* e, int k) { return reinterpret_cast<uint64_t*>(e) + k; }

// Find-or-insert of one TxHash (linear probing).  A lane that claims an empty slot (CAS on the
// state word) writes the entry's words through to the coherent level (sc1), waits for them
// (s_waitcnt vmcnt(0)) and only then publishes the state.  Probing: a plain (cached) copy of
// the entry is trusted for one conclusion only -- "this is my key" -- and only when it shows a
// published entry (state set, key pointer set: key_off is stored + 1, so a copy fetched before
// the entry was written reads 0) whose hash, length and key bytes all equal mine.  Every other
// conclusion (empty -> claim, different key -> next slot) is drawn from sc1 loads of the coherent
// copy: a stale or torn cached copy can then cost one extra coherent read, never a duplicate
// entry.  A lane that meets a slot being written re-reads it in its next iteration: the writer
// finished inside the iteration in which it claimed the slot, whether it is in the same wave or
// not, so no lane waits on a lane that waits on it.
template <bool kRegs>
__device__ __forceinline__ bool key_matches(const uint8_t* stored, const uint8_t* kp, const KeyRegs& kr, uint32_t len) {
  if constexpr (kRegs) return key_eq_regs(kr, stored, len);
  else return key_eq(stored, kp, len);
}

#ifndef TXV_ROUTE_SLEEP
#define TXV_ROUTE_SLEEP 2
#endif
#if TXV_ROUTE_SLEEP
#define TXV_ROUTE_BACKOFF() __builtin_amdgcn_s_sleep(TXV_ROUTE_SLEEP)
#else
#define TXV_ROUTE_BACKOFF() ((void)0)
#endif

// kRegs: the key is in registers (keys of <= 64 bytes), else compared from memory
template <bool kRegs>
__device__ __forceinline__ uint32_t set_find_or_insert(const FlowState& fs, const FlowBatch& b, uint64_t h,
                                                       const uint8_t* kp, const KeyRegs& kr, uint32_t len,
                                                       uint64_t key_off, uint32_t i) {
  uint32_t slot = (uint32_t)h & fs.tab_mask;
  uint32_t probes = 0;
  for (;;) {
    SetEntry* e = fs.tab + slot;
    {
      // optimistic cached read: accept a match, decide nothing else
      const uint4 lo = *reinterpret_cast<const uint4*>(e);        // h, (state, len)
      const uint4 hi = *(reinterpret_cast<const uint4*>(e) + 1);  // key_off + 1, (first, id)
      const uint32_t st = lo.z;
      const uint64_t ek = (uint64_t)hi.x | ((uint64_t)hi.y << 32);
      if ((st == TXV_SE_BATCH || st == TXV_SE_KEPT) && ek != 0 && lo.w == len &&
          ((uint64_t)lo.x | ((uint64_t)lo.y << 32)) == h &&
          key_matches<kRegs>((st == TXV_SE_BATCH ? b.th : fs.keys) + (ek - 1), kp, kr, len)) {
        if (st == TXV_SE_BATCH && hi.z > i) atomicMin(&e->first, i);   // a stale first: one extra min
        return slot;
      }
    }
    const uint64_t sl = ld_sc1(w64(e, 1));                     // (state, len), coherent
    const uint32_t st = (uint32_t)sl;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");     // keep the loads below after it
    if (st == TXV_SE_EMPTY) {
      if (atomicCAS(&e->state, TXV_SE_EMPTY, TXV_SE_BUSY) == TXV_SE_EMPTY) {
        st_sc1(w64(e, 0), h);
        st_sc1(w64(e, 2), key_off + 1);
        st_sc1(w64(e, 3), (uint64_t)i | ((uint64_t)TXV_NONE << 32));   // first = i, id = none
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                 // entry words landed
        st_sc1(w64(e, 1), (uint64_t)TXV_SE_BATCH | ((uint64_t)len << 32));
        return slot;
      }
      // lost the claim: re-read the slot in the next iteration
      TXV_ROUTE_BACKOFF();
    } else if (st == TXV_SE_BUSY) {
      // another lane is writing this entry: give the SIMD's issue slots to it (and to K1b,
      // which this kernel runs beside) instead of re-reading at once
      TXV_ROUTE_BACKOFF();
    } else {
      if ((uint32_t)(sl >> 32) == len && ld_sc1(w64(e, 0)) == h &&
          key_matches<kRegs>((st == TXV_SE_BATCH ? b.th : fs.keys) + (ld_sc1(w64(e, 2)) - 1), kp, kr, len)) {
        if (st == TXV_SE_BATCH && (uint32_t)ld_sc1(w64(e, 3)) > i) atomicMin(&e->first, i);
        return slot;
      }
      slot = (slot + 1) & fs.tab_mask;
      if (++probes > fs.tab_mask) {
        atomicOr(&fs.ctr->err, TXV_FERR_TABLE);
        return TXV_NONE;
      }
    }
  }
}

// ValidatorSet.GetByAddress (tendermint, external; called at types/vote_set.go:102) over the
// registry's address table: the 20 address bytes as 5 little-endian words
__device__ __forceinline__ uint32_t find_validator(const FlowState& fs, const uint32_t a[5]) {
  if (!fs.addr_slots) return TXV_NONE;
  const uint64_t c0 = (uint64_t)a[0] | ((uint64_t)a[1] << 32), c1 = (uint64_t)a[2] | ((uint64_t)a[3] << 32);
  const uint64_t h = txv_hash::hash_chunks(20, kAddrSeed, [&](uint32_t k) -> uint64_t {
    return k == 0 ? c0 : (k == 8 ? c1 : (uint64_t)a[4]);
  });
  for (uint32_t s = (uint32_t)h & fs.addr_mask;; s = (s + 1) & fs.addr_mask) {
    const uint32_t v = fs.addr_slots[s];
    if (v == TXV_NONE) return TXV_NONE;
    const uint32_t* r = fs.val_addr + (size_t)v * 5;
    if (((r[0] ^ a[0]) | (r[1] ^ a[1]) | (r[2] ^ a[2]) | (r[3] ^ a[3]) | (r[4] ^ a[4])) == 0) return v;
  }
}

// ------------------------------------------------------------------ route
// Two kernels, so that the verify kernels never wait for the TxFlow state:
//   prep  (verify stream) everything a vote's verification needs and nothing keyed by the
//         TxFlow: signature transpose, nil / empty-address / unknown-validator pre-checks,
//         validator lookup, SignBytes length and amino time check
//   key   (flow stream, in batch order after the previous batch's tally) TxHash find-or-insert
//         into the set table
__global__ void __launch_bounds__(256) txv_k_route_prep(FlowState fs, FlowBatch b) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= b.n) return;
  b.ev_flag[i] = 0;
  b.mark[i] = 0;
  // signature: [n][64] bytes -> [16][n_pad] words, zero beyond min(len, 64)
  {
    const uint32_t sl = b.sig_len[i];
    const uint4* src = reinterpret_cast<const uint4*>(b.sig_raw + (size_t)i * 64);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = src[q];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t byte0 = 16u * q + 4u * j;
        uint32_t x = w[j];
        if (sl <= byte0) x = 0;
        else if (sl < byte0 + 4) x &= 0xFFFFFFFFu >> (8 * (byte0 + 4 - sl));
        b.sig[(size_t)(4 * q + j) * b.n_pad + i] = x;
      }
    }
  }
  if (b.nil && b.nil[i]) {   // nil *TxVote: AddVote's first check
    b.pre[i] = TXV_S_NIL; b.flags[i] = 0; b.msg_len[i] = 0; b.val[i] = 0;
    return;
  }
  // AddVote pre-checks (types/vote_set.go:93-106)
  uint32_t v = TXV_NONE;
  uint8_t pre = TXV_S_PENDING;
  const uint32_t al = b.vcode ? 0u : b.addr_len[i];
  if (b.vcode) {                             // looked up on the host (txv_submit_votes staging)
    const uint32_t code = b.vcode[i];
    if (code == TXV_VCODE_EMPTY) pre = TXV_S_EMPTY_ADDR;
    else if (code == TXV_VCODE_UNKNOWN) pre = TXV_S_UNKNOWN_VALIDATOR;
    else v = code;
  } else if (al == 0) {
    pre = TXV_S_EMPTY_ADDR;
  } else if (al == 20) {
    const uint32_t* ap = reinterpret_cast<const uint32_t*>(b.addr + (size_t)i * 20);
    const uint32_t a[5] = {ap[0], ap[1], ap[2], ap[3], ap[4]};
    v = find_validator(fs, a);
    if (v == TXV_NONE) pre = TXV_S_UNKNOWN_VALIDATOR;
  } else {
    pre = TXV_S_UNKNOWN_VALIDATOR;
  }
  const int L = signbytes_len(b.height[i], b.th_len[i], b.ts_sec[i], b.ts_nanos[i], b.chain_len);
  b.pre[i] = pre;
  b.val[i] = v == TXV_NONE ? 0u : v;
  b.msg_len[i] = (pre == TXV_S_PENDING && L > 0) ? (uint32_t)L : 0u;
  b.flags[i] = pre != TXV_S_PENDING ? 0
               : (uint8_t)(TXV_FLAG_PENDING | (b.sig_len[i] == 64 ? TXV_FLAG_SIG64 : 0) | (L < 0 ? TXV_FLAG_BADMSG : 0));
}

// TxVoteSets[vote.TxHash], created on first sight for every non-nil vote (txflow/service.go:200-209).
// TXV_ROUTE_KEY_REGS=0 compares keys from memory (36 instead of 86 VGPRs), so that two route
// waves fit beside K1b's on a SIMD; measured slower (573-604 vs 605-615M votes/s): the
// co-resident waves cost K1b more than the route gains, so the key stays in registers
#ifndef TXV_ROUTE_KEY_REGS
#define TXV_ROUTE_KEY_REGS 1
#endif
__global__ void __launch_bounds__(256) txv_k_route_key(FlowState fs, FlowBatch b) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= b.n) return;
  if (b.nil && b.nil[i]) {
    b.entry[i] = TXV_NONE;
    return;
  }
  const uint32_t len = b.th_len[i];
  const uint32_t off = b.th_off[i];
  const uint8_t* kp = b.th + off;
  KeyRegs kr;
  if (TXV_ROUTE_KEY_REGS && len <= kKeyRegBytes) {
    load_key(kp, len, kr);
    b.entry[i] = set_find_or_insert<true>(fs, b, hash_regs(kr, len, fs.hash_seed), kp, kr, len, off, i);
  } else {
    const uint64_t h = txv_hash::hash_chunks(len, fs.hash_seed, [&](uint32_t k) { return ld64u(kp + k); });
    b.entry[i] = set_find_or_insert<false>(fs, b, h, kp, kr, len, off, i);
  }
}

// ------------------------------------------------------------------ block scan helpers
// exclusive scan of c over the 256 threads of a block; *total = block sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t c, uint32_t* total) {
  __shared__ uint32_t wsum[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < w) before += wsum[k];
    all += wsum[k];
  }
  __syncthreads();
  *total = all;
  return before + x - c;
}

// A scan block covers items b*1024 + k*256 + t (round k < 4, thread t): consecutive lanes hold
// consecutive items, so the predicate's and the action's column accesses coalesce per wave.
template <class Pred>
__global__ void __launch_bounds__(256) txv_k_scan_count(Pred p, uint32_t n, uint32_t* blk) {
  const uint32_t base = blockIdx.x * kScanItems + threadIdx.x;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) c += (base + 256u * k < n && p(base + 256u * k)) ? 1u : 0u;
  uint32_t total;
  (void)block_excl_scan(c, &total);
  if (threadIdx.x == 0) blk[blockIdx.x] = total;
}

// exclusive offsets of nb block counts (nb <= 8192), blk[nb] = total.  One 256-thread block
// (4 waves): it runs beside K1b of the next batch, whose waves leave room for one wave per SIMD
// but not for the 16 waves of a 1024-thread block (which then waited for K1b to drain).
__global__ void __launch_bounds__(256) txv_k_scan_top(uint32_t* blk, uint32_t nb) {
  const uint32_t t = threadIdx.x;
  const uint32_t per = (nb + 255) / 256;          // consecutive counts per thread (<= 32)
  const uint32_t lo = min(t * per, nb), hi = min(lo + per, nb);
  uint32_t s = 0;
  for (uint32_t j = lo; j < hi; ++j) s += blk[j];
  uint32_t total;
  uint32_t run = block_excl_scan(s, &total);
  for (uint32_t j = lo; j < hi; ++j) {
    const uint32_t v = blk[j];
    blk[j] = run;
    run += v;
  }
  if (t == 0) blk[nb] = total;
}

template <class Pred, class Act>
__global__ void __launch_bounds__(256) txv_k_scan_apply(Pred p, Act act, uint32_t n, const uint32_t* blk) {
  __shared__ uint32_t cnt[4][4];     // [round][wave] flagged items
  const uint32_t base = blockIdx.x * kScanItems + threadIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  bool f[4];
  uint64_t m[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[k] = base + 256u * k < n && p(base + 256u * k);
    m[k] = __ballot(f[k]);
    if (lane == 0) cnt[k][w] = (uint32_t)__popcll(m[k]);
  }
  __syncthreads();
  uint32_t rank = blk[blockIdx.x];
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t before = 0, round = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      before += q < w ? cnt[k][q] : 0u;
      round += cnt[k][q];
    }
    if (f[k]) act(base + 256u * k, rank + before + (uint32_t)__popcll(m[k] & below));
    rank += round;
  }
}

// ------------------------------------------------------------------ new set ids
struct NewSetPred {
  FlowState fs;
  FlowBatch b;
  __device__ bool operator()(uint32_t i) const {
    const uint32_t e = b.entry[i];
    if (e == TXV_NONE) return false;
    const SetEntry& s = fs.tab[e];
    return s.state == TXV_SE_BATCH && s.first == i;
  }
};

// the vote that first carried a new TxHash: number its set (first-seen order), move the key
// bytes into the set's key slot (or the overflow arena), record the set's TxKey
// (service.go:201-207); its exchange name comes later, from the pack's digest pass
struct NewSetAct {
  FlowState fs;
  FlowBatch b;
  __device__ void operator()(uint32_t i, uint32_t rank) const {
    const uint32_t slot = b.entry[i];
    SetEntry& e = fs.tab[slot];
    const uint32_t id = fs.ctr->n_sets + rank;
    e.state = TXV_SE_KEPT;
    if (id >= fs.max_txs) {
      atomicOr(&fs.ctr->err, TXV_FERR_SETS);
      e.id = TXV_NONE;
      return;
    }
    const uint32_t len = e.len, span = (len + 7u) & ~7u;
    uint64_t ko = (uint64_t)id * TXV_KEY_SLOT;
    if (len > TXV_KEY_SLOT) {
      const unsigned long long o = atomicAdd((unsigned long long*)&fs.ctr->key_used, (unsigned long long)span);
      if (o + span + 16 > fs.keys_cap) {
        atomicOr(&fs.ctr->err, TXV_FERR_KEYS);
        e.id = TXV_NONE;
        return;
      }
      ko = (uint64_t)fs.max_txs * TXV_KEY_SLOT + o;
    }
    const uint8_t* src = b.th + (e.key_off - 1);
    uint64_t* dst = reinterpret_cast<uint64_t*>(fs.keys + ko);
    for (uint32_t k = 0; k < span; k += 8)
      dst[k / 8] = ld64u(src + k) & (k + 8 <= len ? ~0ull : ((1ull << (8 * (len - k))) - 1ull));
    e.key_off = ko + 1;
    e.id = id;
    fs.set_entry[id] = slot;
    uint32_t* tk = fs.set_txkey + (size_t)id * 8;
    if (b.txkey) {
      const uint4* s4 = reinterpret_cast<const uint4*>(b.txkey + (size_t)i * 32);
      const uint4 a = s4[0], c = s4[1];
      tk[0] = a.x; tk[1] = a.y; tk[2] = a.z; tk[3] = a.w; tk[4] = c.x; tk[5] = c.y; tk[6] = c.z; tk[7] = c.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) tk[j] = 0;
    }
  }
};

// ------------------------------------------------------------------ tally
__device__ __forceinline__ uint64_t cand_key(uint32_t stamp, uint32_t i) {
  return ((uint64_t)(0xFFFFFFFFu - stamp) << 32) | i;
}
// the cell's first verified vote of this batch, or TXV_NONE (stale stamp = an earlier batch's)
__device__ __forceinline__ uint32_t cand_of(uint64_t c, uint32_t stamp) {
  return (uint32_t)(c >> 32) == 0xFFFFFFFFu - stamp ? (uint32_t)c : TXV_NONE;
}

// every vote's set id (after the new-id step); each verified pending vote posts its arrival
// index to its (set, validator) cell: the cell then holds the FIRST verified vote of the group
// (cells that already hold an accepted vote skip: their votes are decided without verification).
// The atomic's old value tells each vote whether it can be ADDED without tally_resolve reading
// the cell again: status[i] (scratch until resolve) = 1 when the cell must be read (accepted
// earlier, not verified, or a smaller arrival index was already there), and a vote that takes
// the cell from a larger index k marks k.  A vote with status 0 and no mark is its cell's first
// verified vote: ADDED.  With shuffled arrival order every cell access is a random 128-byte line
// (profiles/r03/tally_calib), so resolve's re-read was a line per vote.
constexpr uint8_t kReadCell = 1;
__global__ void __launch_bounds__(256) txv_k_tally_min(FlowState fs, FlowBatch b, uint32_t nb) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i == 0) {
    const uint32_t created = b.blk[nb];
    const uint32_t ns = fs.ctr->n_sets + created;
    fs.ctr->n_sets = ns > fs.max_txs ? fs.max_txs : ns;
    fs.ctr->n_stamped = 0;
    fs.ctr->ev_ticket = 0;
  }
  if (i >= b.n) return;
  const uint32_t e = b.entry[i];
  const uint32_t s = e == TXV_NONE ? TXV_NONE : fs.tab[e].id;
  b.set[i] = s;
  if (s == TXV_NONE || b.pre[i] != TXV_S_PENDING) return;
  if (b.ok[i] != 1) { b.status[i] = kReadCell; return; }
  TallyCell& c = fs.cell[(size_t)s * fs.n_vals + b.val[i]];
  if (c.acc != 0) { b.status[i] = kReadCell; return; }
  const uint64_t key = cand_key(b.stamp, i);
  const uint64_t old = atomicMin((unsigned long long*)&c.cand, (unsigned long long)key);
  uint8_t tf = 0;
  if (old < key) tf = kReadCell;                           // an earlier vote of the batch holds it
  else if (cand_of(old, b.stamp) != TXV_NONE) b.mark[(uint32_t)old] = 1;   // took it from a later one
  b.status[i] = tf;
}

__device__ __forceinline__ bool pending_in_set(const FlowBatch& b, uint32_t i) {
  return b.pre[i] == TXV_S_PENDING && b.set[i] != TXV_NONE;
}

__device__ __forceinline__ bool sig_eq_arena(const FlowState& fs, const FlowBatch& b, uint32_t i, uint32_t r) {
  uint32_t d = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) d |= b.sig[(size_t)j * b.n_pad + i] ^ fs.arena_sig[(size_t)j * fs.max_accepted + r];
  return d == 0;
}
__device__ __forceinline__ bool sig_eq_votes(const FlowBatch& b, uint32_t i, uint32_t f) {
  uint32_t d = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) d |= b.sig[(size_t)j * b.n_pad + i] ^ b.sig[(size_t)j * b.n_pad + f];
  return d == 0;
}

// each pending vote's code from its cell (types/vote_set.go:109-119); an ADDED vote takes an
// arena row (one atomic per 1024-vote block for the block's ADDED votes) and stores the accepted vote in full
// (the reference's votes[addr] = vote, vote_set.go:154); the cell keeps the row for the crossing
// step, which publishes it as the cell's accepted vote once no vote of the batch reads acc
__global__ void __launch_bounds__(1024) txv_k_tally_resolve(FlowState fs, FlowBatch b, int stamp_only) {
  __shared__ uint32_t wsum[16], wnew[16];
  __shared__ uint32_t base_s, nbase_s;
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  bool added = false;
  uint32_t s = TXV_NONE;
  TallyCell* cell = nullptr;
  if (i < b.n && pending_in_set(b, i)) {
    s = b.set[i];
    const uint8_t fl = b.flags[i];
    const bool sig64 = (fl & TXV_FLAG_SIG64) != 0;
    cell = fs.cell + (size_t)s * fs.n_vals + b.val[i];
    const bool first = b.status[i] == 0 && b.mark[i] == 0;   // tally_min: its cell's first verified vote
    const uint32_t acc = first ? 0u : cell->acc;
    uint8_t st;
    if (first) {
      st = TXV_S_ADDED;
      added = true;
    } else if (acc) {                                   // accepted in an earlier batch (vote_set.go:109-114)
      st = sig64 && sig_eq_arena(fs, b, i, acc - 1) ? TXV_S_DUPLICATE : TXV_S_NONDETERMINISTIC;
    } else {
      const uint32_t f = cand_of(cell->cand, b.stamp);
      if (f == i) { st = TXV_S_ADDED; added = true; }   // the reference stores it (vote_set.go:154)
      else if (f != TXV_NONE && f < i)           // an earlier vote of the batch was accepted
        st = sig64 && sig_eq_votes(b, i, f) ? TXV_S_DUPLICATE : TXV_S_NONDETERMINISTIC;
      else                                       // no accepted vote before it and it did not verify
        st = (fl & TXV_FLAG_BADMSG) ? TXV_S_SIGNBYTES : TXV_S_INVALID_SIGNATURE;
    }
    b.status[i] = st;
  }
  // the set's first ADDED vote of the batch lists the set for the crossing step.  The block's
  // ADDED votes first elect one vote per set in an LDS hash set (C5's tx-major arrival order puts
  // ~8 votes of each of ~128 sets in a block: one device-scope exchange per (block, set) instead of
  // per vote, which serialised on the ~200 hot stamps); the electee's coherent read filters the
  // sets already stamped, and the exchange decides the one vote that lists the set.
  // stamp_only (large batches, random arrival: a 1024-vote block holds ~1000 sets, each set
  // ~100 blocks' electees, and their exchanges cost C2's resolve 146 -> 387 us): the electee only
  // stamps the set with a plain store (every writer stores the same value), and a compaction
  // over the set ids after this launch lists the stamped ones
  bool fresh = false;
  if (stamp_only) {               // (block-uniform) no election: a store per ADDED vote whose XCD
    if (added && fs.set_stamp[s] != b.stamp) fs.set_stamp[s] = b.stamp;   // has not seen the stamp
  } else {
    __shared__ uint32_t l_set[2048];
    for (uint32_t k = threadIdx.x; k < 2048; k += 1024) l_set[k] = TXV_NONE;
    __syncthreads();
    bool rep = false;
    if (added) {
      for (uint32_t h = (s * 0x9E3779B1u) >> 21;; h = (h + 1) & 2047u) {
        const uint32_t o = atomicCAS(&l_set[h], TXV_NONE, s);
        if (o == TXV_NONE) { rep = true; break; }
        if (o == s) break;
      }
    }
    if (rep && __hip_atomic_load(&fs.set_stamp[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != b.stamp)
      fresh = atomicExch(&fs.set_stamp[s], b.stamp) != b.stamp;
  }
  // the block's ADDED votes take consecutive arena rows and its fresh sets consecutive list
  // entries: one atomic per 1024 votes each (a hot counter serialises at ~10k atomics per 50 us)
  const uint64_t m = __ballot(added), mf = __ballot(fresh);
  if (lane == 0) { wsum[w] = (uint32_t)__popcll(m); wnew[w] = (uint32_t)__popcll(mf); }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0, tf = 0;
    for (int k = 0; k < 16; ++k) { t += wsum[k]; tf += wnew[k]; }
    base_s = t ? atomicAdd(&fs.ctr->arena_used, t) : 0u;
    nbase_s = tf ? atomicAdd(&fs.ctr->n_stamped, tf) : 0u;
  }
  __syncthreads();
  if (!added) return;
  const uint64_t below = (1ull << lane) - 1ull;
  if (fresh) {
    uint32_t q = nbase_s + (uint32_t)__popcll(mf & below);
    for (int k = 0; k < w; ++k) q += wnew[k];
    b.stamped[q] = s;                         // q < sets touched by the batch <= n
  }
  uint32_t r = base_s + (uint32_t)__popcll(m & below);
  for (int k = 0; k < w; ++k) r += wsum[k];
  if (r >= fs.max_accepted) {
    atomicOr(&fs.ctr->err, TXV_FERR_ARENA);
    cell->row = 0;
    return;
  }
  cell->row = r + 1;
  const size_t M = fs.max_accepted;
#pragma unroll
  for (int j = 0; j < 16; ++j) fs.arena_sig[j * M + r] = b.sig[(size_t)j * b.n_pad + i];
  fs.arena_height[r] = b.height[i];
  fs.arena_sec[r] = b.ts_sec[i];
  fs.arena_nanos[r] = b.ts_nanos[i];
  fs.arena_val[r] = b.val[i];
  fs.arena_seq[r] = b.seq_base + i;
  uint32_t tk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (b.txkey) {
    const uint4* s4 = reinterpret_cast<const uint4*>(b.txkey + (size_t)i * 32);
    const uint4 x = s4[0], y = s4[1];
    tk[0] = x.x; tk[1] = x.y; tk[2] = x.z; tk[3] = x.w; tk[4] = y.x; tk[5] = y.y; tk[6] = y.z; tk[7] = y.w;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) fs.arena_txkey[j * M + r] = tk[j];
}

__device__ __forceinline__ int64_t wave_sum64(int64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

constexpr uint32_t kListCap = 1024;   // ADDED votes of a set kept in LDS (every set of a <= 1024-validator registry)
constexpr uint32_t kDigitBits = 6;     // crossing search: one 64-bucket histogram level per 6 arrival-index bits

__device__ __forceinline__ int64_t wave_incl_scan64(int64_t x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// One wave per set that ADDED votes in this batch (the work list tally_resolve compacted): its
// ADDED votes are the cells of its row whose candidate carries this batch's stamp (a stamped cell
// had no accepted vote when the batch began: tally_min posts to no other), listed in LDS as
// (arrival index, stake); the accepted rows are published in the same pass (every vote of the batch
// read acc in the resolve step).  The crossing (addVerifiedVote, types/vote_set.go:143-166, in
// arrival order) is the smallest arrival index whose prefix stake reaches `need`: found digit by
// digit over the arrival index, 6 bits per level from the top -- each level a 64-bucket stake
// histogram of the entries under the prefix chosen so far (LDS atomics), one wave-wide inclusive
// scan (DPP shuffles) and a ballot for the first bucket whose running stake reaches `need`.
// ceil(log2(n) / 6) levels (3 for a 64k batch, 4 for 1M), each one pass over the list: O(k) per
// set instead of the O(k^2) pairwise prefix sums and the row-rescanning binary lifting it
// replaced.  Sets with more ADDED votes than the list holds read their row
// again per level instead of the list.
// One-wave blocks: the kernel runs beside the next batch's K1b, whose entry buffers leave ~32 KB
// of a CU's LDS free -- so the list holds Cap entries: 1024 (12.5 KB) for large validator sets,
// 128 (2 KB) when no set can have more (n_vals <= 128, C2's 100), which lets 16 blocks share a CU
// beside K1b instead of 2 (with 2 the C2 tally's crossing pass crawled beside the whole K1b).
template <uint32_t Cap>
__global__ void __launch_bounds__(64) txv_k_tally_cross(FlowState fs, FlowBatch b, const uint32_t* n_stamped) {
  __shared__ __attribute__((aligned(16))) uint32_t l_vote[1][Cap];
  __shared__ __attribute__((aligned(16))) int64_t l_pow[1][Cap];
  __shared__ int64_t l_hist[1][64];
  const int lane = threadIdx.x & 63;
  constexpr uint32_t wv = 0;
  const uint32_t gw = blockIdx.x, n_waves = gridDim.x;
  const uint32_t n_list = *n_stamped;
  const uint32_t nbits = 32u - (uint32_t)__builtin_clz(max(b.n, 2u) - 1u);
  const uint32_t levels = (nbits + kDigitBits - 1) / kDigitBits;
  for (uint32_t j = gw; j < n_list; j += n_waves) {
    const uint32_t s = b.stamped[j];
    TallyCell* row = fs.cell + (size_t)s * fs.n_vals;
    // list this set's ADDED votes (compacted in validator order) and publish their rows
    uint32_t k = 0;
    int64_t part = 0;
    for (uint32_t v0 = 0; v0 < fs.n_vals; v0 += 64) {
      const uint32_t v = v0 + lane;
      uint32_t f = TXV_NONE;
      if (v < fs.n_vals) {
        const TallyCell c = row[v];
        f = cand_of(c.cand, b.stamp);
        if (f != TXV_NONE) row[v].acc = c.row;
      }
      const bool added = f != TXV_NONE;
      const uint64_t m = __ballot(added);
      if (added) {
        const uint32_t e = k + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        const int64_t pw = fs.power[v];
        if (e < Cap) { l_vote[wv][e] = f; l_pow[wv][e] = pw; }
        part += pw;
      }
      k += (uint32_t)__popcll(m);
    }
    __threadfence_block();
    const int64_t prior = fs.set_sum[s];
    const int64_t total = prior + wave_sum64(part);
    uint32_t cross = TXV_NO_CROSS;
    if (prior >= fs.quorum) {
      cross = 0;                              // already committed: every ADDED vote re-fires
    } else if (total >= fs.quorum) {
      const int64_t need = fs.quorum - prior;
      const bool in_lds = k <= Cap;
      uint32_t pfx = 0;                       // the crossing index's digits chosen so far
      int64_t before = 0;                     // stake of the entries below the prefix's range
      for (uint32_t lv = 0; lv < levels; ++lv) {
        const uint32_t sh = kDigitBits * (levels - 1u - lv);
        l_hist[wv][lane] = 0;
        __threadfence_block();
        if (in_lds) {
          for (uint32_t e = lane; e < k; e += 64) {
            const uint32_t f = l_vote[wv][e];
            if (((f >> sh) >> kDigitBits) == pfx)
              atomicAdd((unsigned long long*)&l_hist[wv][(f >> sh) & 63u], (unsigned long long)l_pow[wv][e]);
          }
        } else {
          for (uint32_t v = lane; v < fs.n_vals; v += 64) {
            const uint32_t f = cand_of(row[v].cand, b.stamp);
            if (f != TXV_NONE && ((f >> sh) >> kDigitBits) == pfx)
              atomicAdd((unsigned long long*)&l_hist[wv][(f >> sh) & 63u], (unsigned long long)fs.power[v]);
          }
        }
        __threadfence_block();
        const int64_t h = l_hist[wv][lane];
        const int64_t inc = wave_incl_scan64(h, lane);
        const uint64_t hit = __ballot(before + inc >= need);   // non-empty: the range holds >= need
        const int c = (int)__builtin_ctzll(hit);
        before += __shfl(inc, c, 64) - __shfl(h, c, 64);
        pfx = (pfx << kDigitBits) | (uint32_t)c;
      }
      cross = pfx;
    }
    if (lane == 0) {
      fs.set_sum[s] = total;
      fs.set_cross[s] = cross;
      if (prior < fs.quorum && total >= fs.quorum) b.ev_flag[cross] = 1;   // the commit event
    }
  }
}

struct EventPred {
  FlowBatch b;
  __device__ bool operator()(uint32_t i) const { return b.ev_flag[i] != 0; }
};
struct EventAct {
  FlowState fs;
  FlowBatch b;
  __device__ void operator()(uint32_t i, uint32_t rank) const {
    const uint32_t s = b.set[i];
    FlowEvent e;
    e.vote_index = i;
    e.tx_index = s;
    e.sum = fs.set_sum[s];
    b.ev_host[rank] = e;
  }
};

// final statuses into mapped host memory (an ADDED vote at or after its set's crossing index
// fires), and the number of commit events per scan block (items b*1024 + k*256 + t, as
// txv_k_scan_count) for the event compaction
__global__ void __launch_bounds__(256) txv_k_status_out(FlowState fs, FlowBatch b) {
  const uint32_t base = blockIdx.x * kScanItems + threadIdx.x;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = base + 256u * k;
    if (i >= b.n) continue;
    const uint8_t p = b.pre[i];
    uint8_t st = p;
    if (p == TXV_S_PENDING) {
      const uint32_t s = b.set[i];
      if (s == TXV_NONE) {
        st = TXV_S_INVALID_SIGNATURE;
      } else {
        st = b.status[i];
        if (st == TXV_S_ADDED) {
          const uint32_t x = fs.set_cross[s];
          if (x != TXV_NO_CROSS && i >= x) st |= TXV_S_FIRED;
        }
      }
    }
    b.status_host[i] = st;
    c += b.ev_flag[i] != 0;
  }
  uint32_t total;
  (void)block_excl_scan(c, &total);
  if (threadIdx.x == 0) b.blk[blockIdx.x] = total;
}

// the event compaction's scan top, then the batch summary into mapped host memory
__global__ void __launch_bounds__(256) txv_k_event_top(FlowState fs, FlowBatch b, uint32_t nb) {
  const uint32_t t = threadIdx.x;
  const uint32_t per = (nb + 255) / 256;
  const uint32_t lo = min(t * per, nb), hi = min(lo + per, nb);
  uint32_t s = 0;
  for (uint32_t j = lo; j < hi; ++j) s += b.blk[j];
  uint32_t total;
  uint32_t run = block_excl_scan(s, &total);
  for (uint32_t j = lo; j < hi; ++j) {
    const uint32_t v = b.blk[j];
    b.blk[j] = run;
    run += v;
  }
  if (t == 0) {
    b.blk[nb] = total;
    FlowSummary sm;
    sm.n_sets = fs.ctr->n_sets;
    sm.n_events = total;
    sm.arena_used = min(fs.ctr->arena_used, fs.max_accepted);
    sm.err = fs.ctr->err;
    sm.key_used = fs.ctr->key_used;
    *b.summary_host = sm;
  }
}

// Batches of up to kFusedEventTiles scan tiles (C5's 64k): one kernel after the crossing step --
// the final statuses as txv_k_status_out, the commit events compacted in vote order by a
// single-pass look-back scan (lookback.h; tiles taken by ticket, words tagged with the batch
// stamp), and the batch summary by the last tile -- instead of the three launches above (C5
// tally after verify in the pipeline 0.085 -> 0.078 ms, profiles/r05/ev).  Over the 977 tiles of a
// 1M-vote batch running at once, the look-back walks back through many aggregate-only words: the
// standalone C2 tally took 0.216 vs 0.204 ms, so large batches keep the three launches.
constexpr uint32_t kFusedEventTiles = 128;
__global__ void __launch_bounds__(256) txv_k_status_events(FlowState fs, FlowBatch b, uint32_t n_tiles) {
  const uint32_t tile = take_tile(&fs.ctr->ev_ticket);
  const uint32_t base = tile * kScanItems + threadIdx.x;
  bool f[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = base + 256u * k;
    f[k] = false;
    if (i >= b.n) continue;
    const uint8_t p = b.pre[i];
    uint8_t st = p;
    if (p == TXV_S_PENDING) {
      const uint32_t s = b.set[i];
      if (s == TXV_NONE) {
        st = TXV_S_INVALID_SIGNATURE;
      } else {
        st = b.status[i];
        if (st == TXV_S_ADDED) {
          const uint32_t x = fs.set_cross[s];
          if (x != TXV_NO_CROSS && i >= x) st |= TXV_S_FIRED;
        }
      }
    }
    b.status_host[i] = st;
    f[k] = b.ev_flag[i] != 0;
  }
  uint32_t rank[4], total;
  tile_scan(f, rank, b.ev_tiles, tile, b.stamp, &fs.ctr->err, TXV_FERR_LOOKBACK, &total);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (!f[k]) continue;
    const uint32_t i = base + 256u * k, s = b.set[i];
    FlowEvent e;
    e.vote_index = i;
    e.tx_index = s;
    e.sum = fs.set_sum[s];
    b.ev_host[rank[k]] = e;
  }
  if (tile + 1 == n_tiles && threadIdx.x == 0) {
    FlowSummary sm;
    sm.n_sets = fs.ctr->n_sets;
    sm.n_events = total;
    sm.arena_used = min(fs.ctr->arena_used, fs.max_accepted);
    // (a tile that timed out in its look-back or-ed its bit in before it published its word)
    sm.err = __hip_atomic_load(&fs.ctr->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sm.key_used = fs.ctr->key_used;
    *b.summary_host = sm;
  }
}

// ------------------------------------------------------------------ reset / readers
__global__ void __launch_bounds__(256) txv_k_reset_sets(FlowState fs, int keep_ids) {
  const uint32_t ns = fs.ctr->n_sets;
  const uint64_t cells = (uint64_t)ns * fs.n_vals;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < cells; c += stride)
    *reinterpret_cast<uint64_t*>(&fs.cell[c].acc) = 0;   // acc and row
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < ns; s += stride) {
    fs.set_sum[s] = 0;
    if (!keep_ids) {
      SetEntry& e = fs.tab[fs.set_entry[s]];
      e.h = 0; e.len = 0; e.key_off = 0; e.first = 0; e.id = 0; e.state = TXV_SE_EMPTY;
    }
  }
}

__global__ void __launch_bounds__(256) txv_k_init_cells(FlowState fs, uint64_t cells, int clear_acc) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < cells; c += stride) {
    fs.cell[c].cand = ~0ull;                          // stamp 0: no candidate
    if (clear_acc) *reinterpret_cast<uint64_t*>(&fs.cell[c].acc) = 0;
  }
}

__global__ void txv_k_reset_counters(FlowState fs, int keep_ids) {
  if (!keep_ids) {
    fs.ctr->n_sets = 0;
    fs.ctr->n_digested = 0;
    fs.ctr->key_used = 0;
    fs.ctr->err = 0;
  } else {
    fs.ctr->err &= ~TXV_FERR_ARENA;
  }
  fs.ctr->arena_used = 0;
}

__global__ void __launch_bounds__(256) txv_k_lookup(FlowState fs, const uint8_t* keys, const uint32_t* off,
                                                    const uint32_t* len, uint32_t n, uint32_t* out_id) {
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  if (q >= n) return;
  const uint8_t* kp = keys + off[q];
  const uint32_t l = len[q];
  const uint64_t h = txv_hash::hash_chunks(l, fs.hash_seed, [&](uint32_t k) { return ld64u(kp + k); });
  uint32_t id = TXV_NONE;
  for (uint32_t slot = (uint32_t)h & fs.tab_mask, probes = 0; probes <= fs.tab_mask; slot = (slot + 1) & fs.tab_mask, ++probes) {
    const SetEntry& e = fs.tab[slot];
    if (e.state == TXV_SE_EMPTY) break;
    if (e.state == TXV_SE_KEPT && e.h == h && e.len == l && key_eq(fs.keys + (e.key_off - 1), kp, l)) {
      id = e.id;
      break;
    }
  }
  out_id[q] = id;
}

__global__ void __launch_bounds__(256) txv_k_gather(FlowState fs, const uint32_t* ids, uint32_t n, int64_t* out_sum,
                                                    uint32_t* out_txkey, AccRow* out_rows) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t q = (uint32_t)(t / fs.n_vals), v = (uint32_t)(t % fs.n_vals);
  if (q >= n) return;
  const uint32_t id = ids[q];
  const bool ok = id != TXV_NONE && id < fs.max_txs;
  if (v == 0) {
    if (out_sum) out_sum[q] = ok ? fs.set_sum[id] : 0;
    if (out_txkey)
      for (int j = 0; j < 8; ++j) out_txkey[(size_t)q * 8 + j] = ok ? fs.set_txkey[(size_t)id * 8 + j] : 0u;
  }
  if (!out_rows) return;
  AccRow r{};
  r.val = TXV_NONE;
  const uint32_t a = ok ? fs.cell[(size_t)id * fs.n_vals + v].acc : 0u;
  if (a) {
    const size_t M = fs.max_accepted, k = a - 1;
    for (int j = 0; j < 16; ++j) r.sig[j] = fs.arena_sig[j * M + k];
    for (int j = 0; j < 8; ++j) r.txkey[j] = fs.arena_txkey[j * M + k];
    r.height = fs.arena_height[k];
    r.ts_sec = fs.arena_sec[k];
    r.ts_nanos = fs.arena_nanos[k];
    r.val = fs.arena_val[k];
    r.seq = fs.arena_seq[k];
  }
  out_rows[t] = r;
}

__global__ void __launch_bounds__(256) txv_k_keys(FlowState fs, const uint32_t* ids, uint32_t n, uint64_t* out_off,
                                                  uint32_t* out_len) {
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  if (q >= n) return;
  const uint32_t id = ids[q];
  if (id == TXV_NONE || id >= fs.max_txs) { out_off[q] = 0; out_len[q] = 0; return; }
  const SetEntry& e = fs.tab[fs.set_entry[id]];
  out_off[q] = e.key_off - 1;
  out_len[q] = e.len;
}

// bit s of word t: TxVoteSet s has +2/3 (maj23 is sticky and the sum only grows)
__device__ __forceinline__ uint32_t commit_word(const FlowState& fs, uint32_t t, uint32_t ns) {
  uint32_t w = 0;
  for (uint32_t j = 0; j < 32; ++j) {
    const uint32_t s = t * 32 + j;
    if (s < ns && fs.set_sum[s] >= fs.quorum) w |= 1u << j;
  }
  return w;
}

// the exchange names SHA-256(TxHash)[0:16] of the sets numbered since the last pack (only a
// multi-rank step packs: the AddVote chain itself computes none)
__global__ void __launch_bounds__(256) txv_k_digest(FlowState fs, uint32_t n_cap) {
  const uint32_t id = fs.ctr->n_digested + blockIdx.x * 256 + threadIdx.x;
  if (id >= min(fs.ctr->n_sets, n_cap)) return;
  const SetEntry& e = fs.tab[fs.set_entry[id]];
  uint32_t h[8];
  txv::sha256_bytes(fs.keys + (e.key_off - 1), e.len, h);
#pragma unroll
  for (int j = 0; j < 4; ++j) fs.set_digest[(size_t)id * 4 + j] = __builtin_bswap32(h[j]);   // bytes in order
}

__global__ void __launch_bounds__(256) txv_k_pack(FlowState fs, uint32_t* dst, uint32_t bm_words, uint32_t n_cap) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  const uint32_t ns = min(fs.ctr->n_sets, n_cap);
  if (t == 0) { dst[0] = ns; dst[1] = 1; fs.ctr->n_digested = ns; }   // word 1: layout 1 = with the per-set digests
  if (t < bm_words) dst[2 + t] = commit_word(fs, t, ns);
  if (t < n_cap) {
    const int64_t sm = t < ns ? fs.set_sum[t] : 0;
    dst[2 + bm_words + 2 * t] = (uint32_t)(uint64_t)sm;
    dst[2 + bm_words + 2 * t + 1] = (uint32_t)((uint64_t)sm >> 32);
    uint32_t* dg = dst + 2 + bm_words + 2 * (size_t)n_cap + 4 * (size_t)t;
#pragma unroll
    for (int j = 0; j < 4; ++j) dg[j] = t < ns ? fs.set_digest[(size_t)t * 4 + j] : 0u;
  }
}

__global__ void __launch_bounds__(256) txv_k_bitmap(FlowState fs, uint32_t* dst, uint32_t bm_words) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t < bm_words) dst[t] = commit_word(fs, t, min(fs.ctr->n_sets, fs.max_txs));
}

// the sets the batch stamped (tally_resolve with stamp_only), listed in id order
constexpr uint32_t kStampCompactMin = 1u << 18;
struct StampPred {
  FlowState fs;
  FlowBatch b;
  __device__ bool operator()(uint32_t s) const { return fs.set_stamp[s] == b.stamp; }
};
struct StampAct {
  FlowBatch b;
  __device__ void operator()(uint32_t s, uint32_t rank) const { b.stamped[rank] = s; }
};

template <class Pred, class Act>
hipError_t compact(Pred p, Act act, uint32_t n, uint32_t* blk, hipStream_t st) {
  const uint32_t nb = (n + kScanItems - 1) / kScanItems;
  if (nb) hipLaunchKernelGGL((txv_k_scan_count<Pred>), dim3(nb), dim3(256), 0, st, p, n, blk);
  hipLaunchKernelGGL(txv_k_scan_top, dim3(1), dim3(256), 0, st, blk, nb);
  if (nb) hipLaunchKernelGGL((txv_k_scan_apply<Pred, Act>), dim3(nb), dim3(256), 0, st, p, act, n, blk);
  return hipGetLastError();
}

// Experiment builds only (tools/profile/build_variant_flow.sh -DTXV_EXP_SKIP): TXV_EXP_SKIP=<mask>
// leaves flow kernels out of every chain (wrong results; for attributing co-running costs):
// 1 tally_min, 2 resolve, 16 cross, 32 status + events,
// 64 route_key, 128 new-id compaction
#ifdef TXV_EXP_SKIP
uint32_t exp_skip() {
  static const uint32_t m = getenv("TXV_EXP_SKIP") ? (uint32_t)strtoul(getenv("TXV_EXP_SKIP"), nullptr, 0) : 0u;
  return m;
}
#define TXV_SKIP(bit) (exp_skip() & (bit))
#else
#define TXV_SKIP(bit) false
#endif

}  // namespace

extern "C" {

hipError_t txv_flow_prep(const FlowState* fs, const FlowBatch* b, hipStream_t st) {
  if (((uint64_t)b->n + kScanItems - 1) / kScanItems > 8192) return hipErrorInvalidValue;
  const uint32_t g = (b->n + 255) / 256;
  if (g) hipLaunchKernelGGL(txv_k_route_prep, dim3(g), dim3(256), 0, st, *fs, *b);
  return hipGetLastError();
}

hipError_t txv_flow_route(const FlowState* fs, const FlowBatch* b, hipStream_t st) {
  if (((uint64_t)b->n + kScanItems - 1) / kScanItems > 8192) return hipErrorInvalidValue;
  const uint32_t g = (b->n + 255) / 256;
  if (g && !TXV_SKIP(64)) hipLaunchKernelGGL(txv_k_route_key, dim3(g), dim3(256), 0, st, *fs, *b);
  return hipGetLastError();
}

hipError_t txv_flow_new_ids(const FlowState* fs, const FlowBatch* b, hipStream_t st) {
  if (TXV_SKIP(128)) return hipSuccess;
  return compact(NewSetPred{*fs, *b}, NewSetAct{*fs, *b}, b->n, b->blk, st);
}

// sets_bound: an upper bound on the set ids in use after this batch (the host's count as of
// the last waited batch + this batch's votes, at most max_txs): the crossing step covers it
hipError_t txv_flow_tally(const FlowState* fs, const FlowBatch* b, uint32_t sets_bound, hipStream_t st) {
  const uint32_t nb = (b->n + kScanItems - 1) / kScanItems;
  const uint32_t g = (b->n + 255) / 256;
  if (!TXV_SKIP(1)) hipLaunchKernelGGL(txv_k_tally_min, dim3(g ? g : 1), dim3(256), 0, st, *fs, *b, nb);
  sets_bound = std::min(sets_bound, fs->max_txs);
  // large batches list their stamped sets by a compaction over the set ids (see tally_resolve)
  const bool stamp_only = b->n >= kStampCompactMin;
  if (b->n && !TXV_SKIP(2))
    hipLaunchKernelGGL(txv_k_tally_resolve, dim3((b->n + 1023) / 1024), dim3(1024), 0, st, *fs, *b, stamp_only ? 1 : 0);
  const uint32_t* n_stamped = &fs->ctr->n_stamped;
  if (stamp_only) {
    hipError_t e;
    if ((e = compact(StampPred{*fs, *b}, StampAct{*b}, sets_bound, fs->set_blk, st))) return e;
    n_stamped = fs->set_blk + (sets_bound + kScanItems - 1) / kScanItems;   // scan_top's total
  }
  // persistent waves over the batch's stamped sets (at most min(sets, votes) of them): one wave per set
  // TXV_CROSS_BLOCKS (experiment): the persistent one-wave blocks' cap (default 4096)
  static const uint32_t cross_cap = getenv("TXV_CROSS_BLOCKS") ? (uint32_t)atoi(getenv("TXV_CROSS_BLOCKS")) : 4096u;
  const uint32_t cross_blocks = std::max<uint32_t>(1, std::min<uint32_t>(std::min(sets_bound, b->n), cross_cap));
  if (!TXV_SKIP(16)) {
    if (fs->n_vals <= 128) hipLaunchKernelGGL(txv_k_tally_cross<128>, dim3(cross_blocks), dim3(64), 0, st, *fs, *b, n_stamped);
    else hipLaunchKernelGGL(txv_k_tally_cross<kListCap>, dim3(cross_blocks), dim3(64), 0, st, *fs, *b, n_stamped);
  }
  if (TXV_SKIP(32)) return hipGetLastError();
  if (nb <= kFusedEventTiles) {
    const uint32_t n_tiles = nb ? nb : 1u;   // an empty batch still writes its summary
    hipLaunchKernelGGL(txv_k_status_events, dim3(n_tiles), dim3(256), 0, st, *fs, *b, n_tiles);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(txv_k_status_out, dim3(nb), dim3(256), 0, st, *fs, *b);
  hipLaunchKernelGGL(txv_k_event_top, dim3(1), dim3(256), 0, st, *fs, *b, nb);
  hipLaunchKernelGGL((txv_k_scan_apply<EventPred, EventAct>), dim3(nb), dim3(256), 0, st, EventPred{*b},
                     EventAct{*fs, *b}, b->n, b->blk);
  return hipGetLastError();
}

// a column every element of which is the same value (the host saw a uniform column and did not
// upload it: txv_submit_votes' staging)
__global__ void __launch_bounds__(256) txv_k_fill64(uint64_t* dst, uint64_t v, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] = v;
}

// TxKey from TxHash: a batch whose every non-nil vote carries TxKey == the 32 bytes its 64-char
// upper-hex TxHash spells (TxKey = SHA-256(tx), TxHash = %X of the same digest,
// types/tx_vote.go:38-45; the host checked it, txv_submit_votes' staging) does not upload the
// TxKey column: each vote's key is decoded here from the TxHash arena, 8 hex chars per load
__device__ __forceinline__ uint32_t hex_nibbles8(uint64_t c) {   // 8 chars of [0-9A-F] -> 4 bytes in order
  uint32_t out = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t ch = (uint32_t)(c >> (8 * k)) & 0xFFu;
    const uint32_t nib = ch <= '9' ? ch - '0' : ch - 'A' + 10u;
    out |= nib << ((k & 1) ? 8 * (k >> 1) : 8 * (k >> 1) + 4);
  }
  return out;
}

__global__ void __launch_bounds__(256) txv_k_txkey_from_hash(const uint8_t* th, const uint32_t* off, const uint8_t* nil,
                                                             uint32_t n, uint8_t* txkey) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!(nil && nil[i])) {
    const uint8_t* p = th + off[i];
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = hex_nibbles8(ld64u(p + 8 * k));
  }
  uint4* d = reinterpret_cast<uint4*>(txkey + (size_t)i * 32);
  d[0] = make_uint4(w[0], w[1], w[2], w[3]);
  d[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

hipError_t txv_txkey_from_hash(const uint8_t* th, const uint32_t* off, const uint8_t* nil, uint32_t n, uint8_t* txkey,
                               hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_txkey_from_hash, dim3((n + 255) / 256), dim3(256), 0, st, th, off, nil, n, txkey);
  return hipGetLastError();
}

hipError_t txv_fill64(uint64_t* dst, uint64_t v, uint32_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_fill64, dim3((n + 255) / 256), dim3(256), 0, st, dst, v, n);
  return hipGetLastError();
}

hipError_t txv_flow_reset(const FlowState* fs, int keep_ids, hipStream_t st) {
  hipLaunchKernelGGL(txv_k_reset_sets, dim3(1024), dim3(256), 0, st, *fs, keep_ids);
  hipLaunchKernelGGL(txv_k_reset_counters, dim3(1), dim3(1), 0, st, *fs, keep_ids);
  return hipGetLastError();
}

hipError_t txv_flow_init_cells(const FlowState* fs, uint64_t cells, int clear_acc, hipStream_t st) {
  if (!cells) return hipSuccess;
  hipLaunchKernelGGL(txv_k_init_cells, dim3((uint32_t)std::min<uint64_t>((cells + 255) / 256, 8192)), dim3(256), 0, st,
                     *fs, cells, clear_acc);
  return hipGetLastError();
}

hipError_t txv_flow_lookup(const FlowState* fs, const uint8_t* keys, const uint32_t* off, const uint32_t* len,
                           uint32_t n, uint32_t* out_id, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_lookup, dim3((n + 255) / 256), dim3(256), 0, st, *fs, keys, off, len, n, out_id);
  return hipGetLastError();
}

hipError_t txv_flow_gather(const FlowState* fs, const uint32_t* ids, uint32_t n, int64_t* out_sum, uint32_t* out_txkey,
                           AccRow* out_rows, hipStream_t st) {
  const uint64_t t = (uint64_t)n * std::max<uint32_t>(fs->n_vals, 1);
  if (!t || !fs->n_vals) return hipSuccess;
  hipLaunchKernelGGL(txv_k_gather, dim3((uint32_t)((t + 255) / 256)), dim3(256), 0, st, *fs, ids, n, out_sum, out_txkey,
                     out_rows);
  return hipGetLastError();
}

hipError_t txv_flow_keys(const FlowState* fs, const uint32_t* ids, uint32_t n, uint64_t* out_off, uint32_t* out_len,
                         hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(txv_k_keys, dim3((n + 255) / 256), dim3(256), 0, st, *fs, ids, n, out_off, out_len);
  return hipGetLastError();
}

hipError_t txv_flow_pack(const FlowState* fs, uint32_t* dst, uint32_t bm_words, uint32_t n_cap, hipStream_t st) {
  const uint32_t t = std::max<uint32_t>(std::max(bm_words, n_cap), 1);
  hipLaunchKernelGGL(txv_k_digest, dim3((std::max<uint32_t>(n_cap, 1) + 255) / 256), dim3(256), 0, st, *fs, n_cap);
  hipLaunchKernelGGL(txv_k_pack, dim3((t + 255) / 256), dim3(256), 0, st, *fs, dst, bm_words, n_cap);
  return hipGetLastError();
}

hipError_t txv_flow_bitmap(const FlowState* fs, uint32_t* dst, uint32_t bm_words, hipStream_t st) {
  if (!bm_words) return hipSuccess;
  hipLaunchKernelGGL(txv_k_bitmap, dim3((bm_words + 255) / 256), dim3(256), 0, st, *fs, dst, bm_words);
  return hipGetLastError();
}

}  // extern "C"
