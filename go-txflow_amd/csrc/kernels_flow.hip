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
//   route    one lane per vote: validator lookup (address hash table), pre-checks, SignBytes
//            length / amino time check, signature transpose into the column-major layout the
//            verify kernels read, and find-or-insert of the TxHash into the set table; a key
//            seen for the first time records the smallest arrival index that carries it
//   new ids  a stream compaction over the arrival order of "first occurrence of a new key"
//            numbers the new sets exactly as the sequential loop would (first-seen order)
//   set ids  every vote reads its set id; the (set, validator) cells of pending votes are
//            cleared for the resolution below
//   (SignBytes + K1a/K1b verify run here, kernels_signbytes.hip / kernels_verify.hip)
//   min      every verified pending vote posts its arrival index to its cell (atomic min):
//            the cell then holds the FIRST verified vote of the (set, validator) group
//   resolve  each pending vote decides its code from its cell: earlier accepted vote ->
//            signature compare; first verified == itself -> ADDED (an arena row is taken);
//            first verified earlier -> signature compare with it; none -> invalid signature
//   bucket   the ADDED votes of each set (<= one per validator) are listed in the set's cell row
//   cross    one wave per set with ADDED votes: stake sum, and the arrival index at which the
//            prefix (in arrival order) of the stake first reaches quorum, by binary lifting
//            over the index bits; ADDED votes at or after it carry the fired bit
//   events   compaction of the crossing votes in arrival order -> commit events
//   out      final statuses (pre-check or tally) into mapped host memory
#include <algorithm>

#include "txv_device.h"
#include "txv_flow.h"

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

__device__ __forceinline__ uint32_t ld_state(const SetEntry* e) {
  return __hip_atomic_load(&e->state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ const uint8_t* entry_key(const FlowState& fs, const FlowBatch& b, const SetEntry& e,
                                                     uint32_t state) {
  return (state == TXV_SE_BATCH ? b.th : fs.keys) + e.key_off;
}

// Find-or-insert of one TxHash (linear probing).  A lane that claims an empty slot writes the
// entry and publishes it with a release store in the same loop iteration; a lane that meets a
// slot still being written re-reads it in its next iteration (the writer has finished by then,
// whether it is in the same wave or not), so no lane ever waits on a lane that waits on it.
__device__ uint32_t set_find_or_insert(const FlowState& fs, const FlowBatch& b, uint64_t h, const uint8_t* kp,
                                       uint32_t len, uint64_t key_off, uint32_t i) {
  uint32_t slot = (uint32_t)h & fs.tab_mask;
  uint32_t probes = 0;
  for (;;) {
    SetEntry* e = fs.tab + slot;
    const uint32_t st = ld_state(e);
    if (st == TXV_SE_EMPTY) {
      if (atomicCAS(&e->state, TXV_SE_EMPTY, TXV_SE_BUSY) == TXV_SE_EMPTY) {
        e->h = h;
        e->len = len;
        e->key_off = key_off;
        e->first = i;
        e->id = TXV_NONE;
        __hip_atomic_store(&e->state, TXV_SE_BATCH, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        return slot;
      }
      // lost the claim: re-read the slot with acquire ordering in the next iteration
    } else if (st != TXV_SE_BUSY) {
      if (e->h == h && e->len == len && key_eq(entry_key(fs, b, *e, st), kp, len)) {
        if (st == TXV_SE_BATCH) atomicMin(&e->first, i);
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
__global__ void __launch_bounds__(256) txv_k_route(FlowState fs, FlowBatch b) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= b.n) return;
  b.ev_flag[i] = 0;
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
  if (b.nil && b.nil[i]) {   // nil *TxVote: no set is created (AddVote's first check)
    b.pre[i] = TXV_S_NIL; b.flags[i] = 0; b.entry[i] = TXV_NONE; b.msg_len[i] = 0; b.val[i] = 0;
    return;
  }
  // TxVoteSets[vote.TxHash], created on first sight (txflow/service.go:200-209)
  const uint32_t len = b.th_len[i];
  const uint32_t off = b.th_off[i];
  const uint8_t* kp = b.th + off;
  const uint64_t h = txv_hash::hash_chunks(len, fs.hash_seed, [&](uint32_t k) { return ld64u(kp + k); });
  b.entry[i] = set_find_or_insert(fs, b, h, kp, len, off, i);
  // AddVote pre-checks (types/vote_set.go:93-106)
  const uint32_t al = b.addr_len[i];
  uint32_t v = TXV_NONE;
  uint8_t pre = TXV_S_PENDING;
  if (al == 0) {
    pre = TXV_S_EMPTY_ADDR;
  } else if (al == 20) {
    const uint32_t* ap = reinterpret_cast<const uint32_t*>(b.addr + (size_t)i * 20);
    const uint32_t a[5] = {ap[0], ap[1], ap[2], ap[3], ap[4]};
    v = find_validator(fs, a);
    if (v == TXV_NONE) pre = TXV_S_UNKNOWN_VALIDATOR;
  } else {
    pre = TXV_S_UNKNOWN_VALIDATOR;
  }
  const int L = signbytes_len(b.height[i], len, b.ts_sec[i], b.ts_nanos[i], b.chain_len);
  b.pre[i] = pre;
  b.val[i] = v == TXV_NONE ? 0u : v;
  b.msg_len[i] = (pre == TXV_S_PENDING && L > 0) ? (uint32_t)L : 0u;
  b.flags[i] = pre != TXV_S_PENDING ? 0
               : (uint8_t)(TXV_FLAG_PENDING | (b.sig_len[i] == 64 ? TXV_FLAG_SIG64 : 0) | (L < 0 ? TXV_FLAG_BADMSG : 0));
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

template <class Pred>
__global__ void __launch_bounds__(256) txv_k_scan_count(Pred p, uint32_t n, uint32_t* blk) {
  const uint32_t base = blockIdx.x * kScanItems + threadIdx.x * 4;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) c += (base + k < n && p(base + k)) ? 1u : 0u;
  uint32_t total;
  (void)block_excl_scan(c, &total);
  if (threadIdx.x == 0) blk[blockIdx.x] = total;
}

// exclusive offsets of nb block counts (nb <= 8192), blk[nb] = total
__global__ void __launch_bounds__(1024) txv_k_scan_top(uint32_t* blk, uint32_t nb) {
  __shared__ uint32_t wsum[16];
  const uint32_t t = threadIdx.x;
  uint32_t v[8], s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t j = t * 8 + k;
    v[k] = j < nb ? blk[j] : 0u;
    s += v[k];
  }
  const int lane = t & 63, w = t >> 6;
  uint32_t x = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
  for (int k = 0; k < 16; ++k) {
    if (k < w) before += wsum[k];
    all += wsum[k];
  }
  uint32_t run = before + x - s;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t j = t * 8 + k;
    if (j < nb) blk[j] = run;
    run += v[k];
  }
  if (t == 0) blk[nb] = all;
}

template <class Pred, class Act>
__global__ void __launch_bounds__(256) txv_k_scan_apply(Pred p, Act act, uint32_t n, const uint32_t* blk) {
  const uint32_t base = blockIdx.x * kScanItems + threadIdx.x * 4;
  bool f[4];
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[k] = base + k < n && p(base + k);
    c += f[k] ? 1u : 0u;
  }
  uint32_t total;
  uint32_t rank = blk[blockIdx.x] + block_excl_scan(c, &total);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (f[k]) act(base + k, rank++);
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
// bytes into the persistent key arena, record the set's TxKey (service.go:201-207)
struct NewSetAct {
  FlowState fs;
  FlowBatch b;
  __device__ void operator()(uint32_t i, uint32_t rank) const {
    const uint32_t slot = b.entry[i];
    SetEntry& e = fs.tab[slot];
    const uint32_t id = fs.ctr->n_sets + rank;
    const uint32_t len = e.len, span = (len + 7u) & ~7u;
    const unsigned long long ko = atomicAdd((unsigned long long*)&fs.ctr->key_used, (unsigned long long)span);
    if (ko + span + 16 > fs.keys_cap) {
      atomicOr(&fs.ctr->err, TXV_FERR_KEYS);
    } else {
      const uint8_t* src = b.th + e.key_off;
      uint64_t* dst = reinterpret_cast<uint64_t*>(fs.keys + ko);
      for (uint32_t k = 0; k < span; k += 8) dst[k / 8] = ld64u(src + k) & (k + 8 <= len ? ~0ull : ((1ull << (8 * (len - k))) - 1ull));
      e.key_off = ko;
    }
    e.state = TXV_SE_KEPT;
    if (id >= fs.max_txs) {
      atomicOr(&fs.ctr->err, TXV_FERR_SETS);
      e.id = TXV_NONE;
      return;
    }
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

// every vote's set id; pending votes clear their (set, validator) cell
__global__ void __launch_bounds__(256) txv_k_set_ids(FlowState fs, FlowBatch b, uint32_t nb) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i == 0) {
    const uint32_t created = b.blk[nb];
    const uint32_t ns = fs.ctr->n_sets + created;
    fs.ctr->n_sets = ns > fs.max_txs ? fs.max_txs : ns;
    fs.ctr->n_touched = 0;
    fs.ctr->batch += 1;
  }
  if (i >= b.n) return;
  const uint32_t e = b.entry[i];
  const uint32_t s = e == TXV_NONE ? TXV_NONE : fs.tab[e].id;
  b.set[i] = s;
  if (s != TXV_NONE && b.pre[i] == TXV_S_PENDING) fs.cand[(size_t)s * fs.n_vals + b.val[i]] = TXV_NONE;
}

// ------------------------------------------------------------------ tally
__device__ __forceinline__ bool pending_in_set(const FlowBatch& b, uint32_t i) {
  return b.pre[i] == TXV_S_PENDING && b.set[i] != TXV_NONE;
}

// the cell's first verified vote of the batch (votes of cells with an accepted vote skip)
__global__ void __launch_bounds__(256) txv_k_tally_min(FlowState fs, FlowBatch b) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= b.n || !pending_in_set(b, i) || b.ok[i] != 1) return;
  const size_t cell = (size_t)b.set[i] * fs.n_vals + b.val[i];
  if (fs.acc[cell] == 0) atomicMin(&fs.cand[cell], i);
}

__device__ __forceinline__ bool sig_eq_words(const FlowBatch& b, uint32_t i, const uint32_t* q) {
  uint32_t d = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) d |= b.sig[(size_t)j * b.n_pad + i] ^ q[j];
  return d == 0;
}
__device__ __forceinline__ bool sig_eq_votes(const FlowBatch& b, uint32_t i, uint32_t f) {
  uint32_t d = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) d |= b.sig[(size_t)j * b.n_pad + i] ^ b.sig[(size_t)j * b.n_pad + f];
  return d == 0;
}

__global__ void __launch_bounds__(256) txv_k_tally_resolve(FlowState fs, FlowBatch b) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= b.n || !pending_in_set(b, i)) return;
  const uint32_t s = b.set[i], v = b.val[i];
  const uint8_t fl = b.flags[i];
  const bool sig64 = (fl & TXV_FLAG_SIG64) != 0;
  const size_t cell = (size_t)s * fs.n_vals + v;
  const uint32_t acc = fs.acc[cell];
  uint8_t st;
  if (acc) {                                   // accepted in an earlier batch (vote_set.go:109-114)
    st = sig64 && sig_eq_words(b, i, fs.arena[acc - 1].sig) ? TXV_S_DUPLICATE : TXV_S_NONDETERMINISTIC;
  } else {
    const uint32_t f = fs.cand[cell];
    if (f == i) {                              // ADDED: the reference stores the vote (vote_set.go:154)
      st = TXV_S_ADDED;
      const uint32_t r = atomicAdd(&fs.ctr->arena_used, 1u);
      if (r < fs.max_accepted) {
        AccRow* row = fs.arena + r;
#pragma unroll
        for (int j = 0; j < 16; ++j) row->sig[j] = b.sig[(size_t)j * b.n_pad + i];
        row->height = b.height[i];
        row->ts_sec = b.ts_sec[i];
        row->ts_nanos = b.ts_nanos[i];
        row->val = v;
        row->seq = b.seq_base + i;
        if (b.txkey) {
          const uint4* s4 = reinterpret_cast<const uint4*>(b.txkey + (size_t)i * 32);
          const uint4 a = s4[0], c = s4[1];
          row->txkey[0] = a.x; row->txkey[1] = a.y; row->txkey[2] = a.z; row->txkey[3] = a.w;
          row->txkey[4] = c.x; row->txkey[5] = c.y; row->txkey[6] = c.z; row->txkey[7] = c.w;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) row->txkey[j] = 0;
        }
        b.row[i] = r;
      } else {
        atomicOr(&fs.ctr->err, TXV_FERR_ARENA);
        b.row[i] = TXV_NONE;
      }
    } else if (f < i) {                        // an earlier vote of the batch was accepted
      st = sig64 && sig_eq_votes(b, i, f) ? TXV_S_DUPLICATE : TXV_S_NONDETERMINISTIC;
    } else {                                   // no accepted vote before it and it did not verify
      st = (fl & TXV_FLAG_BADMSG) ? TXV_S_SIGNBYTES : TXV_S_INVALID_SIGNATURE;
    }
  }
  b.status[i] = st;
}

// list the ADDED votes of each set in its cell row (at most one per validator)
__global__ void __launch_bounds__(256) txv_k_tally_bucket(FlowState fs, FlowBatch b) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= b.n || !pending_in_set(b, i) || b.status[i] != TXV_S_ADDED) return;
  const uint32_t s = b.set[i];
  const uint32_t k = atomicAdd(&fs.set_cnt[s], 1u);
  fs.cand[(size_t)s * fs.n_vals + k] = i;
  if (k == 0) fs.touched[atomicAdd(&fs.ctr->n_touched, 1u)] = s;
}

__device__ __forceinline__ int64_t wave_sum64(int64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

constexpr uint32_t kListCap = 512;   // ADDED votes of a set kept in LDS (every set of a <= 512-validator registry)

// one wave per set with ADDED votes (persistent waves over the device-side touched count)
__global__ void __launch_bounds__(256) txv_k_tally_cross(FlowState fs, FlowBatch b) {
  __shared__ uint32_t l_vote[4][kListCap];
  __shared__ int64_t l_pow[4][kListCap];
  const int lane = threadIdx.x & 63;
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t n_touched = fs.ctr->n_touched;
  const uint32_t n_waves = gridDim.x * 4;
  for (uint32_t t = blockIdx.x * 4 + wv; t < n_touched; t += n_waves) {
    const uint32_t s = fs.touched[t];
    const uint32_t k = fs.set_cnt[s];
    const uint32_t* list = fs.cand + (size_t)s * fs.n_vals;
    const bool in_lds = k <= kListCap;
    int64_t part = 0;
    for (uint32_t c = lane; c < k; c += 64) {
      const uint32_t ie = list[c];
      const int64_t pw = fs.power[b.val[ie]];
      part += pw;
      if (in_lds) { l_vote[wv][c] = ie; l_pow[wv][c] = pw; }
    }
    __threadfence_block();
    const int64_t prior = fs.set_sum[s];
    const int64_t total = prior + wave_sum64(part);
    uint32_t cross = TXV_NO_CROSS;
    if (prior >= fs.quorum) {
      cross = 0;                                // already committed: every ADDED vote re-fires
    } else if (total >= fs.quorum) {
      // crossing = the arrival index T at which the stake prefix (in arrival order) first reaches
      // quorum: with g(t) = stake of listed votes with arrival < t (monotone), T is the largest t
      // with prior + g(t) < quorum, found bit by bit; each probe is one list pass + a wave sum
      const int64_t need = fs.quorum - prior;
      uint32_t T = 0;
      for (int bit = 31 - __builtin_clz(max(b.n, 2u) - 1u); bit >= 0; --bit) {
        const uint32_t cand = T | (1u << bit);
        int64_t sm = 0;
        if (in_lds) {
          for (uint32_t c = lane; c < k; c += 64)
            if (l_vote[wv][c] < cand) sm += l_pow[wv][c];
        } else {
          for (uint32_t c = lane; c < k; c += 64) {
            const uint32_t ie = list[c];
            if (ie < cand) sm += fs.power[b.val[ie]];
          }
        }
        if (wave_sum64(sm) < need) T = cand;
      }
      cross = T;
    }
    for (uint32_t c = lane; c < k; c += 64) {
      const uint32_t ie = in_lds ? l_vote[wv][c] : list[c];
      const bool fire = cross != TXV_NO_CROSS && ie >= cross;
      b.status[ie] = (uint8_t)(TXV_S_ADDED | (fire ? TXV_S_FIRED : 0u));
      const uint32_t r = b.row[ie];
      fs.acc[(size_t)s * fs.n_vals + b.val[ie]] = r == TXV_NONE ? 0u : r + 1u;
    }
    if (lane == 0) {
      fs.set_sum[s] = total;
      fs.set_cnt[s] = 0;
      if (total >= fs.quorum) atomicOr(&fs.bitmap[s >> 5], 1u << (s & 31));
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

// final statuses into mapped host memory (coalesced), then the batch summary
__global__ void __launch_bounds__(256) txv_k_status_out(FlowState fs, FlowBatch b, uint32_t nb) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < b.n) {
    const uint8_t p = b.pre[i];
    b.status_host[i] = p == TXV_S_PENDING ? (b.set[i] == TXV_NONE ? (uint8_t)TXV_S_INVALID_SIGNATURE : b.status[i]) : p;
  }
  if (i == 0) {
    FlowSummary s;
    s.n_sets = fs.ctr->n_sets;
    s.n_events = b.blk[nb];
    s.arena_used = fs.ctr->arena_used;
    s.err = fs.ctr->err;
    s.key_used = fs.ctr->key_used;
    *b.summary_host = s;
  }
}

// ------------------------------------------------------------------ reset / readers
__global__ void __launch_bounds__(256) txv_k_reset_sets(FlowState fs, int keep_ids) {
  const uint32_t ns = fs.ctr->n_sets;
  const uint64_t cells = (uint64_t)ns * fs.n_vals;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < cells; c += stride) fs.acc[c] = 0;
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < ns; s += stride) {
    fs.set_sum[s] = 0;
    fs.set_cnt[s] = 0;
    if (!keep_ids) {
      SetEntry& e = fs.tab[fs.set_entry[s]];
      e.h = 0; e.len = 0; e.key_off = 0; e.first = 0; e.id = 0; e.state = TXV_SE_EMPTY;
    }
  }
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < ((uint64_t)ns + 31) / 32; w += stride) fs.bitmap[w] = 0;
}

__global__ void txv_k_reset_counters(FlowState fs, int keep_ids) {
  if (!keep_ids) {
    fs.ctr->n_sets = 0;
    fs.ctr->key_used = 0;
    fs.ctr->err = 0;
  } else {
    fs.ctr->err &= ~TXV_FERR_ARENA;
  }
  fs.ctr->arena_used = 0;
  fs.ctr->n_touched = 0;
  fs.ctr->batch = 0;
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
    if (e.state == TXV_SE_KEPT && e.h == h && e.len == l && key_eq(fs.keys + e.key_off, kp, l)) {
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
  AccRow r;
  const uint32_t a = ok ? fs.acc[(size_t)id * fs.n_vals + v] : 0u;
  if (a) {
    r = fs.arena[a - 1];
  } else {
    r = AccRow{};
    r.val = TXV_NONE;
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
  out_off[q] = e.key_off;
  out_len[q] = e.len;
}

__global__ void __launch_bounds__(256) txv_k_pack(FlowState fs, uint32_t* dst, uint32_t bm_words, uint32_t n_cap) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  const uint32_t ns = min(fs.ctr->n_sets, n_cap);
  if (t == 0) { dst[0] = ns; dst[1] = 0; }
  if (t < bm_words) dst[2 + t] = (t * 32 < ns) ? fs.bitmap[t] & (t * 32 + 32 <= ns ? ~0u : ((1u << (ns & 31)) - 1u)) : 0u;
  if (t < n_cap) {
    const int64_t sm = t < ns ? fs.set_sum[t] : 0;
    dst[2 + bm_words + 2 * t] = (uint32_t)(uint64_t)sm;
    dst[2 + bm_words + 2 * t + 1] = (uint32_t)((uint64_t)sm >> 32);
  }
}

template <class Pred, class Act>
hipError_t compact(Pred p, Act act, uint32_t n, uint32_t* blk, hipStream_t st) {
  const uint32_t nb = (n + kScanItems - 1) / kScanItems;
  if (nb) hipLaunchKernelGGL((txv_k_scan_count<Pred>), dim3(nb), dim3(256), 0, st, p, n, blk);
  hipLaunchKernelGGL(txv_k_scan_top, dim3(1), dim3(1024), 0, st, blk, nb);
  if (nb) hipLaunchKernelGGL((txv_k_scan_apply<Pred, Act>), dim3(nb), dim3(256), 0, st, p, act, n, blk);
  return hipGetLastError();
}

}  // namespace

extern "C" {

hipError_t txv_flow_route(const FlowState* fs, const FlowBatch* b, hipStream_t st) {
  if (((uint64_t)b->n + kScanItems - 1) / kScanItems > 8192) return hipErrorInvalidValue;
  const uint32_t nb = (b->n + kScanItems - 1) / kScanItems;
  const uint32_t g = (b->n + 255) / 256;
  if (g) hipLaunchKernelGGL(txv_k_route, dim3(g), dim3(256), 0, st, *fs, *b);
  hipError_t e = compact(NewSetPred{*fs, *b}, NewSetAct{*fs, *b}, b->n, b->blk, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(txv_k_set_ids, dim3(g ? g : 1), dim3(256), 0, st, *fs, *b, nb);
  return hipGetLastError();
}

hipError_t txv_flow_tally(const FlowState* fs, const FlowBatch* b, hipStream_t st) {
  const uint32_t nb = (b->n + kScanItems - 1) / kScanItems;
  const uint32_t g = (b->n + 255) / 256;
  if (g) {
    hipLaunchKernelGGL(txv_k_tally_min, dim3(g), dim3(256), 0, st, *fs, *b);
    hipLaunchKernelGGL(txv_k_tally_resolve, dim3(g), dim3(256), 0, st, *fs, *b);
    hipLaunchKernelGGL(txv_k_tally_bucket, dim3(g), dim3(256), 0, st, *fs, *b);
    // persistent waves: enough to cover every set of a C2-sized batch in one round
    const uint32_t sets_max = std::min<uint32_t>(b->n, fs->max_txs);
    const uint32_t cross_blocks = std::max<uint32_t>(1, std::min<uint32_t>((sets_max + 3) / 4, 4096));
    hipLaunchKernelGGL(txv_k_tally_cross, dim3(cross_blocks), dim3(256), 0, st, *fs, *b);
  }
  hipError_t e = compact(EventPred{*b}, EventAct{*fs, *b}, b->n, b->blk, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(txv_k_status_out, dim3(g ? g : 1), dim3(256), 0, st, *fs, *b, nb);
  return hipGetLastError();
}

hipError_t txv_flow_reset(const FlowState* fs, int keep_ids, hipStream_t st) {
  hipLaunchKernelGGL(txv_k_reset_sets, dim3(1024), dim3(256), 0, st, *fs, keep_ids);
  hipLaunchKernelGGL(txv_k_reset_counters, dim3(1), dim3(1), 0, st, *fs, keep_ids);
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
  hipLaunchKernelGGL(txv_k_pack, dim3((t + 255) / 256), dim3(256), 0, st, *fs, dst, bm_words, n_cap);
  return hipGetLastError();
}

}  // extern "C"
