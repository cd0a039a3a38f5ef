// pool_dev.h — TxVotePool CheckTx decisions on the GPU (kernels_pool.hip), shared by the kernels
// and the host engine (runtime.cpp).
//
// One batch of CheckTxWithInfo calls (txvotepool/txvotepool.go:187-261) decided in parallel by
// LRU stack distance, the same formulation as pool.cpp's batch_check, with the cache
// (mapTxCache, :416-438) held in HBM: a key array in recency order (front = least recent) and an
// open-addressing index over it, double-buffered (the batch reads buffer `old`, writes `new`).
// Preconditions the host checks before enqueueing (else pool.cpp's host path runs): the pool's
// Size / MaxTxsBytes caps cannot bind inside the batch, and every vote's key is on the device.
#pragma once
#include <stdint.h>

// The pool list (txs + txsMap, txvotepool.go:265-270 / :339-344) in HBM: entries in insertion
// order at positions [0, tail) -- key [8] words, TxVote.Size(), alive flag -- and an
// open-addressing index over them (u64 slots: tag << 32 | position + 1; 0 empty, low word
// kListTomb a removed entry).  A list position is never reused before a compaction, so the list
// order is the reference's clist order: appends at the tail, removals leave a dead entry behind.
constexpr uint32_t kListTomb = 0xFFFFFFFFu;
struct PoolListArgs {
  uint32_t* lk;               // [cap][8] entry keys
  uint32_t* lsz;              // [cap] entry Size()
  uint8_t* lfl;               // [cap] 1 = alive
  unsigned long long* li;     // [icap] index slots
  uint32_t imask;             // icap - 1
  uint64_t seed;              // the engine's secret hash seed (list_home)
  const uint32_t* tail_in;    // the tail before the batch
  uint32_t* tail_out;         // the tail after it (the other word of the pair)
};

struct PoolDevArgs {
  uint32_t n;                 // votes in the batch (arrival order)
  const uint32_t* keys;       // [n][8] key words (SHA-256(Signature) bytes in memory order)
  const uint32_t* sizes;      // [n] TxVote.Size()
  const uint8_t* valid;       // [n - n_force] or null: valid[i - n_force] != valid_ok = the message did not
                              // decode (no CheckTx, status NOT_CHECKED)
  uint32_t valid_ok;          // the value of valid[] that means "decoded"
  int64_t max_tx;             // a vote is pushed to the cache iff Size() <= max_tx (MaxMsgBytes - 8)
  uint32_t C;                 // cache capacity (config.CacheSize); 0 = nopTxCache
  uint32_t wal;               // a WAL is configured: Size() == 0 -> ErrEncoding after the push
  // the cache: keys [C][8] and index [icap] (slot = position + 1, 0 empty), old -> new
  const uint32_t* ck_old;
  uint32_t* ck_new;
  const uint32_t* ci_old;
  uint32_t* ci_new;
  uint32_t icap;              // power of two >= 2 C
  uint32_t* clen;             // [1] cache length: L0 read, the new length written at the end
  // scratch (n entries unless noted)
  uint32_t* push;             // 1 = reaches cache.Push
  uint32_t* aidx;             // exclusive scan of push: the push's index in S after the L0 cache entries
  uint32_t* hkey;             // sort keys (a 24-bit slice of the key's seeded hash; non-pushes 0xFFFFFF)
  uint32_t* hidx;             // 0..n-1
  uint32_t* skey;             // sorted
  uint32_t* sidx;
  uint32_t* last;             // 1 = the last push of its key in the batch
  uint32_t* lpos;             // exclusive scan of last
  uint8_t* dec;               // 0 not pushed, 1 miss, 2 hit, 3 far (decided by the nested-pair count)
  uint64_t* pst;              // pair (previous occurrence, this push) in doubled S positions, when evicting
  uint64_t* pend;
  uint32_t* far;              // [n] far pushes
  uint32_t* nfar;             // [1] far pushes
  uint32_t* xs;               // [ceil(n / 1024) * 1024] per block of 1024 votes: its pairs' starts, sorted
  uint32_t* xn;               // [ceil(n / 1024)] pairs per block
  uint8_t* detached;          // [C] cached keys pushed again in this batch (cleared at the end)
  uint32_t* surv;             // [C] old entries not pushed again
  uint32_t* spos;             // [C] exclusive scan of surv
  uint64_t* tiles;            // look-back words: [ceil(n/1024)] push, [ceil(n/1024)] last, [ceil(C/1024)] surv,
                              // [ceil(n/1024)] appends
  uint32_t* tk;               // [4] tile tickets (pd_init, pd_status n-chain, pd_status C-chain)
  uint32_t epoch;             // this batch's tag for the look-back words (30 bits)
  uint64_t seed;              // the engine's secret hash seed (sort slice, cache index: kernels_pool.hip)
  uint32_t* err;              // [1] sticky: 1 = a look-back scan timed out (a broken invariant)
  uint32_t* err_host;         // [1] mapped: *err copied there by the chain's last launch
  uint32_t* okpos;            // [n] exclusive scan of the appended votes (list_on)
  uint64_t* res;              // (list_on) per 1024-vote tile (appended entries, their Size() sum), mapped
  uint64_t* res_rm;           // (list_on) per 1024-vote tile of [0, n_force): (removed entries, bytes), mapped
  // Update's committed votes fused into the batch: entries [0, n_force) push unconditionally, get
  // no status, and leave the pool list before the batch's own votes (entries [n_force, n)) are
  // appended (the reference's order: Update, then the CheckTx calls after it)
  uint32_t n_force;
  uint32_t list_on;           // the pool list is held in HBM: removals, appends (l)
  PoolListArgs l;
  void* tmp;                  // hipcub temporary storage
  size_t tmp_bytes;
  uint8_t* status;            // [n] out: TXV_POOL_* per vote
  uint8_t* status_out;        // [n - n_force] the batch's own statuses again, in mapped host memory
  uint8_t* status_copy;       // [n - n_force] and once more in HBM for a consumer's kernels, or null
};

