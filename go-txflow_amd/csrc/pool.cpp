// pool.cpp — TxVotePool (txvotepool/txvotepool.go) behind include/txvote.h.
//
// A batch of CheckTx calls is split the MI355X way: the per-vote work that is independent of
// order -- txVoteKey = SHA-256(Signature) (:467-469) on the GPU (txv_sig_keys), TxVote.Size
// (types/tx_vote.go:144-150) on the host threads -- runs for the whole batch first; then the
// order-dependent part runs sequentially in arrival order exactly as CheckTxWithInfo does it
// per vote (:187-261):
//   0. txSize = TxVote.Size(), which is 0 when amino rejects the timestamp (types/tx_vote.go:144-150):
//      such a vote goes through every step below with size 0 -- it is cached and admitted --
//      unless a WAL is configured (TXV_POOL_WAL): then MustMarshalBinaryBare panics in the WAL
//      write (:231-242) right after the cache push, reported as TXV_POOL_ERR_ENCODING
//   1. Size() >= config.Size || txSize + TxsBytes() > config.MaxTxsBytes -> ErrMempoolIsFull
//   2. txSize > MaxMsgBytes - aminoOverheadForTxMessage (8, reactor.go:27,379) -> ErrTxTooLarge
//   3. cache.Push(key) false (key present: moved to the back) -> ErrTxInCache
//      (mapTxCache.Push :416-438: evicts the front when full; nopTxCache when CacheSize == 0)
//   4. addTx (:265-270): txs.PushBack, txsMap[key] = element, txsBytes += Size()
// Update (:329-359) pushes every committed key to the cache and removes the pool element
// txsMap[key] (removeTx :275-284, which subtracts the *committed* vote's Size()).
// Sender bookkeeping (MempoolTxVote.Senders), the WAL and metrics carry no verdicts and are
// not restated.
#include "../../include/txvote.h"
#include "amino.hpp"
#include "txv_hash.h"
#include <random>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <cstdlib>
#include <cstring>
#include <sys/mman.h>
#include <functional>
#include <memory>
#include <mutex>
#include <system_error>
#include <thread>
#include <algorithm>
#include <atomic>
#include <new>
#include <vector>

namespace {

struct Key {
  uint8_t b[32];
  bool operator==(const Key& o) const { return memcmp(b, o.b, 32) == 0; }
};
// Keys are SHA-256 of peer-supplied signature bytes that CheckTx never verifies
// (txvotepool.go:467-469): a peer can grind signatures until their keys share any fixed slice, so
// the host tables place keys by txv_hash::key32 under a secret per-process seed (an unseeded slice
// let one peer's ground keys pile onto one home slot: every probe of a batch walks the cluster).
uint64_t make_key_seed() {
  return ((uint64_t)std::random_device{}() << 32 | std::random_device{}()) ^ 0x686f73746b657973ULL;
}
const uint64_t g_key_seed = make_key_seed();   // drawn once per process, at load
inline uint64_t key_hash(const Key& k, uint64_t salt) {
  uint32_t w[8];
  memcpy(w, k.b, 32);
  return txv_hash::key32(w, g_key_seed ^ salt);
}

// open-addressing index Key -> node of a KeyList (linear probing, backward-shift deletion, no
// tombstones).  A slot is 8 bytes (32-bit hash tag + node index; the key itself is compared in
// the list node), and the table sits on transparent huge pages: the CheckTx loop is bound by
// one random access per map per vote, so TLB reach and slot size decide its speed.
struct KeyList;
struct FlatIndex {
  struct Slot { uint32_t tag; int32_t idx; };     // tag 0 = empty
  Slot* t = nullptr;
  size_t cap = 0, mask = 0, n = 0;
  uint32_t shift = 32;                            // home slot = Fibonacci hash of the tag's 32 bits
  const KeyList* owner = nullptr;
  explicit FlatIndex(const KeyList* o) : owner(o) { alloc(1024); }
  ~FlatIndex() { free(t); }
  FlatIndex(const FlatIndex&) = delete;
  FlatIndex& operator=(const FlatIndex&) = delete;
  static uint64_t h(const Key& k) { return key_hash(k, 0); }
  static uint32_t tag(uint64_t hv) { return (uint32_t)(hv >> 32) | 1u; }
  // the home slot from the stored tag alone (the high bits of its Fibonacci hash: the partition
  // bits PartIndex takes from the same word are mixed in), so the backward-shift erase and the
  // rehash never read a node's key
  size_t home(uint32_t tg) const { return (size_t)((uint32_t)(tg * 0x9E3779B1u) >> shift); }
  void alloc(size_t c) {
    const size_t bytes = c * sizeof(Slot);
    const size_t align = bytes >= (2u << 20) ? (2u << 20) : 64;
    t = (Slot*)aligned_alloc(align, (bytes + align - 1) / align * align);
#ifdef MADV_HUGEPAGE
    if (align == (2u << 20)) madvise(t, bytes, MADV_HUGEPAGE);
#endif
    memset(t, 0, bytes);
    cap = c; mask = c - 1; n = 0;
    shift = 32;
    for (size_t x = c; x > 1; x >>= 1) --shift;
  }
  inline const Key& key_of(int32_t idx) const;
  void prefetch(const Key& k) const { __builtin_prefetch(&t[home(tag(h(k)))]); }
  int32_t find(const Key& k) const {
    const uint32_t tg = tag(h(k));
    for (size_t i = home(tg); t[i].tag; i = (i + 1) & mask)
      if (t[i].tag == tg && key_of(t[i].idx) == k) return t[i].idx;
    return -1;
  }
  // one probe for "find, else insert": returns the existing index, or -1 after the caller's
  // make_idx() result was inserted (capacity is ensured before probing)
  template <typename F>
  int32_t find_or_insert(const Key& k, F&& make_idx) {
    if ((n + 1) * 2 > cap) grow();
    const uint32_t tg = tag(h(k));
    size_t i = home(tg);
    for (; t[i].tag; i = (i + 1) & mask)
      if (t[i].tag == tg && key_of(t[i].idx) == k) return t[i].idx;
    t[i] = Slot{tg, make_idx()};
    ++n;
    return -1;
  }
  void put(const Key& k, int32_t idx) {    // insert or overwrite
    if ((n + 1) * 2 > cap) grow();
    const uint32_t tg = tag(h(k));
    size_t i = home(tg);
    for (; t[i].tag; i = (i + 1) & mask)
      if (t[i].tag == tg && key_of(t[i].idx) == k) { t[i].idx = idx; return; }
    t[i] = Slot{tg, idx};
    ++n;
  }
  // remove the key and return its index (-1: absent); one probe
  int32_t take(const Key& k) {
    const uint32_t tg = tag(h(k));
    size_t i = home(tg);
    for (; t[i].tag; i = (i + 1) & mask)
      if (t[i].tag == tg && key_of(t[i].idx) == k) break;
    if (!t[i].tag) return -1;
    const int32_t idx = t[i].idx;
    size_t j = i;
    for (;;) {   // backward shift: entry j moves into hole i iff i lies cyclically in [home(j), j)
      j = (j + 1) & mask;
      if (!t[j].tag) break;
      const size_t hj = home(t[j].tag);
      if (((j - hj) & mask) >= ((j - i) & mask)) { t[i] = t[j]; i = j; }
    }
    t[i].tag = 0;
    --n;
    return idx;
  }
  bool erase(const Key& k) { return take(k) >= 0; }
  void clear() { memset(t, 0, cap * sizeof(Slot)); n = 0; }   // keeps the capacity
  void reserve(size_t m) { if (m * 2 > cap) { size_t c = cap; while (m * 2 > c) c *= 2; rehash(c); } }
  void grow() { rehash(cap * 2); }
  void rehash(size_t c) {
    Slot* old = t;
    const size_t oc = cap;
    alloc(c);
    for (size_t i = 0; i < oc; ++i)
      if (old[i].tag) {
        size_t j = home(old[i].tag);
        while (t[j].tag) j = (j + 1) & mask;
        t[j] = old[i];
        ++n;
      }
    free(old);
  }
};

// TXV_PROFILE_HOST=1: per-call phase times of the pool's calls on stderr ("[txv pool] <what> a=.. b=..")
struct PTimer {
  bool on;
  std::chrono::steady_clock::time_point t;
  std::string line;
  explicit PTimer(const char* what) : on(getenv("TXV_PROFILE_HOST") != nullptr), t(std::chrono::steady_clock::now()) {
    if (on) {   // the start on the monotonic clock (Python's time.perf_counter), for traces
      char b[48];
      snprintf(b, sizeof b, " @%.4f", std::chrono::duration<double>(t.time_since_epoch()).count());
      line = std::string(what) + b;
    }
  }
  void mark(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    char b[64];
    snprintf(b, sizeof b, " %s=%.3f", what, std::chrono::duration<double, std::milli>(now - t).count());
    line += b;
    t = now;
  }
  ~PTimer() { if (on) fprintf(stderr, "[txv pool] %s\n", line.c_str()); }
};

// doubly linked list in a vector (stable indices)
struct KeyList {
  struct Node {
    Key k; uint32_t size; int32_t prev, next;
    Node() {}   // left unset: a batch grows the array by 64k nodes whose every field is written after
    Node(const Key& k_, uint32_t s, int32_t p, int32_t n) : k(k_), size(s), prev(p), next(n) {}
  };
  std::vector<Node> nodes;
  std::vector<int32_t> free_;
  int32_t head = -1, tail = -1;
  size_t len = 0;
  int32_t push_back(const Key& k, uint32_t size) {
    int32_t i;
    if (!free_.empty()) { i = free_.back(); free_.pop_back(); }
    else { i = (int32_t)nodes.size(); nodes.push_back(Node{}); }
    nodes[i] = Node{k, size, tail, -1};
    if (tail >= 0) nodes[tail].next = i; else head = i;
    tail = i;
    ++len;
    return i;
  }
  void unlink(int32_t i) {
    Node& n = nodes[i];
    if (n.prev >= 0) nodes[n.prev].next = n.next; else head = n.next;
    if (n.next >= 0) nodes[n.next].prev = n.prev; else tail = n.prev;
    free_.push_back(i);
    --len;
  }
  void detach(int32_t i) {                        // unlink without freeing the node
    Node& n = nodes[i];
    if (n.prev >= 0) nodes[n.prev].next = n.next; else head = n.next;
    if (n.next >= 0) nodes[n.next].prev = n.prev; else tail = n.prev;
    --len;
  }
  void append_linked(const std::vector<int32_t>& idx) {   // detached / fresh nodes, in order
    for (int32_t i : idx) {
      nodes[i].prev = tail;
      nodes[i].next = -1;
      if (tail >= 0) nodes[tail].next = i; else head = i;
      tail = i;
    }
    len += idx.size();
  }
  void move_to_back(int32_t i) {
    if (i == tail) return;
    Node& n = nodes[i];
    if (n.prev >= 0) nodes[n.prev].next = n.next; else head = n.next;
    nodes[n.next].prev = n.prev;
    n.prev = tail; n.next = -1;
    nodes[tail].next = i;
    tail = i;
  }
  void clear() { nodes.clear(); free_.clear(); head = tail = -1; len = 0; }
};

inline const Key& FlatIndex::key_of(int32_t idx) const { return owner->nodes[idx].k; }

// kParts independent FlatIndex tables, chosen by hash bits the in-table slot does not use: the
// same sequential API, and a batch can be inserted by several threads, each owning whole
// partitions (txv_pool_check's fast path)
constexpr uint32_t kParts = 16;
struct PartIndex {
  std::vector<std::unique_ptr<FlatIndex>> p;
  explicit PartIndex(const KeyList* o) {
    for (uint32_t i = 0; i < kParts; ++i) p.emplace_back(new FlatIndex(o));
  }
  static uint32_t part(const Key& k) { return (uint32_t)(FlatIndex::h(k) >> 40) & (kParts - 1); }
  FlatIndex& of(const Key& k) { return *p[part(k)]; }
  const FlatIndex& of(const Key& k) const { return *p[part(k)]; }
  void prefetch(const Key& k) const { of(k).prefetch(k); }
  int32_t find(const Key& k) const { return of(k).find(k); }
  template <typename F>
  int32_t find_or_insert(const Key& k, F&& make_idx) { return of(k).find_or_insert(k, make_idx); }
  void put(const Key& k, int32_t idx) { of(k).put(k, idx); }
  bool erase(const Key& k) { return of(k).erase(k); }
  void clear() { for (auto& f : p) f->clear(); }
  void reserve(size_t m) { for (auto& f : p) f->reserve(m / kParts + m / (4 * kParts) + 64); }
};

// batch_check's per-call arrays, kept across calls.  Per-vote arrays are indexed by arrival
// index i; per-partition ones by position j in the partition order (order[j] = i, pos[i] = j), so
// the threads of the per-partition passes write disjoint contiguous ranges
struct BatchScratch {
  std::vector<uint32_t> cnt, order, pos, aidx, hist;
  std::vector<int32_t> prevj, nextj, firstj, cnodej, qpos, adm;
  std::vector<uint8_t> decj, dec;           // 0 not a push (too large), 1 miss, 2 hit, 3 far
  std::vector<int32_t> qtouched;
  // per partition, filled by the scan: pairs (start, next occurrence) of consecutive pushes of one
  // key in doubled S positions (only while evicting), distinct keys pushed, cached keys pushed
  std::vector<std::pair<uint64_t, uint64_t>> pairs[16];
  uint32_t firsts[16];
  std::vector<int32_t> cached_firsts[16];
  std::vector<uint8_t> dmark;               // per cache node: pushed again by this batch
};

}  // namespace

// runtime.cpp: the device cache engine (TXV_POOL_DEVICE_CACHE)
struct PoolDev;
void pooldev_free(PoolDev* s);
bool pooldev_same_device(const txv_ctx* c, const PoolDev* s);
uint32_t pooldev_cap(const PoolDev* s);
int pooldev_bind(txv_ctx* c, PoolDev** sp, uint32_t C, uint32_t n);
int pooldev_put_cache(txv_ctx* c, PoolDev* s, const uint8_t* keys, uint32_t L);
int pooldev_get_cache(txv_ctx* c, PoolDev* s, std::vector<uint8_t>& keys);
int pooldev_check(txv_ctx* c, PoolDev* s, const txv_votes* v, const uint8_t* h_keys_in, const uint32_t* h_sizes,
                  const uint32_t* d_keys, const uint32_t* d_sizes, const uint8_t* d_valid, uint32_t valid_ok, uint32_t n,
                  int64_t max_tx, bool wal, uint8_t* keys_out, uint8_t* status_out, void* after, bool list_on,
                  uint64_t live_ub, int slot, uint32_t n_upd);
int pooldev_enqueue(txv_ctx* c, PoolDev* s, int slot, const txv_votes* v, const uint8_t* h_keys_in,
                    const uint32_t* h_sizes, const uint32_t* d_keys, const uint32_t* d_sizes, const uint8_t* d_valid,
                    uint32_t valid_ok, uint32_t n, int64_t max_tx, bool wal, bool keys_back, void* after_ev,
                    bool list_on, uint64_t live_ub, uint32_t n_upd, uint8_t* d_status_copy = nullptr,
                    void* then_stream = nullptr);
int pooldev_stage(txv_ctx* c, PoolDev* s, int slot, uint32_t off, const txv_votes* v, const uint32_t* h_sizes);
void pooldev_list_hint(PoolDev* s, uint64_t entries);
int pooldev_finish(txv_ctx* c, PoolDev* s, int slot, const uint8_t** status, const uint8_t** keys, const uint32_t** sizes);
int pooldev_list_put(txv_ctx* c, PoolDev* s, const uint8_t* keys, const uint32_t* sizes, const uint8_t* ins, uint32_t L);
int pooldev_list_get(txv_ctx* c, PoolDev* s, std::vector<uint8_t>& keys, std::vector<uint32_t>& sizes,
                     std::vector<uint8_t>& ins);
void pooldev_result(const PoolDev* s, int slot, int64_t res[4]);
constexpr int kPdRing = 8;   // = PoolDev::kPdRing (runtime.cpp)
void pooldev_set_occupant(PoolDev* s, int slot, uint64_t id, uint32_t n_upd, uint32_t n);
bool pooldev_holds(const PoolDev* s, uint64_t id);
std::mutex& txv_ctx_submit_mu(txv_ctx* c);
std::mutex& txv_ctx_route_mu(txv_ctx* c);
int txv_ctx_fail(txv_ctx* c, int code, const char* msg);
int route_checked_stage(txv_ctx* c, const txv_votes* v, uint64_t stride);
int route_checked_consume(txv_ctx* c, PoolDev* dev, uint64_t pool_ticket, uint32_t n);
int route_checked_launch(txv_ctx* c, const txv_votes* v, const uint8_t* host_st, uint32_t G, void* dst, uint64_t stride,
                         txv_route_meta* meta);
int submit_checked_stage(txv_ctx* c, const txv_votes* v, uint32_t* slot_out);
int submit_checked_consume(txv_ctx* c, uint32_t slot, PoolDev* dev, uint64_t pool_ticket, const txv_votes* v);
int submit_checked_run(txv_ctx* c, uint32_t slot, const txv_votes* v, const uint8_t* host_st, int why, uint64_t* ticket);

struct txv_pool {
  txv_pool_config cfg{};
  bool cache_on = true;
  int64_t height = 0;
  std::mutex mu;                                   // proxyMtx
  KeyList cache;                                   // mapTxCache.list
  PartIndex cache_map{&cache};                     // mapTxCache.map_
  KeyList txs;                                     // txs (clist of MempoolTxVote)
  PartIndex txs_map{&txs};                         // txsMap
  int64_t txs_bytes = 0;
  std::vector<uint8_t> keys;                       // batch scratch
  std::vector<uint32_t> sizes;                     // batch scratch: TxVote.Size() per vote
  std::vector<int32_t> idx_c, idx_t;               // batch scratch: node indices (fast path)
  std::vector<uint8_t> part;                       // batch scratch: index partition per key (batch path)
  BatchScratch bs;                                 // batch scratch (batch path)
  std::shared_ptr<void> workers;                   // batch passes of calls without a context
  // TXV_POOL_DEVICE_CACHE: the cache's copy in HBM (runtime.cpp's PoolDev) and which copy is current
  PoolDev* dev = nullptr;
  enum { kSynced, kDevAhead, kHostAhead } dev_state = kHostAhead;
  // ... and the pool list (txs + txsMap) too: a device batch appends its admitted votes there and
  // a device Update removes its committed ones (runtime.cpp's list kernels), so while list_dev the
  // host's txs / txs_map are stale -- a host reader or writer brings the list back first
  // (list_to_host), the next device batch takes it up again (list_to_dev).  txs.len and txs_bytes
  // stay current either way: they follow each finished device batch's counts.
  bool list_dev = false;
  // Size() / TxsBytes() as published after every change (the reference's atomics, read without
  // proxyMtx): txs.len / txs_bytes themselves are written under mu, so a reader not holding it
  // must not touch them
  std::atomic<int64_t> pub_len{0}, pub_bytes{0};
  std::vector<uint8_t> rm_flag;                    // remove_keys scratch: per pool-list node
  std::vector<uint8_t> rm_part;                    // ... per key: its txsMap partition
  std::vector<uint32_t> rm_order;                  // ... the keys by partition
  std::vector<int32_t> rm_all;                     // ... the nodes removed
  // engines replaced while a waiter (txv_pool_check_wait, outside mu) may still sync on one of
  // their flight events: freed when the last waiter is done
  int waiters = 0;
  std::vector<PoolDev*> retired;
  // device batches submitted (txv_pool_check_submit) and not yet waited, in order; a device one
  // holds flight slot `slot` of the engine until finished (its statuses then kept in st).
  // infl_*: the pushes / Size() sums of the unfinished ones (upper bounds for the caps check)
  struct Ticket {
    uint64_t id = 0;
    uint32_t n = 0;
    int slot = -1;
    bool done = false;
    txv_ctx* ctx = nullptr;
    uint64_t pushes = 0, bytes = 0;
    std::vector<uint8_t> st;
    int err = 0;
    // an Update batch (txv_pool_update_submit) run alone: its keys pushed and its votes removed
    // from the pool list by the engine in submission order; no caller waits for it.  (Usually an
    // Update rides with the next CheckTx batch instead: n_upd entries staged ahead of its votes.)
    bool upd = false;
    uint32_t n_upd = 0;
  };
  std::deque<Ticket> tickets;
  // the statuses of the last tickets waited (txv_submit_checked may come after the wait)
  std::deque<std::pair<uint64_t, std::vector<uint8_t>>> recent;
  // Update entries staged (keyed on the engine's stream) in flight slot pend_slot, decided with the
  // next device CheckTx batch, which takes that slot, or alone by flush_pending
  int pend_slot = -1;
  uint32_t pend_n = 0;
  txv_ctx* pend_ctx = nullptr;
  uint64_t next_ticket = 1;
  int next_slot = 0;
  uint32_t batch_hint = 0;                         // the largest CheckTx batch submitted to the device
  int64_t infl_len = 0, infl_bytes = 0;
  ~txv_pool();

  bool cache_push(const Key& k) {                  // mapTxCache.Push
    if (!cache_on) return true;
    if (cache.len >= cfg.cache_size && cache.head >= 0) {   // full: the eviction comes first
      const int32_t e = cache_map.find(k);
      if (e >= 0) { cache.move_to_back(e); return false; }
      cache_map.erase(cache.nodes[cache.head].k);   // before unlink: the index reads the node's key
      cache.unlink(cache.head);
      cache_map.put(k, cache.push_back(k, 0));
      return true;
    }
    // not full: one probe finds the key or inserts it
    const int32_t e = cache_map.find_or_insert(k, [&] { return cache.push_back(k, 0); });
    if (e >= 0) { cache.move_to_back(e); return false; }
    return true;
  }
};

int txv_sig_keys_overlap(txv_ctx* c, const txv_votes* v, const uint8_t* sig_full, const uint64_t* sig_full_off,
                         uint8_t* keys_out, const std::function<void()>& overlap);   // runtime.cpp

namespace {

int batch_keys(txv_pool* p, txv_ctx* ctx, const txv_votes* v, const uint8_t* sig_full, const uint64_t* sig_full_off,
               const std::function<void()>& overlap = nullptr) {
  p->keys.resize((size_t)v->n * 32 + 32);
  return txv_sig_keys_overlap(ctx, v, sig_full, sig_full_off, p->keys.data(), overlap);
}

}  // namespace

void txv_sha256_bytes(const uint8_t* p, uint64_t n, uint8_t out[32]);   // runtime.cpp
void txv_host_parallel_for(txv_ctx* c, uint32_t n, const std::function<void(uint32_t, uint32_t)>& fn,
                           uint32_t min_chunk = 4096);   // runtime.cpp (the context's host workers)

std::shared_ptr<void> txv_host_workers_new();   // runtime.cpp: a standalone worker pool
void txv_host_workers_for(void* w, uint32_t n, const std::function<void(uint32_t, uint32_t)>& fn, uint32_t min_chunk);

namespace {

// the batch passes' worker threads: the context's when there is one, else the pool's own
// (created on the first batch-path call without a context: TXV_HOST_THREADS, else min(16, cores))
void pool_parallel_for(txv_pool* p, txv_ctx* ctx, uint32_t n, const std::function<void(uint32_t, uint32_t)>& fn,
                       uint32_t min_chunk = 4096) {
  if (ctx) { txv_host_parallel_for(ctx, n, fn, min_chunk); return; }
  if (!p->workers) p->workers = txv_host_workers_new();
  txv_host_workers_for(p->workers.get(), n, fn, min_chunk);
}

}  // namespace

namespace {

// node indices a KeyList hands out to its next n push_backs (free list from the back first)
void next_indices(const KeyList& L, uint32_t n, std::vector<int32_t>& idx) {
  idx.resize(n);
  const size_t nf = L.free_.size();
  for (uint32_t i = 0; i < n; ++i)
    idx[i] = i < nf ? L.free_[nf - 1 - i] : (int32_t)(L.nodes.size() + (i - nf));
}

// the n nodes at idx (keys already written) appended in order: links (on the host workers),
// head / tail, free list
void link_appended(txv_ctx* ctx, KeyList& L, const std::vector<int32_t>& idx, uint32_t n) {
  const int32_t tail = L.tail;
  txv_host_parallel_for(ctx, n, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; ++i) {
      KeyList::Node& nd = L.nodes[idx[i]];
      nd.prev = i ? idx[i - 1] : tail;
      nd.next = i + 1 < n ? idx[i + 1] : -1;
    }
  });
  if (L.tail >= 0) L.nodes[L.tail].next = idx[0]; else L.head = idx[0];
  L.tail = idx[n - 1];
  L.len += n;
  const size_t nf = L.free_.size();
  L.free_.resize(nf - std::min<size_t>(nf, n));
}

}  // namespace

namespace {

// amino nameToDisfix("tendermint/txvotepool/TxVoteMessage") (go-amino, external): SHA-256 of the
// registered name, zero bytes skipped, 3 disambiguation bytes, zero bytes skipped, 4 prefix bytes
void txvote_msg_disfix(uint8_t disamb[3], uint8_t prefix[4]) {
  static const char name[] = "tendermint/txvotepool/TxVoteMessage";
  uint8_t h[32];
  txv_sha256_bytes(reinterpret_cast<const uint8_t*>(name), sizeof name - 1, h);
  int i = 0;
  while (h[i] == 0) ++i;
  memcpy(disamb, h + i, 3);
  i += 3;
  while (h[i] == 0) ++i;
  memcpy(prefix, h + i, 4);
}

inline uint32_t vote_size(const txv_votes* v, uint32_t i) {
  return (uint32_t)txv_host::txvote_size(v->height[i], v->txhash_len[i], v->ts_sec[i], v->ts_nanos[i], v->addr_len[i],
                                         v->sig_len[i]);
}

}  // namespace

namespace {

// slots prefetched ahead in the per-partition loops (DRAM-latency bound, as the sequential loop)
constexpr uint32_t kAdmitAhead = 16;

// Batch CheckTxWithInfo (txvotepool.go:187-261) without the sequential loop, exact for any mix of
// new keys, in-batch repeats, cached replays and LRU evictions.
//
// The cache (mapTxCache, :416-438) is an LRU of capacity C over the keys of the votes that reach
// cache.Push -- every vote that is neither rejected as full nor too large -- whether the push hits
// (move to back) or misses (push back, evicting the front when full).  So with S = the cache's
// entries front to back followed by the batch's pushes, a push of key k at position e hits iff k
// occurs earlier in S (last at p) and the number of DISTINCT keys in S(p, e) is below C: LRU's
// stack-distance property.  That count is (e - p - 1) minus the pairs (i, next(i)) of consecutive
// occurrences of one key nested inside (p, e), so every decision is independent of the others:
//   - k neither cached nor earlier in the batch: miss;
//   - L0 + pushes <= C (nothing can be evicted), or e - p - 1 < C: hit;
//   - a cached key beyond the first min(L0, pushes) entries from the front cannot be evicted by
//     this batch's pushes: hit;
//   - otherwise count the nested pairs (offline sweep over a Fenwick tree; only these "far"
//     repeats pay for it).
// The pool's Size cap cuts the batch at the first vote that finds the pool full: every later vote
// is ErrMempoolIsFull and pushes nothing, so the decisions before the cut stand.  When the
// MaxTxsBytes cap could bind (it is not monotone in the batch), the sequential loop runs instead.
// The state is then written directly: the new LRU = the C most recent distinct keys, the pool list
// = the admitted votes appended in order (txsMap.Store overwriting, as addTx does).

uint64_t batch_tab_hash(const Key& k) { return key_hash(k, 0x9e3779b97f4a7c15ULL); }

bool batch_check(txv_pool* p, txv_ctx* ctx, BatchScratch& S, const Key* keys, uint32_t n, uint8_t* status_out) {
  static const bool prof = getenv("TXV_PROFILE_HOST") != nullptr;
  std::chrono::steady_clock::time_point tp[16];
  int ntp = 0;
  auto mark = [&] { if (prof) tp[ntp++] = std::chrono::steady_clock::now(); };
  mark();
  const int64_t max_tx = (int64_t)p->cfg.max_msg_bytes - 8;
  const bool wal = (p->cfg.flags & TXV_POOL_WAL) != 0, cache_on = p->cache_on;
  const uint64_t C = p->cfg.cache_size, L0 = cache_on ? p->cache.len : 0;
  const uint32_t* sizes = p->sizes.data();
  auto is_push = [&](uint32_t i) { return (int64_t)sizes[i] <= max_tx; };
  p->part.resize(n);
  uint8_t* part = p->part.data();
  // 0. per chunk of arrival order: each key's index partition, the summed sizes, per-partition
  //    counts and pushes; then the stable partition order and the push index aidx[i] (position
  //    L0 + aidx[i] in S)
  const uint32_t P = std::max<uint32_t>(1, std::min<uint32_t>(64, n / 2048));
  const uint32_t HW = kParts + 2;                          // per chunk: kParts counts, pushes, -
  S.hist.assign((size_t)P * HW, 0);
  std::vector<uint64_t> sum_c(P, 0);
  S.order.resize(n); S.pos.resize(n); S.aidx.resize(n);
  auto chunk = [&](uint32_t c, uint32_t& lo, uint32_t& hi) {
    lo = (uint32_t)((uint64_t)n * c / P); hi = (uint32_t)((uint64_t)n * (c + 1) / P);
  };
  pool_parallel_for(p, ctx, P, [&](uint32_t c0, uint32_t c1) {
    for (uint32_t c = c0; c < c1; ++c) {
      uint32_t lo, hi, pushes = 0;
      uint64_t sm = 0;
      chunk(c, lo, hi);
      uint32_t* h = S.hist.data() + (size_t)c * HW;
      for (uint32_t i = lo; i < hi; ++i) {
        const uint8_t q = (uint8_t)PartIndex::part(keys[i]);
        part[i] = q;
        ++h[q];
        pushes += is_push(i);
        sm += sizes[i];
      }
      h[kParts] = pushes;
      sum_c[c] = sm;
    }
  }, 1);
  uint64_t sum = 0;
  for (uint32_t c = 0; c < P; ++c) sum += sum_c[c];
  if (p->txs_bytes + (int64_t)sum > (int64_t)p->cfg.max_txs_bytes) return false;   // the bytes cap could bind
  S.cnt.assign(kParts + 1, 0);
  uint32_t na = 0;
  {
    uint32_t run = 0;
    for (uint32_t q = 0; q < kParts; ++q) {
      S.cnt[q] = run;
      for (uint32_t c = 0; c < P; ++c) {
        uint32_t& h = S.hist[(size_t)c * HW + q];
        const uint32_t t = h;
        h = run;
        run += t;
      }
    }
    S.cnt[kParts] = run;
    for (uint32_t c = 0; c < P; ++c) {
      uint32_t& h = S.hist[(size_t)c * HW + kParts];
      const uint32_t t = h;
      h = na;
      na += t;
    }
  }
  pool_parallel_for(p, ctx, P, [&](uint32_t c0, uint32_t c1) {
    for (uint32_t c = c0; c < c1; ++c) {
      uint32_t lo, hi;
      chunk(c, lo, hi);
      uint32_t* h = S.hist.data() + (size_t)c * HW;
      uint32_t a = h[kParts];
      for (uint32_t i = lo; i < hi; ++i) {
        const uint32_t j = h[part[i]]++;
        S.order[j] = i;
        S.pos[i] = j;
        S.aidx[i] = a;
        a += is_push(i);
      }
    }
  }, 1);
  const bool evict = cache_on && L0 + na > C;
  auto per_part = [&](const std::function<void(uint32_t)>& fn) {
    pool_parallel_for(p, ctx, kParts, [&](uint32_t lo, uint32_t hi) { for (uint32_t q = lo; q < hi; ++q) fn(q); }, 1);
  };
  S.prevj.resize(n); S.firstj.resize(n); S.cnodej.resize(n); S.nextj.resize(n); S.decj.resize(n);
  mark();
  // 1. front ranks: only the first min(L0, pushes) cache entries can be evicted by this batch
  if (evict) {
    if (S.qpos.size() < p->cache.nodes.size()) S.qpos.resize(p->cache.nodes.size(), -1);
    const uint64_t F = std::min<uint64_t>(L0, na);
    S.qtouched.clear();
    int32_t e = p->cache.head;
    for (uint64_t r = 0; r < F && e >= 0; ++r, e = p->cache.nodes[e].next) {
      S.qpos[e] = (int32_t)r;
      S.qtouched.push_back(e);
    }
  }
  mark();
  // 2. per partition, in batch order: the previous push of the same key in the batch, the first
  //    one, the cache node of a first push whose key is cached (a hash tag beside each slot: keys
  //    are compared only on a tag match), and the decision (1 miss, 2 hit, 3 far: counted below)
  std::vector<std::vector<uint32_t>> far_q(kParts);
  // doubled positions: front entry r -> 2r, an entry beyond the front -> 2 L0 - 1, push i -> 2 (L0 + aidx)
  auto pos2 = [&](uint32_t i) -> uint64_t { return 2 * (L0 + S.aidx[i]); };
  auto init2 = [&](int32_t node) -> uint64_t { const int32_t r = S.qpos[node]; return r >= 0 ? 2 * (uint64_t)r : 2 * L0 - 1; };
  per_part([&](uint32_t q) {
    const uint32_t lo = S.cnt[q], hi = S.cnt[q + 1];
    auto& pairs = S.pairs[q];
    auto& cfirst = S.cached_firsts[q];
    pairs.clear();
    cfirst.clear();
    uint32_t firsts = 0;
    uint32_t cap = 16;
    while (cap < 2 * (hi - lo)) cap *= 2;
    std::vector<uint64_t> tab(cap, 0);            // (tag << 32) | (j + 1) of the key's last push
    const FlatIndex& cf = *p->cache_map.p[q];
    for (uint32_t j = lo; j < hi; ++j) {
      if (j + 2 * kAdmitAhead < hi) __builtin_prefetch(&keys[S.order[j + 2 * kAdmitAhead]]);   // the key, then its slot
      if (cache_on && j + kAdmitAhead < hi) cf.prefetch(keys[S.order[j + kAdmitAhead]]);
      const uint32_t i = S.order[j];
      S.cnodej[j] = -1;
      S.nextj[j] = -1;
      if (!is_push(i)) { S.prevj[j] = -2; S.firstj[j] = (int32_t)j; S.decj[j] = 0; continue; }
      const uint64_t hv = batch_tab_hash(keys[i]);
      const uint64_t tag = (hv >> 32) | 1u;
      size_t sl = hv & (cap - 1);
      for (; tab[sl]; sl = (sl + 1) & (cap - 1))
        if ((tab[sl] >> 32) == tag && keys[S.order[(uint32_t)tab[sl] - 1]] == keys[i]) break;
      uint8_t d;
      if (tab[sl]) {
        const uint32_t pj = (uint32_t)tab[sl] - 1;
        S.prevj[j] = (int32_t)pj;
        S.firstj[j] = S.firstj[pj];
        S.nextj[pj] = (int32_t)j;
        d = !cache_on ? 1 : ((!evict || S.aidx[i] - S.aidx[S.order[pj]] - 1 < C) ? 2 : 3);
        if (evict) pairs.emplace_back(pos2(S.order[pj]), pos2(i));
      } else {
        S.prevj[j] = -1;
        S.firstj[j] = (int32_t)j;
        ++firsts;
        d = 1;
        if (cache_on) {
          const int32_t cn = cf.find(keys[i]);
          S.cnodej[j] = cn;
          if (cn >= 0) {
            const int32_t r = evict ? S.qpos[cn] : -1;
            d = (r < 0 || L0 + S.aidx[i] - (uint64_t)r - 1 < C) ? 2 : 3;
            cfirst.push_back(cn);
            if (evict) pairs.emplace_back(init2(cn), pos2(i));
          }
        }
      }
      tab[sl] = (tag << 32) | (j + 1);
      S.decj[j] = d;
      if (d == 3) far_q[q].push_back(i);
    }
    S.firsts[q] = firsts;
  });
  std::vector<uint32_t> far;
  for (auto& v : far_q) far.insert(far.end(), v.begin(), v.end());
  mark();
  if (!far.empty()) {
    std::sort(far.begin(), far.end());                     // by position = batch order
    const size_t F = far.size();
    std::vector<uint64_t> fe(F), fp(F);                    // each far push's window (p, e)
    for (size_t f = 0; f < F; ++f) {
      const uint32_t i = far[f], j = S.pos[i];
      fe[f] = pos2(i);
      fp[f] = S.prevj[j] >= 0 ? pos2(S.order[S.prevj[j]]) : init2(S.cnodej[j]);
    }
    auto decide_far = [&](size_t f, uint64_t nested) {
      const uint64_t window = (fe[f] - fp[f]) / 2 - 1;     // pushes strictly between (p is exact here)
      S.decj[S.pos[far[f]]] = window - nested < C ? 2 : 1;
    };
    size_t npairs = 0;
    for (uint32_t q = 0; q < kParts; ++q) npairs += S.pairs[q].size();
    if (F <= 64 || F * npairs <= (size_t)1 << 21) {
      // few far repeats: every partition counts its nested pairs for each of them directly
      std::vector<uint32_t> cnt_qf(kParts * F, 0);
      per_part([&](uint32_t q) {
        uint32_t* cf = cnt_qf.data() + (size_t)q * F;
        for (const auto& ab : S.pairs[q])                  // pair (start, next occurrence)
          for (size_t f = 0; f < F; ++f) cf[f] += (uint32_t)(ab.first > fp[f]) & (uint32_t)(ab.second < fe[f]);
      });
      for (size_t f = 0; f < F; ++f) {
        uint64_t nested = 0;
        for (uint32_t q = 0; q < kParts; ++q) nested += cnt_qf[(size_t)q * F + f];
        decide_far(f, nested);
      }
    } else {
    // pairs (next occurrence, occurrence) of consecutive pushes of one key
    std::vector<std::pair<uint64_t, uint64_t>> pairs;
    for (uint32_t q = 0; q < kParts; ++q)
      for (const auto& ab : S.pairs[q]) pairs.emplace_back(ab.second, ab.first);
    std::sort(pairs.begin(), pairs.end());                 // by next occurrence: the sweep order
    std::vector<uint64_t> starts(pairs.size());            // Fenwick tree over the distinct starts
    for (size_t k = 0; k < pairs.size(); ++k) starts[k] = pairs[k].second;
    std::sort(starts.begin(), starts.end());
    starts.erase(std::unique(starts.begin(), starts.end()), starts.end());
    const size_t M = starts.size();
    std::vector<uint32_t> fen(M + 1, 0);
    uint32_t added = 0;
    size_t pi = 0;
    for (size_t f = 0; f < F; ++f) {
      for (; pi < pairs.size() && pairs[pi].first < fe[f]; ++pi, ++added) {
        const size_t x0 = std::lower_bound(starts.begin(), starts.end(), pairs[pi].second) - starts.begin() + 1;
        for (size_t x = x0; x <= M; x += x & (~x + 1)) ++fen[x];
      }
      uint32_t upto = 0;                                   // pairs starting at or before p
      for (size_t x = std::upper_bound(starts.begin(), starts.end(), fp[f]) - starts.begin(); x > 0; x -= x & (~x + 1))
        upto += fen[x];
      decide_far(f, added - upto);
    }
    }
  }
  if (evict)
    for (int32_t e : S.qtouched) S.qpos[e] = -1;
  mark();
  // 3. statuses in arrival order, the Size cap's cut (only when the batch could reach it); the
  //    admitted votes' pool nodes written and linked in the same passes
  S.dec.resize(n); S.adm.resize(n);
  uint32_t m = n;
  uint64_t admitted = 0, admitted_bytes = 0;
  auto status_of = [&](uint32_t i, uint8_t d) -> uint8_t {
    if (d == 0) return TXV_POOL_ERR_TOO_LARGE;
    if (d == 2) return TXV_POOL_ERR_IN_CACHE;
    return (!sizes[i] && wal) ? TXV_POOL_ERR_ENCODING : TXV_POOL_OK;
  };
  std::vector<uint64_t> base_c(P, 0);
  const bool may_cut = (int64_t)p->txs.len + (int64_t)na >= (int64_t)p->cfg.size;
  if (!may_cut) {
    std::vector<uint64_t> cnt_c(P, 0), bytes_c(P, 0);
    pool_parallel_for(p, ctx, P, [&](uint32_t c0, uint32_t c1) {
      for (uint32_t c = c0; c < c1; ++c) {
        uint32_t lo, hi;
        chunk(c, lo, hi);
        uint64_t k = 0, b = 0;
        for (uint32_t i = lo; i < hi; ++i) {
          const uint8_t d = S.decj[S.pos[i]];
          S.dec[i] = d;
          const uint8_t st = status_of(i, d);
          status_out[i] = st;
          if (st == TXV_POOL_OK) { ++k; b += sizes[i]; }
        }
        cnt_c[c] = k;
        bytes_c[c] = b;
      }
    }, 1);
    for (uint32_t c = 0; c < P; ++c) { base_c[c] = admitted; admitted += cnt_c[c]; admitted_bytes += bytes_c[c]; }
  } else {
    for (uint32_t i = 0; i < n; ++i) {
      if ((int64_t)p->txs.len + (int64_t)admitted >= (int64_t)p->cfg.size) { m = i; break; }
      const uint8_t d = S.decj[S.pos[i]];
      S.dec[i] = d;
      const uint8_t st = status_of(i, d);
      status_out[i] = st;
      S.adm[i] = -1;
      if (st == TXV_POOL_OK) { S.adm[i] = (int32_t)admitted++; admitted_bytes += sizes[i]; }
    }
    if (m < n) {
      memset(status_out + m, TXV_POOL_ERR_FULL, n - m);
      for (uint32_t i = m; i < n; ++i) { S.dec[i] = 0; S.adm[i] = -1; }
    }
  }
  const uint32_t A = (uint32_t)admitted;
  const int32_t old_tail = p->txs.tail;
  if (A) {
    next_indices(p->txs, A, p->idx_t);
    p->txs.nodes.resize(std::max<size_t>(p->txs.nodes.size(), (size_t)p->idx_t[A - 1] + 1));
  }
  auto write_node = [&](uint32_t i, uint32_t a) {
    p->txs.nodes[p->idx_t[a]] = KeyList::Node{keys[i], sizes[i], a ? p->idx_t[a - 1] : old_tail,
                                              a + 1 < A ? p->idx_t[a + 1] : -1};
  };
  if (!may_cut) {
    pool_parallel_for(p, ctx, P, [&](uint32_t c0, uint32_t c1) {
      for (uint32_t c = c0; c < c1; ++c) {
        uint32_t lo, hi;
        chunk(c, lo, hi);
        uint32_t a = (uint32_t)base_c[c];
        for (uint32_t i = lo; i < hi; ++i) {
          if (status_out[i] == TXV_POOL_OK) { S.adm[i] = (int32_t)a; write_node(i, a); ++a; }
          else S.adm[i] = -1;
        }
      }
    }, 1);
  } else {
    for (uint32_t i = 0; i < m; ++i)
      if (S.adm[i] >= 0) write_node(i, (uint32_t)S.adm[i]);
  }
  if (A) {                                                 // addTx: txs.PushBack in arrival order
    if (old_tail >= 0) p->txs.nodes[old_tail].next = p->idx_t[0]; else p->txs.head = p->idx_t[0];
    p->txs.tail = p->idx_t[A - 1];
    p->txs.len += A;
    const size_t nf = p->txs.free_.size();
    p->txs.free_.resize(nf - std::min<size_t>(nf, A));
  }
  mark();
  // 4. the cache: the C most recent distinct keys of S up to the cut, in recency order
  if (cache_on) {
    // U = distinct keys pushed before m (each one's last push is kept in recency order), detached
    // = cached keys pushed again (they leave their place in the old list)
    std::vector<uint32_t> last;
    uint64_t U = 0, detached = 0;
    const bool whole = m == n;                             // no cut: the scan's counts hold
    if (whole)
      for (uint32_t q = 0; q < kParts; ++q) { U += S.firsts[q]; detached += S.cached_firsts[q].size(); }
    else {
      last.reserve(na);
      for (uint32_t i = 0; i < m; ++i) {
        if (!S.dec[i]) continue;
        const uint32_t j = S.pos[i];
        const int32_t nj = S.nextj[j];
        if (nj < 0 || S.order[nj] >= m) last.push_back(i);
        if (S.prevj[j] == -1 && S.cnodej[j] >= 0) ++detached;
      }
      U = last.size();
    }
    const uint64_t keepU = std::min<uint64_t>(U, C), L1 = p->cache.len - detached;
    auto cnode_of = [&](uint32_t i) { return S.cnodej[S.firstj[S.pos[i]]]; };
    const uint64_t keep_old = std::min<uint64_t>(L1, C - keepU), evicted = L1 - keep_old;
    if (keep_old < evicted + detached) {
      // most of the old LRU goes: rebuild list and index from the survivors + this batch's keys
      std::vector<Key> fin_keys(keep_old + keepU);
      if (keep_old) {                                      // the last keep_old entries not pushed again
        if (S.dmark.size() < p->cache.nodes.size()) S.dmark.resize(p->cache.nodes.size(), 0);
        auto mark_pushed = [&](uint8_t v) {
          if (whole) {
            for (uint32_t q = 0; q < kParts; ++q)
              for (int32_t e : S.cached_firsts[q]) S.dmark[e] = v;
          } else {
            for (uint32_t i = 0; i < m; ++i) {
              const uint32_t j = S.pos[i];
              if (S.dec[i] && S.prevj[j] == -1 && S.cnodej[j] >= 0) S.dmark[S.cnodej[j]] = v;
            }
          }
        };
        mark_pushed(1);
        uint64_t r = keep_old;
        for (int32_t e = p->cache.tail; r && e >= 0; e = p->cache.nodes[e].prev)
          if (!S.dmark[e]) fin_keys[--r] = p->cache.nodes[e].k;
        mark_pushed(0);
      }
      // the last push of each of the keepU most recent distinct keys, from the end of the batch back
      uint64_t kf = keep_old + keepU;
      if (whole) {
        for (uint32_t i = m; i-- > 0 && kf > keep_old;)
          if (S.dec[i] && S.nextj[S.pos[i]] < 0) fin_keys[--kf] = keys[i];
      } else {
        for (size_t u = U; u-- > U - keepU;) fin_keys[--kf] = keys[last[u]];
      }
      mark();
      const uint32_t L = (uint32_t)fin_keys.size();
      p->cache.clear();
      p->cache.nodes.resize(L);
      for (uint32_t k = 0; k < L; ++k)
        p->cache.nodes[k] = KeyList::Node{fin_keys[k], 0, (int32_t)k - 1, k + 1 < L ? (int32_t)k + 1 : -1};
      p->cache.head = L ? 0 : -1;
      p->cache.tail = (int32_t)L - 1;
      p->cache.len = L;
      mark();
      std::vector<uint8_t> kpart(L);
      pool_parallel_for(p, ctx, L, [&](uint32_t lo, uint32_t hi) {
        for (uint32_t k = lo; k < hi; ++k) kpart[k] = (uint8_t)PartIndex::part(fin_keys[k]);
      });
      mark();
      per_part([&](uint32_t q) {
        FlatIndex& f = *p->cache_map.p[q];
        f.clear();
        for (uint32_t k = 0; k < L; ++k)
          if (kpart[k] == q) f.put(fin_keys[k], (int32_t)k);
      });
    } else {
      if (whole) {                                         // every push's key, in order, for the lists below
        last.reserve(U);
        for (uint32_t i = 0; i < m; ++i)
          if (S.dec[i] && S.nextj[S.pos[i]] < 0) last.push_back(i);
      }
      for (uint32_t q = 0; q < kParts && whole; ++q)       // cached keys pushed again leave their place
        for (int32_t e : S.cached_firsts[q]) p->cache.detach(e);
      if (!whole)
        for (uint32_t i = 0; i < m; ++i) {
          const uint32_t j = S.pos[i];
          if (S.dec[i] && S.prevj[j] == -1 && S.cnodej[j] >= 0) p->cache.detach(S.cnodej[j]);
        }
      for (uint64_t r = 0; r < evicted; ++r) {             // evictions from the front
        const int32_t h = p->cache.head;
        p->cache_map.erase(p->cache.nodes[h].k);
        p->cache.unlink(h);
      }
      std::vector<int32_t> fin(keepU);
      uint32_t n_new = 0;
      for (size_t u = 0; u < U; ++u) {
        const uint32_t i = last[u];
        const int32_t cn = cnode_of(i);
        if (u < U - keepU) {                               // pushed, then evicted inside the batch
          if (cn >= 0) { p->cache_map.erase(keys[i]); p->cache.free_.push_back(cn); }
        } else {
          fin[u - (U - keepU)] = cn;
          n_new += cn < 0;
        }
      }
      next_indices(p->cache, n_new, p->idx_c);
      if (n_new) {
        const size_t old = p->cache.nodes.size();
        p->cache.nodes.resize(std::max<size_t>(old, (size_t)p->idx_c[n_new - 1] + 1));
        const size_t nf = p->cache.free_.size();
        p->cache.free_.resize(nf - std::min<size_t>(nf, n_new));
      }
      std::vector<std::vector<std::pair<uint32_t, int32_t>>> ins(kParts);
      for (size_t u = 0, k = 0; u < keepU; ++u)
        if (fin[u] < 0) {
          const uint32_t i = last[U - keepU + u];
          fin[u] = p->idx_c[k++];
          p->cache.nodes[fin[u]] = KeyList::Node{keys[i], 0, -1, -1};
          ins[part[i]].emplace_back(i, fin[u]);
        }
      per_part([&](uint32_t q) {                           // index the new nodes
        FlatIndex& f = *p->cache_map.p[q];
        const auto& L = ins[q];
        for (size_t j = 0; j < L.size(); ++j) {
          if (j + kAdmitAhead < L.size()) f.prefetch(keys[L[j + kAdmitAhead].first]);
          f.put(keys[L[j].first], L[j].second);
        }
      });
      p->cache.append_linked(fin);
    }
  }
  mark();
  // 5. txsMap.Store of the admitted votes (batch order within each partition: a key admitted
  //    twice keeps its later node, as the sequential Store does)
  if (A) {
    per_part([&](uint32_t q) {
      FlatIndex& f = *p->txs_map.p[q];
      const uint32_t lo = S.cnt[q], hi = S.cnt[q + 1];
      for (uint32_t j = lo; j < hi; ++j) {
        if (j + 2 * kAdmitAhead < hi) __builtin_prefetch(&keys[S.order[j + 2 * kAdmitAhead]]);
        if (j + kAdmitAhead < hi) f.prefetch(keys[S.order[j + kAdmitAhead]]);
        const uint32_t i = S.order[j];
        if (S.adm[i] >= 0) f.put(keys[i], p->idx_t[S.adm[i]]);
      }
    });
    p->txs_bytes += (int64_t)admitted_bytes;
  }
  mark();
  if (prof) {
    auto ms = [&](int a) { return std::chrono::duration<double, std::milli>(tp[a + 1] - tp[a]).count(); };
    if (ntp == 8)
      fprintf(stderr, "[txv pool] batch: order=%.3f front=%.3f scan+decide=%.3f far(%zu)=%.3f status+nodes=%.3f cache=%.3f txs=%.3f ms\n",
              ms(0), ms(1), ms(2), far.size(), ms(3), ms(4), ms(5), ms(6));
    else if (ntp == 11)   // the cache rebuilt: survivors + last pushes, list, partitions, index
      fprintf(stderr, "[txv pool] batch: order=%.3f front=%.3f scan+decide=%.3f far(%zu)=%.3f status+nodes=%.3f "
              "cache=%.3f (keys %.3f list %.3f part %.3f index %.3f) txs=%.3f ms\n", ms(0), ms(1), ms(2), far.size(), ms(3),
              ms(4), std::chrono::duration<double, std::milli>(tp[9] - tp[5]).count(), ms(5), ms(6), ms(7), ms(8), ms(9));
  }
  return true;
}

}  // namespace

txv_pool::~txv_pool() {
  pooldev_free(dev);
  for (PoolDev* d : retired) pooldev_free(d);
}

extern "C" {

int txv_pool_new(const txv_pool_config* cfg, int64_t height, txv_pool** out) {
  if (!out) return TXV_EINVAL;
  txv_pool* p = new (std::nothrow) txv_pool();
  if (!p) return TXV_ENOMEM;
  if (cfg) p->cfg = *cfg;
  // tendermint config.DefaultMempoolConfig (external): Size 5000, CacheSize 10000,
  // MaxTxsBytes 1 GiB, MaxMsgBytes 1 MiB
  if (!p->cfg.size) p->cfg.size = 5000;
  if (!p->cfg.cache_size) p->cfg.cache_size = 10000;
  if (!p->cfg.max_txs_bytes) p->cfg.max_txs_bytes = 1ull << 30;
  if (!p->cfg.max_msg_bytes) p->cfg.max_msg_bytes = 1u << 20;
  p->cache_on = p->cfg.cache_size != TXV_POOL_NO_CACHE;
  p->height = height;
  if (p->cache_on) p->cache_map.reserve(std::min<uint32_t>(p->cfg.cache_size, 1u << 22));
  p->txs_map.reserve(std::min<uint32_t>(p->cfg.size, 1u << 22));
  p->txs.nodes.reserve(std::min<uint32_t>(p->cfg.size, 1u << 22));   // no reallocation while the pool fills
  *out = p;
  return TXV_OK;
}

void txv_pool_free(txv_pool* p) { delete p; }

}  // extern "C"

namespace {

// CheckTxWithInfo for n votes in arrival order whose keys (keys) and TxVote.Size() values
// (p->sizes) are known: the order-dependent part (caps, cache, pool list).  p->mu is held.
int cache_to_host(txv_pool* p, txv_ctx* ctx);
void host_cache_written(txv_pool* p);
int list_to_host(txv_pool* p, txv_ctx* ctx);

int drain_flights(txv_pool* p, bool flush = true);
void publish_locked(txv_pool* p);

int pool_admit_body(txv_pool* p, txv_ctx* ctx, const Key* keys, uint32_t n, uint8_t* status_out);
int pool_admit(txv_pool* p, txv_ctx* ctx, const Key* keys, uint32_t n, uint8_t* status_out) {
  const int r = pool_admit_body(p, ctx, keys, n, status_out);
  publish_locked(p);
  return r;
}
int pool_admit_body(txv_pool* p, txv_ctx* ctx, const Key* keys, uint32_t n, uint8_t* status_out) {
  if (int r = drain_flights(p)) return r;
  if (int r = list_to_host(p, ctx)) return r;
  if (int r = cache_to_host(p, ctx)) return r;
  host_cache_written(p);
  const auto t1 = std::chrono::steady_clock::now();
  const int64_t max_tx = (int64_t)p->cfg.max_msg_bytes - 8;   // calcMaxTxSize
  if (n >= 4096 && batch_check(p, ctx, p->bs, keys, n, status_out)) {
    if (getenv("TXV_PROFILE_HOST")) {
      const auto t2 = std::chrono::steady_clock::now();
      fprintf(stderr, "[txv pool] batch-check=%.3fms n=%u\n", std::chrono::duration<double, std::milli>(t2 - t1).count(), n);
    }
    return TXV_OK;
  }
  // The sequential CheckTx loop (DRAM-latency bound on the two hash tables: prefetched ahead).
  // A two-thread split (decisions + cache on one thread, the admitted votes replayed into
  // txs / txsMap on another) measured slower: 3.0 vs 2.4 ms per 64k votes
  // (tools/debug/pool_ab.py, profiles/r02/pool_ab.log).
#ifndef TXV_POOL_AHEAD
#define TXV_POOL_AHEAD 16
#endif
  constexpr uint32_t kAhead = TXV_POOL_AHEAD;
  for (uint32_t i = 0; i < n; ++i) {
    if (i + kAhead < n) {
      if (p->cache_on) p->cache_map.prefetch(keys[i + kAhead]);
      p->txs_map.prefetch(keys[i + kAhead]);
    }
    const uint32_t sz = p->sizes[i];   // 0: amino error (Size() swallows it)
    if ((int64_t)p->txs.len >= (int64_t)p->cfg.size || (int64_t)sz + p->txs_bytes > (int64_t)p->cfg.max_txs_bytes) {
      status_out[i] = TXV_POOL_ERR_FULL;
      continue;
    }
    if ((int64_t)sz > max_tx) { status_out[i] = TXV_POOL_ERR_TOO_LARGE; continue; }
    if (!p->cache_push(keys[i])) { status_out[i] = TXV_POOL_ERR_IN_CACHE; continue; }
    if (!sz && (p->cfg.flags & TXV_POOL_WAL)) { status_out[i] = TXV_POOL_ERR_ENCODING; continue; }
    p->txs_map.put(keys[i], p->txs.push_back(keys[i], sz));     // addTx (txsMap.Store overwrites)
    p->txs_bytes += sz;
    status_out[i] = TXV_POOL_OK;
  }
  if (getenv("TXV_PROFILE_HOST")) {
    const auto t2 = std::chrono::steady_clock::now();
    fprintf(stderr, "[txv pool] lru=%.3fms n=%u\n", std::chrono::duration<double, std::milli>(t2 - t1).count(), n);
  }
  return TXV_OK;
}

// ---- TXV_POOL_DEVICE_CACHE: the cache's copy in HBM (pool_dev.h) ----
// Exactly one of the two copies is current after any call (dev_state): a batch decided on the
// device leaves the host's list stale (kDevAhead) until a host-side reader or writer of the cache
// (the sequential / keys-only check paths, Update, cache_keys) fetches it back; a host-side write
// leaves the device's stale (kHostAhead) until the next device batch uploads the list.
bool dev_mode(const txv_pool* p) { return (p->cfg.flags & TXV_POOL_DEVICE_CACHE) != 0; }

// the host's cache list = keys [L] front to back, index rebuilt (partitions on the workers)
void cache_rebuild(txv_pool* p, txv_ctx* ctx, const Key* keys, uint32_t L) {
  p->cache.clear();
  p->cache.nodes.resize(L);
  for (uint32_t k = 0; k < L; ++k) p->cache.nodes[k] = KeyList::Node{keys[k], 0, (int32_t)k - 1, k + 1 < L ? (int32_t)k + 1 : -1};
  p->cache.head = L ? 0 : -1;
  p->cache.tail = (int32_t)L - 1;
  p->cache.len = L;
  pool_parallel_for(p, ctx, kParts, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t q = lo; q < hi; ++q) {
      FlatIndex& f = *p->cache_map.p[q];
      f.clear();
      for (uint32_t k = 0; k < L; ++k)
        if (PartIndex::part(keys[k]) == q) f.put(keys[k], (int32_t)k);
    }
  }, 1);
}

int cache_to_host(txv_pool* p, txv_ctx* ctx) {
  if (!p->dev || p->dev_state != txv_pool::kDevAhead) return TXV_OK;
  std::vector<uint8_t> kb;
  if (int r = pooldev_get_cache(ctx, p->dev, kb)) return r;
  cache_rebuild(p, ctx, reinterpret_cast<const Key*>(kb.data()), (uint32_t)(kb.size() / 32));
  p->dev_state = txv_pool::kSynced;
  return TXV_OK;
}

void host_cache_written(txv_pool* p) {
  if (p->dev) p->dev_state = txv_pool::kHostAhead;
}

int cache_to_dev(txv_pool* p, txv_ctx* ctx, uint32_t n) {
  // a rebind (another GPU, or a batch above the engine's capacity) frees the flight slots: every
  // submitted batch finished first; moving to another GPU takes the current list along
  if (p->dev && (!pooldev_same_device(ctx, p->dev) || n > pooldev_cap(p->dev)))
    if (int r = drain_flights(p)) return r;
  if (p->dev && !pooldev_same_device(ctx, p->dev)) {
    if (int r = cache_to_host(p, ctx)) return r;
    if (int r = list_to_host(p, ctx)) return r;
  }
  if (p->dev && p->waiters && !pooldev_same_device(ctx, p->dev)) {   // a waiter may still sync on it
    p->retired.push_back(p->dev);
    p->dev = nullptr;
  }
  PoolDev* before = p->dev;
  if (int r = pooldev_bind(ctx, &p->dev, p->cache_on ? p->cfg.cache_size : 0u, n)) return r;
  if (p->dev != before) p->dev_state = txv_pool::kHostAhead;   // a new device copy starts empty
  if (p->dev_state != txv_pool::kHostAhead) return TXV_OK;
  std::vector<Key> kl;
  kl.reserve(p->cache.len);
  for (int32_t e = p->cache.head; e >= 0; e = p->cache.nodes[e].next) kl.push_back(p->cache.nodes[e].k);
  if (int r = pooldev_put_cache(ctx, p->dev, reinterpret_cast<const uint8_t*>(kl.data()), (uint32_t)kl.size())) return r;
  p->dev_state = txv_pool::kSynced;
  return TXV_OK;
}

// the device's pool list back into txs / txsMap, in order (the entries txsMap indexes put there)
int list_to_host(txv_pool* p, txv_ctx* ctx) {
  if (!p->list_dev) return TXV_OK;
  std::vector<uint8_t> kb, ins;
  std::vector<uint32_t> sz;
  if (int r = pooldev_list_get(ctx, p->dev, kb, sz, ins)) return r;
  const uint32_t L = (uint32_t)sz.size();
  const Key* keys = reinterpret_cast<const Key*>(kb.data());
  KeyList& T = p->txs;
  T.clear();
  T.nodes.resize(L);
  for (uint32_t e = 0; e < L; ++e) T.nodes[e] = KeyList::Node{keys[e], sz[e], (int32_t)e - 1, e + 1 < L ? (int32_t)e + 1 : -1};
  T.head = L ? 0 : -1;
  T.tail = (int32_t)L - 1;
  T.len = L;
  pool_parallel_for(p, ctx, kParts, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t q = lo; q < hi; ++q) {
      FlatIndex& f = *p->txs_map.p[q];
      f.clear();
      for (uint32_t e = 0; e < L; ++e)
        if (ins[e] && PartIndex::part(keys[e]) == q) f.put(keys[e], (int32_t)e);
    }
  }, 1);
  p->list_dev = false;
  return TXV_OK;
}

// the host's pool list into HBM before a device batch (p->dev bound)
int list_to_dev(txv_pool* p, txv_ctx* ctx) {
  if (p->list_dev) return TXV_OK;
  pooldev_list_hint(p->dev, p->cfg.size);
  const KeyList& T = p->txs;
  std::vector<Key> kl;
  std::vector<uint32_t> sz;
  std::vector<uint8_t> ins;
  kl.reserve(T.len); sz.reserve(T.len); ins.reserve(T.len);
  for (int32_t e = T.head; e >= 0; e = T.nodes[e].next) {
    kl.push_back(T.nodes[e].k);
    sz.push_back(T.nodes[e].size);
    ins.push_back(p->txs_map.find(T.nodes[e].k) == e);
  }
  if (int r = pooldev_list_put(ctx, p->dev, reinterpret_cast<const uint8_t*>(kl.data()), sz.data(), ins.data(),
                               (uint32_t)kl.size()))
    return r;
  p->list_dev = true;
  return TXV_OK;
}

// with mu held
void publish(txv_pool* p) {
  p->pub_len.store((int64_t)p->txs.len, std::memory_order_relaxed);
  p->pub_bytes.store(p->txs_bytes, std::memory_order_relaxed);
}
void publish_locked(txv_pool* p) { publish(p); }

// removeTx(tx, e, false) for every key of keys[n] the pool holds (Update, txvotepool.go:339-344),
// on the worker threads: (1) per txsMap partition, find + erase its keys (a key twice in the batch
// is found once); (2) the found nodes flagged; (3) one thread per run of consecutive flagged nodes
// (its first node's predecessor unflagged) relinks around the run -- runs touch disjoint
// neighbours, so no two threads write one pointer; (4) free list.  Returns the bytes removed (the
// Update votes' Size(), as the reference subtracts tx.Size()) and *count the nodes removed: the
// caller lowers txs.len.  The pool list is the host's (list_to_host).
int64_t remove_keys(txv_pool* p, txv_ctx* ctx, const Key* keys, const uint32_t* sizes, uint32_t n, size_t* count) {
  *count = 0;
  if (!n) return 0;
  PTimer tm("remove_keys");
  // the keys' partitions in chunks, then each partition's keys in batch order (a counting sort):
  // every worker then walks a dense list with its lookups prefetched ahead (DRAM-latency bound)
  std::vector<uint8_t>& pt = p->rm_part;
  std::vector<uint32_t>& ord = p->rm_order;
  pt.resize(n);
  ord.resize(n);
  const uint32_t nc = std::max<uint32_t>(1, std::min<uint32_t>(64, n / 2048));
  std::vector<uint32_t> cnt((size_t)nc * kParts, 0);
  pool_parallel_for(p, ctx, nc, [&](uint32_t c0, uint32_t c1) {
    for (uint32_t c = c0; c < c1; ++c)
      for (uint32_t i = (uint32_t)((uint64_t)n * c / nc); i < (uint32_t)((uint64_t)n * (c + 1) / nc); ++i) {
        pt[i] = (uint8_t)PartIndex::part(keys[i]);
        ++cnt[(size_t)c * kParts + pt[i]];
      }
  }, 1);
  std::vector<uint32_t> base(kParts + 1, 0), off((size_t)nc * kParts);
  uint32_t run = 0;
  for (uint32_t q = 0; q < kParts; ++q) {
    base[q] = run;
    for (uint32_t c = 0; c < nc; ++c) { off[(size_t)c * kParts + q] = run; run += cnt[(size_t)c * kParts + q]; }
  }
  base[kParts] = run;
  pool_parallel_for(p, ctx, nc, [&](uint32_t c0, uint32_t c1) {
    for (uint32_t c = c0; c < c1; ++c)
      for (uint32_t i = (uint32_t)((uint64_t)n * c / nc); i < (uint32_t)((uint64_t)n * (c + 1) / nc); ++i)
        ord[off[(size_t)c * kParts + pt[i]]++] = i;
  }, 1);
  tm.mark("order");
  std::vector<int32_t> found[kParts];
  int64_t bytes[kParts] = {};
  pool_parallel_for(p, ctx, kParts, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t q = lo; q < hi; ++q) {
      FlatIndex& ix = *p->txs_map.p[q];
      for (uint32_t a = base[q]; a < base[q + 1]; ++a) {
        if (a + 16 < base[q + 1]) ix.prefetch(keys[ord[a + 16]]);
        const uint32_t i = ord[a];
        const int32_t e = ix.take(keys[i]);       // a key twice in the batch: found once
        if (e < 0) continue;
        found[q].push_back(e);
        bytes[q] += sizes[i];
      }
    }
  }, 1);
  std::vector<int32_t>& all = p->rm_all;
  all.clear();
  int64_t removed_bytes = 0;
  for (uint32_t q = 0; q < kParts; ++q) {
    all.insert(all.end(), found[q].begin(), found[q].end());
    removed_bytes += bytes[q];
  }
  tm.mark("take");
  if (all.empty()) return 0;
  KeyList& L = p->txs;
  std::vector<uint8_t>& rm = p->rm_flag;
  if (rm.size() < L.nodes.size()) rm.resize(L.nodes.size(), 0);
  for (int32_t e : all) rm[e] = 1;
  const uint32_t m = (uint32_t)all.size();
  pool_parallel_for(p, ctx, m, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t a = lo; a < hi; ++a) {
      if (a + 8 < hi) __builtin_prefetch(&L.nodes[all[a + 8]]);
      const int32_t e = all[a];
      const int32_t pv = L.nodes[e].prev;
      if (pv >= 0 && rm[pv]) continue;                     // not the first node of its run
      int32_t r = e;
      while (L.nodes[r].next >= 0 && rm[L.nodes[r].next]) r = L.nodes[r].next;
      const int32_t nx = L.nodes[r].next;
      if (pv >= 0) L.nodes[pv].next = nx; else L.head = nx;
      if (nx >= 0) L.nodes[nx].prev = pv; else L.tail = pv;
    }
  }, 4096);
  tm.mark("relink");
  for (int32_t e : all) {
    rm[e] = 0;
    L.free_.push_back(e);
  }
  tm.mark("free");
  *count = m;
  return removed_bytes;
}

// finished Update tickets leave the queue (no caller waits for them)
void prune_updates(txv_pool* p) {
  for (auto it = p->tickets.begin(); it != p->tickets.end();)
    it = (it->upd && it->done) ? p->tickets.erase(it) : it + 1;
}

// a device batch needs the pool's Size and MaxTxsBytes caps not to bind inside it (pushes: the
// votes that reach cache.Push, bytes: the Size() sum of the checked votes)
bool dev_caps_ok(txv_pool* p, uint64_t pushes, uint64_t bytes) {
  return (int64_t)p->txs.len + p->infl_len + (int64_t)pushes < (int64_t)p->cfg.size &&
         p->txs_bytes + p->infl_bytes + (int64_t)bytes <= (int64_t)p->cfg.max_txs_bytes;
}

// an upper bound of the pool list's live entries before the next device batch (its own excluded)
uint64_t live_ub(const txv_pool* p) { return (uint64_t)p->txs.len + (uint64_t)std::max<int64_t>(0, p->infl_len); }

// a device batch's list counts in: its Update entries' removals, its votes' appends
void list_counts(txv_pool* p, int slot) {
  int64_t res[4];
  pooldev_result(p->dev, slot, res);
  p->txs.len = (size_t)((int64_t)p->txs.len + res[0] - res[2]);
  p->txs_bytes += res[1] - res[3];
  publish(p);
}

// a submitted device batch's statuses in (its decisions, appends and removals were made in
// submission order on the engine's stream), its list counts taken, its flight slot free
int finish_ticket(txv_pool* p, txv_pool::Ticket& t) {
  if (t.done) return t.err;
  const uint8_t* st;
  t.done = true;
  p->infl_len -= (int64_t)t.pushes;
  p->infl_bytes -= (int64_t)t.bytes;
  if ((t.err = pooldev_finish(t.ctx, p->dev, t.slot, &st, nullptr, nullptr))) return t.err;
  if (!t.upd) t.st.assign(st, st + t.n);
  list_counts(p, t.slot);
  return TXV_OK;
}

// the slot's previous batch, finished
int finish_slot(txv_pool* p, int slot) {
  for (auto& o : p->tickets)
    if (!o.done && o.slot == slot)
      if (int r = finish_ticket(p, o)) return r;
  return TXV_OK;
}

// staged Update entries with no CheckTx batch to ride: decided alone in their slot
int flush_pending(txv_pool* p) {
  if (!p->pend_n) return TXV_OK;
  txv_pool::Ticket t;
  t.upd = true;
  t.ctx = p->pend_ctx;
  t.slot = p->pend_slot;
  t.n_upd = p->pend_n;
  p->pend_n = 0;
  p->pend_slot = -1;
  if (int r = pooldev_enqueue(t.ctx, p->dev, t.slot, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, INT64_MAX,
                              false, false, nullptr, true, live_ub(p), t.n_upd))
    return r;
  if (p->cache_on) p->dev_state = txv_pool::kDevAhead;
  p->next_slot = (t.slot + 1) % kPdRing;
  p->tickets.push_back(std::move(t));
  return TXV_OK;
}

// every submitted device batch finished (statuses kept for their waits): the device and host
// copies can be synchronised, the pool list read
int drain_flights(txv_pool* p, bool flush) {
  int r = flush ? flush_pending(p) : TXV_OK;
  for (auto& t : p->tickets)
    if (!t.done) { const int e = finish_ticket(p, t); if (e && !r) r = e; }
  prune_updates(p);
  return r;
}

// a synchronous device batch of n votes from ctx: every submitted batch finished, the engine bound
// and current; the staged Update entries ride with it (their slot and count out) unless they came
// from another context or would not fit (then decided alone first)
int sync_batch_begin(txv_pool* p, txv_ctx* ctx, uint32_t n, int* slot, uint32_t* n_upd) {
  int r;
  if (p->pend_n && (p->pend_ctx != ctx || p->pend_n + n > pooldev_cap(p->dev)) && (r = flush_pending(p))) return r;
  if ((r = drain_flights(p, false))) return r;
  if ((r = cache_to_dev(p, ctx, p->pend_n + n))) return r;   // (a rebind flushes them)
  if ((r = list_to_dev(p, ctx))) return r;
  *slot = p->pend_n ? p->pend_slot : 0;                     // (every slot is free now)
  *n_upd = p->pend_n;
  p->pend_n = 0;
  p->pend_slot = -1;
  return TXV_OK;
}

}  // namespace

// CheckTxWithInfo for n decoded messages whose keys, sizes and decode statuses are in HBM (the
// wire ingest, runtime.cpp), enqueued on the context's key stream behind their decode: decided on
// the device when the pool keeps its cache there and the caps cannot bind even if all n pushed
// and their sizes summed to bytes_bound (*done = true; statuses for every message,
// TXV_POOL_NOT_CHECKED for those that did not decode; h_keys / h_sizes, the decode's copies back,
// are read once the statuses are in), else *done = false and the caller runs the host path.
// Takes p->mu.
int txv_pool_check_dev(txv_pool* p, txv_ctx* ctx, const uint32_t* d_keys, const uint32_t* d_sizes,
                       const uint8_t* d_valid, const uint8_t* h_keys, const uint32_t* h_sizes, uint8_t valid_ok,
                       uint32_t n, uint64_t bytes_bound, void* after, uint8_t* status_out, bool* done) {
  *done = false;
  std::lock_guard<std::mutex> g(p->mu);
  if (!dev_mode(p) || !n) return TXV_OK;
  const int64_t max_tx = (int64_t)p->cfg.max_msg_bytes - 8;
  if (!dev_caps_ok(p, n, bytes_bound)) return TXV_OK;
  int r, slot;
  uint32_t n_upd;
  if ((r = sync_batch_begin(p, ctx, n, &slot, &n_upd))) return r;
  if ((r = pooldev_check(ctx, p->dev, nullptr, nullptr, nullptr, d_keys, d_sizes, d_valid, valid_ok, n, max_tx,
                         (p->cfg.flags & TXV_POOL_WAL) != 0, nullptr, status_out, after, true, live_ub(p), slot, n_upd)))
    return r;
  if (p->cache_on) p->dev_state = txv_pool::kDevAhead;
  list_counts(p, slot);
  *done = true;
  return TXV_OK;
}

// The same, submitted (the wire ingest's split admit, runtime.cpp ingest_admit_submit): the
// decisions are enqueued into the engine's next flight slot behind `after` and the call returns
// with a pool ticket (*done = true) whose statuses txv_pool_check_wait collects -- so the admit
// thread hands batch k+1's CheckTx to the GPU while batch k's statuses are still on their way.
// The caps are checked against n pushes of bytes_bound bytes in all (upper bounds: the decode
// has not reported yet), beside the batches in flight.  *done = false: the host path is needed.
// d_status_copy (or null): the batch's statuses written to HBM there too, and then_stream (or null)
// made to wait for them -- the ingest's TxFlow chain reads them without a host round trip.
int txv_pool_check_dev_submit(txv_pool* p, txv_ctx* ctx, const uint32_t* d_keys, const uint32_t* d_sizes,
                              const uint8_t* d_valid, uint8_t valid_ok, uint32_t n, uint64_t bytes_bound, void* after,
                              uint8_t* d_status_copy, void* then_stream, uint64_t* ticket, bool* done) {
  *done = false;
  *ticket = 0;
  std::lock_guard<std::mutex> g(p->mu);
  if (!dev_mode(p) || !n) return TXV_OK;
  if (!dev_caps_ok(p, n, bytes_bound)) return TXV_OK;
  const int64_t max_tx = (int64_t)p->cfg.max_msg_bytes - 8;
  int r;
  p->batch_hint = std::max(p->batch_hint, n);
  if (p->pend_n && (p->pend_ctx != ctx || p->pend_n + n > pooldev_cap(p->dev)) && (r = flush_pending(p))) return r;
  if ((r = cache_to_dev(p, ctx, p->pend_n + n))) return r;
  if ((r = list_to_dev(p, ctx))) return r;
  const int slot = p->next_slot;                       // the staged Update entries' slot, if any
  const uint32_t n_upd = p->pend_n;
  if (!n_upd && (r = finish_slot(p, slot))) return r;  // its previous batch
  p->pend_n = 0;
  p->pend_slot = -1;
  if ((r = pooldev_enqueue(ctx, p->dev, slot, nullptr, nullptr, nullptr, d_keys, d_sizes, d_valid, valid_ok, n, max_tx,
                           (p->cfg.flags & TXV_POOL_WAL) != 0, false, after, true, live_ub(p), n_upd, d_status_copy,
                           then_stream)))
    return r;
  if (p->cache_on) p->dev_state = txv_pool::kDevAhead;
  p->next_slot = (slot + 1) % kPdRing;
  txv_pool::Ticket t;
  t.id = p->next_ticket;
  t.n = n;
  t.ctx = ctx;
  t.slot = slot;
  t.n_upd = n_upd;
  t.pushes = n;
  t.bytes = bytes_bound;
  p->infl_len += (int64_t)t.pushes;
  p->infl_bytes += (int64_t)t.bytes;
  p->tickets.push_back(std::move(t));
  *ticket = p->next_ticket++;
  *done = true;
  return TXV_OK;
}

// the pool's MaxMsgBytes (Reactor.Receive's decodeMsg cap, reactor.go:278-284)
uint32_t txv_pool_max_msg_bytes(txv_pool* p) {
  std::lock_guard<std::mutex> g(p->mu);
  return p->cfg.max_msg_bytes;
}

extern "C" {

// CheckTxWithInfo for n votes whose keys (n x 32 bytes) and Size() values are known (computed on
// the device from decoded wire records by txv_ingest_msgs, or by the caller); ctx may be NULL
// (the batch passes then run on the pool's own worker threads)
int txv_pool_check_keys(txv_pool* p, txv_ctx* ctx, const uint8_t* keys32, const uint32_t* sizes, uint32_t n,
                        uint8_t* status_out) {
  if (!p || (n && (!keys32 || !sizes || !status_out))) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(p->mu);
  if (dev_mode(p) && ctx && n) {   // the device path: keys and sizes uploaded, decided on the GPU
    const int64_t max_tx = (int64_t)p->cfg.max_msg_bytes - 8;
    uint64_t pushes = 0, bytes = 0;
    for (uint32_t i = 0; i < n; ++i) { pushes += (int64_t)sizes[i] <= max_tx; bytes += sizes[i]; }
    if (dev_caps_ok(p, pushes, bytes)) {
      int r, slot;
      uint32_t n_upd;
      if ((r = sync_batch_begin(p, ctx, n, &slot, &n_upd))) return r;
      if ((r = pooldev_check(ctx, p->dev, nullptr, keys32, sizes, nullptr, nullptr, nullptr, 0, n, max_tx,
                             (p->cfg.flags & TXV_POOL_WAL) != 0, nullptr, status_out, nullptr, true, live_ub(p), slot,
                             n_upd)))
        return r;
      if (p->cache_on) p->dev_state = txv_pool::kDevAhead;
      list_counts(p, slot);
      return TXV_OK;
    }
  }
  p->sizes.assign(sizes, sizes + n);
  return pool_admit(p, ctx, reinterpret_cast<const Key*>(keys32), n, status_out);
}

// CheckTxWithInfo for a batch, submitted: with TXV_POOL_DEVICE_CACHE (and no long signature,
// caps that cannot bind, a free flight slot) the keys, decisions and new cache are enqueued on
// the engine's stream and the call returns; otherwise the batch is checked on the host here (any
// device batches still in flight are finished first).  Either way the batch is CheckTx'd in
// submission order, and txv_pool_check_wait returns its statuses.
int txv_pool_check_submit(txv_pool* p, txv_ctx* ctx, const txv_votes* v, const uint8_t* sig_full,
                          const uint64_t* sig_full_off, uint64_t* ticket) {
  if (!p || !ctx || !v || !ticket) return TXV_EINVAL;
  *ticket = 0;
  const auto t0 = std::chrono::steady_clock::now();
  // the device path: Size() on the host workers (with the pushes, the bytes and any long
  // signature) before the pool's lock is taken (cfg is fixed at txv_pool_new), then keys,
  // decisions and the new cache enqueued on the GPU
  const bool dev = dev_mode(p) && v->n;
  const int64_t max_tx = (int64_t)p->cfg.max_msg_bytes - 8;
  std::vector<uint32_t> dsz;
  std::atomic<uint64_t> pushes{0}, bytes{0};
  std::atomic<bool> long_sig{false};
  if (dev) {
    dsz.resize(v->n);
    txv_host_parallel_for(ctx, v->n, [&](uint32_t lo, uint32_t hi) {
      uint64_t pu = 0, by = 0;
      bool lg = false;
      for (uint32_t i = lo; i < hi; ++i) {
        const uint32_t sz = vote_size(v, i);
        dsz[i] = sz;
        pu += (int64_t)sz <= max_tx;
        by += sz;
        lg |= v->sig_len[i] > 64;
      }
      pushes.fetch_add(pu, std::memory_order_relaxed);
      bytes.fetch_add(by, std::memory_order_relaxed);
      if (lg) long_sig.store(true, std::memory_order_relaxed);
    });
  }
  std::lock_guard<std::mutex> g(p->mu);
  txv_pool::Ticket t;
  t.id = p->next_ticket;
  t.n = v->n;
  t.ctx = ctx;
  p->sizes.resize(v->n);
  if (dev) {
    PTimer pt("check_submit");
    if (!long_sig.load() && dev_caps_ok(p, pushes.load(), bytes.load())) {
      int r;
      p->batch_hint = std::max(p->batch_hint, v->n);
      // staged Update entries from another context, or too many to ride with this batch, are decided
      // alone first (a rebind to a larger capacity would drain and reallocate mid-stream)
      if (p->pend_n && (p->pend_ctx != ctx || p->pend_n + v->n > pooldev_cap(p->dev)) && (r = flush_pending(p))) return r;
      if ((r = cache_to_dev(p, ctx, p->pend_n + v->n))) return r;
      if ((r = list_to_dev(p, ctx))) return r;
      const int slot = p->next_slot;                       // the staged Update entries' slot, if any
      const uint32_t n_upd = p->pend_n;
      if (!n_upd && (r = finish_slot(p, slot))) return r;  // its previous batch (staging finished it)
      pt.mark("prev");
      p->pend_n = 0;
      p->pend_slot = -1;
      if ((r = pooldev_enqueue(ctx, p->dev, slot, v, nullptr, dsz.data(), nullptr, nullptr, nullptr, 0, v->n, max_tx,
                               (p->cfg.flags & TXV_POOL_WAL) != 0, false, nullptr, true, live_ub(p), n_upd)))
        return r;
      t.n_upd = n_upd;
      pooldev_set_occupant(p->dev, slot, t.id, n_upd, v->n);   // txv_submit_checked may read it from HBM
      pt.mark("enqueue");
      if (p->cache_on) p->dev_state = txv_pool::kDevAhead;
      p->next_slot = (slot + 1) % kPdRing;
      t.slot = slot;
      t.pushes = pushes.load();
      t.bytes = bytes.load();
      p->infl_len += (int64_t)t.pushes;
      p->infl_bytes += (int64_t)t.bytes;
      p->tickets.push_back(std::move(t));
      *ticket = p->next_ticket++;
      return TXV_OK;
    }
  }
  // the host path: TxVote.Size() of every vote on the worker threads while the GPU hashes
  int r = batch_keys(p, ctx, v, sig_full, sig_full_off, [&] {
    txv_host_parallel_for(ctx, v->n, [&](uint32_t lo, uint32_t hi) {
      for (uint32_t i = lo; i < hi; ++i) p->sizes[i] = vote_size(v, i);
    });
  });
  if (r) return r;
  const Key* keys = reinterpret_cast<const Key*>(p->keys.data());
  if (getenv("TXV_PROFILE_HOST"))
    fprintf(stderr, "[txv pool] keys+sizes=%.3fms n=%u\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), v->n);
  t.st.resize(v->n);
  if ((r = pool_admit(p, ctx, keys, v->n, t.st.data()))) return r;
  t.done = true;
  p->tickets.push_back(std::move(t));
  *ticket = p->next_ticket++;
  return TXV_OK;
}

// TryAddVote for the batch a CheckTx ticket is deciding (include/txvote.h): while the batch is in
// the engine's flight slot its signatures and statuses are read there on the GPU (the TxFlow chain
// queued behind the decisions, no host round trip, no second upload); otherwise the ticket's
// statuses are taken on the host (waiting for them if need be) and the caller's columns staged.
// The pool ticket stays the caller's to wait (txv_pool_check_wait).  Takes p->mu, then the
// context's lock.
int txv_submit_checked(txv_ctx* ctx, const txv_votes* v, txv_pool* p, uint64_t pool_ticket, uint64_t* ticket) {
  if (!ctx || !v || !p || !pool_ticket || !ticket) return TXV_EINVAL;
  std::lock_guard<std::mutex> so(txv_ctx_submit_mu(ctx));   // no other submit between the steps
  uint32_t slot;
  int r;
  if ((r = submit_checked_stage(ctx, v, &slot))) return r;   // the host staging: no pool lock held
  std::vector<uint8_t> st;
  int why = 0;
  bool consumed = false;
  {
    std::lock_guard<std::mutex> g(p->mu);
    // the reads of the engine's slot are enqueued under the pool's lock: a later writer of the
    // slot (also under it) waits for them on the GPU
    if (p->dev && pooldev_same_device(ctx, p->dev) && pooldev_holds(p->dev, pool_ticket)) {
      if ((r = submit_checked_consume(ctx, slot, p->dev, pool_ticket, v)) < 0) return r;
      consumed = r == 0;
    }
  }
  if (consumed) return submit_checked_run(ctx, slot, v, nullptr, 0, ticket);
  {
    std::lock_guard<std::mutex> g(p->mu);
    auto it = std::find_if(p->tickets.begin(), p->tickets.end(), [&](const txv_pool::Ticket& t) { return t.id == pool_ticket; });
    if (it == p->tickets.end()) {                  // waited already: its statuses, if still kept
      why = 1;
      for (const auto& rc : p->recent)
        if (rc.first == pool_ticket) {
          why = rc.second.size() != v->n ? 2 : 0;
          if (!why) st = rc.second;
        }
    } else if (it->upd) {
      why = 1;
    } else if (it->n != v->n) {
      why = 2;
    } else {
      if (!it->done)
        for (auto jt = p->tickets.begin(); jt != p->tickets.end(); ++jt) {   // the earlier ones first: append order
          if (int e = finish_ticket(p, *jt)) return e;
          if (jt == it) break;
        }
      if (it->err) return it->err;
      st = it->st;
    }
  }
  return submit_checked_run(ctx, slot, v, why ? nullptr : st.data(), why, ticket);
}

// txv_route_admitted for the batch a CheckTx ticket is deciding (include/txvote.h): the route
// kernels read its statuses and signatures in HBM behind the decisions while the batch is in the
// engine's flight slot, else the ticket's host statuses and the caller's signatures.  Takes the
// context's route lock, then the pool's, then the context's.
int txv_route_checked(txv_ctx* ctx, const txv_votes* v, txv_pool* p, uint64_t pool_ticket, uint32_t n_shards,
                      void* dst_dev, uint64_t stride, txv_route_meta* meta_out) {
  if (!ctx || !v || !p || !pool_ticket || !dst_dev || !meta_out || !n_shards || n_shards > 255) return TXV_EINVAL;
  if (v->n && (!v->height || !v->txhash || !v->txhash_off || !v->txhash_len || !v->ts_sec || !v->ts_nanos || !v->addr ||
               !v->addr_len || !v->sig || !v->sig_len))
    return TXV_EINVAL;
  std::lock_guard<std::mutex> rl(txv_ctx_route_mu(ctx));
  int r;
  if ((r = route_checked_stage(ctx, v, stride))) return r;
  std::vector<uint8_t> st;
  bool consumed = false;
  {
    std::lock_guard<std::mutex> g(p->mu);
    if (p->dev && pooldev_same_device(ctx, p->dev) && pooldev_holds(p->dev, pool_ticket)) {
      if ((r = route_checked_consume(ctx, p->dev, pool_ticket, v->n)) < 0) return r;
      consumed = r == 0;
    }
    if (!consumed) {
      auto it = std::find_if(p->tickets.begin(), p->tickets.end(), [&](const txv_pool::Ticket& t) { return t.id == pool_ticket; });
      if (it == p->tickets.end()) {
        for (const auto& rc : p->recent)
          if (rc.first == pool_ticket) st = rc.second;
        if (st.empty() && v->n) return txv_ctx_fail(ctx, TXV_ESTATE, "txv_route_checked: unknown pool ticket (already waited?)");
      } else if (it->upd) {
        return txv_ctx_fail(ctx, TXV_ESTATE, "txv_route_checked: unknown pool ticket");
      } else {
        if (!it->done)
          for (auto jt = p->tickets.begin(); jt != p->tickets.end(); ++jt) {
            if (int e = finish_ticket(p, *jt)) return e;
            if (jt == it) break;
          }
        if (it->err) return it->err;
        st = it->st;
      }
      if (st.size() != v->n) return txv_ctx_fail(ctx, TXV_EINVAL, "txv_route_checked: the batch differs from the pool ticket's");
    }
  }
  return route_checked_launch(ctx, v, consumed ? nullptr : st.data(), n_shards, dst_dev, stride, meta_out);
}

// the statuses of a submitted batch (tickets in submission order); the engine's event is waited
// for without p->mu held, so batch k+1 can be submitted meanwhile
int txv_pool_check_wait(txv_pool* p, uint64_t ticket, uint8_t* status_out) {
  if (!p || !ticket) return TXV_EINVAL;
  txv_ctx* ctx = nullptr;
  PoolDev* dev = nullptr;
  int slot = -1;
  {
    std::lock_guard<std::mutex> g(p->mu);
    auto it = std::find_if(p->tickets.begin(), p->tickets.end(), [&](const txv_pool::Ticket& t) { return t.id == ticket; });
    if (it == p->tickets.end()) return TXV_ESTATE;
    if (!it->done) { ctx = it->ctx; slot = it->slot; dev = p->dev; ++p->waiters; }
  }
  PTimer pt("check_wait");
  if (slot >= 0) (void)pooldev_finish(ctx, dev, slot, nullptr, nullptr, nullptr);   // the wait itself
  pt.mark("gpu");
  std::lock_guard<std::mutex> g(p->mu);
  pt.mark("lock");
  if (slot >= 0 && --p->waiters == 0) {
    for (PoolDev* d : p->retired) pooldev_free(d);
    p->retired.clear();
  }
  int r = TXV_OK;
  for (auto it = p->tickets.begin(); it != p->tickets.end(); ++it) {   // the earlier ones first: append order
    const int e = finish_ticket(p, *it);
    if (it->id != ticket) continue;
    r = e;
    if (!r && it->n && status_out) memcpy(status_out, it->st.data(), it->n);
    if (!r && !it->upd) {
      if (p->recent.size() >= 8) p->recent.pop_front();
      p->recent.emplace_back(it->id, std::move(it->st));
    }
    p->tickets.erase(it);
    prune_updates(p);
    pt.mark("finish");
    return r;
  }
  return TXV_ESTATE;
}

int txv_pool_check(txv_pool* p, txv_ctx* ctx, const txv_votes* v, const uint8_t* sig_full,
                   const uint64_t* sig_full_off, uint8_t* status_out) {
  if (!p || !ctx || !v || (v->n && !status_out)) return TXV_EINVAL;
  uint64_t t = 0;
  int r = txv_pool_check_submit(p, ctx, v, sig_full, sig_full_off, &t);
  if (r) return r;
  return txv_pool_check_wait(p, t, status_out);
}

// the order-independent half of CheckTxWithInfo for a batch (txvotepool.go:187-261): every vote's
// txVoteKey (SHA-256(Signature), GPU) and TxVote.Size() (host workers, while the GPU hashes).  No
// pool state is read or written, so a caller may prepare batch k+1 on one thread while
// txv_pool_check_keys admits batch k on another (bench.py's C5 leg)
int txv_pool_prepare(txv_pool* p, txv_ctx* ctx, const txv_votes* v, const uint8_t* sig_full,
                     const uint64_t* sig_full_off, uint8_t* keys_out, uint32_t* sizes_out) {
  if (!p || !ctx || !v || (v->n && (!keys_out || !sizes_out))) return TXV_EINVAL;
  return txv_sig_keys_overlap(ctx, v, sig_full, sig_full_off, keys_out, [&] {
    txv_host_parallel_for(ctx, v->n, [&](uint32_t lo, uint32_t hi) {
      for (uint32_t i = lo; i < hi; ++i) sizes_out[i] = vote_size(v, i);
    });
  });
}

// Update (txvotepool.go:329-359) with the cache and the pool list in HBM: the committed votes'
// keys (SHA-256 of the signatures) are hashed, pushed (every key: cache.Push ignores Size) and
// removed from the pool list by the device engine in stream order behind the batches submitted
// before -- no flight is drained, nothing is copied back but the removal counts.  Size and
// TxsBytes follow once the tickets submitted before are finished (txv_pool_check_wait,
// txv_pool_sync, any reader).  Signatures > 64 bytes take the host path.
int update_submit_dev(txv_pool* p, txv_ctx* ctx, const txv_votes* v, const uint32_t* sizes) {
  const uint32_t n = v->n;
  PTimer pt("update_submit");
  int r;
  // room for the next CheckTx batch beside the staged entries, so they ride with it instead of
  // being decided alone (a chain of their own) when it comes.  Updates that stack up before the
  // next batch and would overflow that room are decided alone first rather than growing the
  // engine: a growth drains every flight and reallocates its pinned buffers (≈ 0.1 s at 1M
  // entries), so the engine grows only for a single Update larger than any before
  if (p->pend_n && (p->pend_ctx != ctx || (p->dev && p->pend_n + n + p->batch_hint > pooldev_cap(p->dev))) &&
      (r = flush_pending(p)))
    return r;
  if ((r = cache_to_dev(p, ctx, p->pend_n + n + p->batch_hint))) return r;   // (a rebind drains: pend_n is 0 then)
  if ((r = list_to_dev(p, ctx))) return r;
  if (!p->pend_n) {                                        // a slot for the entries: its previous batch finished
    if ((r = finish_slot(p, p->next_slot))) return r;
    prune_updates(p);
    p->pend_slot = p->next_slot;
    p->pend_ctx = ctx;
  }
  pt.mark("prev");
  if ((r = pooldev_stage(ctx, p->dev, p->pend_slot, p->pend_n, v, sizes))) return r;
  p->pend_n += n;
  pt.mark("stage");
  return TXV_OK;
}

// Update with the committed votes' keys and Size() values known (every flight and append
// drained first, the cache brought to the host)
int update_host_keys(txv_pool* p, txv_ctx* ctx, const Key* keys, const uint32_t* sizes, uint32_t n) {
  int r;
  if ((r = drain_flights(p))) return r;
  if ((r = list_to_host(p, ctx))) return r;
  if ((r = cache_to_host(p, ctx))) return r;
  host_cache_written(p);
  PTimer pt("update_host");
  if (p->cache_on)                                 // cache.Push of every committed key, in order
    for (uint32_t i = 0; i < n; ++i) {
      if (i + 16 < n) p->cache_map.prefetch(keys[i + 16]);
      (void)p->cache_push(keys[i]);
    }
  pt.mark("cache");
  size_t removed = 0;                              // removeTx(tx, e, false) of the ones the pool holds
  p->txs_bytes -= remove_keys(p, ctx, keys, sizes, n, &removed);
  p->txs.len -= removed;
  publish_locked(p);
  pt.mark("remove");
  return TXV_OK;
}

int update_host(txv_pool* p, txv_ctx* ctx, const txv_votes* v, const uint8_t* sig_full, const uint64_t* sig_full_off) {
  int r = batch_keys(p, ctx, v, sig_full, sig_full_off);
  if (r) return r;
  std::vector<uint32_t> sz(v->n);
  pool_parallel_for(p, ctx, v->n, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; ++i) sz[i] = vote_size(v, i);
  }, 4096);
  return update_host_keys(p, ctx, reinterpret_cast<const Key*>(p->keys.data()), sz.data(), v->n);
}

int txv_pool_update_submit(txv_pool* p, txv_ctx* ctx, int64_t height, const txv_votes* v, const uint8_t* sig_full,
                           const uint64_t* sig_full_off) {
  if (!p || !ctx || !v || (v->n && (!v->sig || !v->sig_len))) return TXV_EINVAL;
  // the device path's TxVote.Size() values before the pool's lock is taken
  std::vector<uint32_t> dsz;
  bool lg = false;
  if (dev_mode(p) && v->n) {
    for (uint32_t i = 0; i < v->n && !lg; ++i) lg = v->sig_len[i] > 64;
    if (!lg) {
      dsz.resize(v->n);
      auto fill = [&](uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; ++i) dsz[i] = vote_size(v, i);
      };
      if (ctx) txv_host_parallel_for(ctx, v->n, fill);
      else fill(0, v->n);
    }
  }
  std::lock_guard<std::mutex> g(p->mu);
  p->height = height;
  if (!dsz.empty()) return update_submit_dev(p, ctx, v, dsz.data());
  return update_host(p, ctx, v, sig_full, sig_full_off);
}

// Update applied when it returns: the device path's submission, then every ticket up to it
// finished (no cache or list copy back)
int txv_pool_update(txv_pool* p, txv_ctx* ctx, int64_t height, const txv_votes* v, const uint8_t* sig_full,
                    const uint64_t* sig_full_off) {
  int r = txv_pool_update_submit(p, ctx, height, v, sig_full, sig_full_off);
  if (r || !dev_mode(p)) return r;
  std::lock_guard<std::mutex> g(p->mu);
  return drain_flights(p);
}

// Update with the committed votes given as (txVoteKey, Size()) pairs (the keys computed by the
// caller, as for txv_pool_check_keys); applied when it returns, ctx optional
int txv_pool_update_keys(txv_pool* p, txv_ctx* ctx, int64_t height, const uint8_t* keys32, const uint32_t* sizes,
                         uint32_t n) {
  if (!p || (n && (!keys32 || !sizes))) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(p->mu);
  p->height = height;
  return update_host_keys(p, ctx, reinterpret_cast<const Key*>(keys32), sizes, n);
}

int txv_pool_reap(txv_pool* p, int64_t max, uint8_t* keys_out, uint32_t* sizes_out, uint64_t cap, uint64_t* n_out) {
  if (!p) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(p->mu);
  if (int r = drain_flights(p)) return r;
  if (int r = list_to_host(p, nullptr)) return r;
  if (max < 0) max = (int64_t)p->txs.len;
  uint64_t n = 0;
  for (int32_t e = p->txs.head; e >= 0 && (int64_t)n <= max; e = p->txs.nodes[e].next, ++n) {
    if (n < cap) {
      if (keys_out) memcpy(keys_out + 32 * n, p->txs.nodes[e].k.b, 32);
      if (sizes_out) sizes_out[n] = p->txs.nodes[e].size;
    }
  }
  if (n_out) *n_out = n;
  return TXV_OK;
}

int txv_pool_receive(txv_pool* p, txv_ctx* ctx, const uint8_t* wire, uint64_t wire_bytes, const uint64_t* msg_off,
                     const uint32_t* msg_len, uint32_t n, uint8_t* wire_status, uint8_t* pool_status) {
  if (!p || !ctx || (n && (!wire_status || !pool_status))) return TXV_EINVAL;
  // decodeMsg for the batch (GPU), then the decoded TxVoteMessages in arrival order
  std::vector<int64_t> height(n), ts_sec(n);
  std::vector<int32_t> ts_nanos(n);
  std::vector<uint32_t> th_off(n), th_len(n), addr_len(n), sig_len(n);
  std::vector<uint64_t> sig_off(n);
  std::vector<uint8_t> addr((size_t)n * 20), sig((size_t)n * 64);
  txv_wire_votes w{};
  w.status = wire_status; w.height = height.data(); w.txhash_off = th_off.data(); w.txhash_len = th_len.data();
  w.ts_sec = ts_sec.data(); w.ts_nanos = ts_nanos.data(); w.addr = addr.data(); w.addr_len = addr_len.data();
  w.sig = sig.data(); w.sig_len = sig_len.data(); w.sig_off = sig_off.data();
  uint32_t max_msg;
  {
    std::lock_guard<std::mutex> g(p->mu);
    max_msg = p->cfg.max_msg_bytes;
  }
  int r = txv_decode_msgs(ctx, wire, wire_bytes, msg_off, msg_len, n, max_msg, &w);
  if (r) return r;
  std::vector<uint32_t> ok;   // compact the decoded messages (the others never reach CheckTx)
  ok.reserve(n);
  for (uint32_t i = 0; i < n; ++i) {
    pool_status[i] = TXV_POOL_NOT_CHECKED;
    if (wire_status[i] == TXV_WIRE_OK) ok.push_back(i);
  }
  if (ok.empty()) return TXV_OK;
  if (ok.size() != n) {
    for (size_t j = 0; j < ok.size(); ++j) {
      const uint32_t i = ok[j];
      height[j] = height[i]; ts_sec[j] = ts_sec[i]; ts_nanos[j] = ts_nanos[i]; th_off[j] = th_off[i];
      th_len[j] = th_len[i]; addr_len[j] = addr_len[i]; sig_len[j] = sig_len[i]; sig_off[j] = sig_off[i];
      memmove(addr.data() + j * 20, addr.data() + (size_t)i * 20, 20);
      memmove(sig.data() + j * 64, sig.data() + (size_t)i * 64, 64);
    }
  }
  txv_votes v{};
  v.n = (uint32_t)ok.size();
  v.height = height.data(); v.txhash = wire; v.txhash_off = th_off.data(); v.txhash_len = th_len.data();
  v.ts_sec = ts_sec.data(); v.ts_nanos = ts_nanos.data(); v.addr = addr.data(); v.addr_len = addr_len.data();
  v.sig = sig.data(); v.sig_len = sig_len.data();
  std::vector<uint8_t> st(v.n);
  r = txv_pool_check(p, ctx, &v, wire, sig_off.data(), st.data());
  if (r) return r;
  for (size_t j = 0; j < ok.size(); ++j) pool_status[ok[j]] = st[j];
  return TXV_OK;
}

int txv_encode_msgs(const txv_votes* v, const uint8_t* txkey, const uint8_t* sig_full, const uint64_t* sig_full_off,
                    uint8_t* out, uint64_t cap, uint64_t* off_out, uint32_t* len_out, uint64_t* bytes_out) {
  if (!v || (v->n && (!off_out || !len_out))) return TXV_EINVAL;
  uint8_t disamb[3], prefix[4];
  txvote_msg_disfix(disamb, prefix);
  uint64_t total = 0;
  for (uint32_t i = 0; i < v->n; ++i) {   // lengths and offsets
    if ((v->is_nil && v->is_nil[i]) || v->addr_len[i] > 20 || (v->sig_len[i] > 64 && (!sig_full || !sig_full_off)))
      return TXV_EINVAL;
    const int64_t m = txv_host::txvote_msg(nullptr, prefix, v->height[i], nullptr, v->txhash_len[i], nullptr,
                                          v->ts_sec[i], v->ts_nanos[i], nullptr, v->addr_len[i], nullptr, v->sig_len[i]);
    if (m < 0) return TXV_EINVAL;           // MustMarshalBinaryBare panics
    off_out[i] = total;
    len_out[i] = (uint32_t)m;
    total += (uint64_t)m;
  }
  if (bytes_out) *bytes_out = total;
  if (total > cap || (total && !out)) return TXV_ECAPACITY;
  const uint32_t n = v->n;
  const uint32_t nt = std::max(1u, std::min<uint32_t>(16, n / 16384));
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nt; ++t) {
    auto part = [&, t] {
      for (uint32_t i = (uint32_t)((uint64_t)n * t / nt); i < (uint32_t)((uint64_t)n * (t + 1) / nt); ++i) {
        const uint8_t* sig = v->sig_len[i] > 64 ? sig_full + sig_full_off[i] : v->sig + (size_t)i * 64;
        txv_host::txvote_msg(out + off_out[i], prefix, v->height[i], v->txhash + v->txhash_off[i], v->txhash_len[i],
                             txkey ? txkey + (size_t)i * 32 : nullptr, v->ts_sec[i], v->ts_nanos[i],
                             v->addr + (size_t)i * 20, v->addr_len[i], sig, v->sig_len[i]);
      }
    };
    try {
      th.emplace_back(part);
    } catch (const std::system_error&) {
      part();
    }
  }
  for (auto& x : th) x.join();
  return TXV_OK;
}

int txv_pool_flush(txv_pool* p) {
  if (!p) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(p->mu);
  (void)drain_flights(p);
  p->cache.clear(); p->cache_map.clear();
  host_cache_written(p);
  p->txs.clear(); p->txs_map.clear();
  p->list_dev = false;                                     // the device's copy is dropped (re-sent empty)
  p->txs_bytes = 0;
  publish_locked(p);
  return TXV_OK;
}

int txv_pool_sync(txv_pool* p) {
  if (!p) return TXV_EINVAL;
  int r;
  {
    std::lock_guard<std::mutex> g(p->mu);
    if (p->pend_n || std::any_of(p->tickets.begin(), p->tickets.end(), [](const txv_pool::Ticket& t) { return t.upd || t.n_upd; }))
      if ((r = drain_flights(p))) return r;               // submitted Updates applied
  }
  return TXV_OK;
}

// Size / TxsBytes as of the last finished batch
int64_t txv_pool_size(txv_pool* p) {
  return p ? p->pub_len.load(std::memory_order_relaxed) : 0;
}
int64_t txv_pool_txs_bytes(txv_pool* p) {
  return p ? p->pub_bytes.load(std::memory_order_relaxed) : 0;
}
int64_t txv_pool_height(txv_pool* p) { return p ? p->height : 0; }

int txv_pool_cache_keys(txv_pool* p, uint8_t* keys_out, uint64_t cap, uint64_t* n_out) {
  if (!p) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(p->mu);
  if (int r = drain_flights(p)) return r;
  if (int r = cache_to_host(p, nullptr)) return r;
  uint64_t n = 0;
  for (int32_t e = p->cache.head; e >= 0; e = p->cache.nodes[e].next, ++n)
    if (keys_out && n < cap) memcpy(keys_out + 32 * n, p->cache.nodes[e].k.b, 32);
  if (n_out) *n_out = n;
  return TXV_OK;
}

}  // extern "C"
