// host_pack.hpp — the host side of batch admission, built for 64k..1M-vote batches:
//
//   * WorkerPool: persistent threads + parallel_for over vote ranges (the pack of a batch
//     is embarrassingly parallel except the TxHash routing, which stays sequential because
//     set ids are assigned in first-seen order, txflow/service.go:200-209).
//   * TxTable: TxHash bytes -> dense TxVoteSet id (open addressing, keys in one arena, seeded
//     64-bit hash so crafted TxHash strings cannot force long probe chains).
//   * AddrTable: 20-byte validator address -> validator index (ValidatorSet.GetByAddress,
//     tendermint, called at types/vote_set.go:102), read-only during a pack.
#pragma once
#include <stdint.h>
#include <string.h>

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace txv_host {

// ------------------------------------------------------------------ hashing
inline uint64_t load64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
inline uint64_t mix64(uint64_t x) {
  x ^= x >> 32; x *= 0xd6e8feb86659fd93ULL; x ^= x >> 32; x *= 0xd6e8feb86659fd93ULL; x ^= x >> 32;
  return x;
}
inline uint64_t hash_bytes(const uint8_t* p, uint32_t n, uint64_t seed) {
  uint64_t h = seed ^ (0x9e3779b97f4a7c15ULL * (n + 1));
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8) h = mix64(h ^ load64(p + i)) + 0x9e3779b97f4a7c15ULL;
  if (i < n) {
    uint64_t t = 0;
    memcpy(&t, p + i, n - i);
    h = mix64(h ^ t ^ ((uint64_t)(n - i) << 56));
  }
  return mix64(h);
}

// ------------------------------------------------------------------ worker pool
class WorkerPool {
 public:
  explicit WorkerPool(unsigned n) {
    for (unsigned t = 1; t < n; ++t) th_.emplace_back([this] { loop(); });
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  unsigned size() const { return (unsigned)th_.size() + 1; }
  // pin every worker thread to `set` (the GPU-local NUMA node's CPUs); false if any call failed
  bool set_affinity(const cpu_set_t& set) {
    bool ok = true;
    for (auto& t : th_) ok &= pthread_setaffinity_np(t.native_handle(), sizeof(cpu_set_t), &set) == 0;
    return ok;
  }
  // fn(lo, hi) over [0, n) in chunks; the caller thread takes part.  Small n runs inline.
  // Each call is its own Job: a worker still draining an earlier job only sees that job's
  // (exhausted) counters, never the new one's.
  void parallel_for(uint32_t n, const std::function<void(uint32_t, uint32_t)>& fn, uint32_t min_chunk = 2048) {
    const uint32_t parts = std::min<uint32_t>(size() * 4, std::max<uint32_t>(1, n / min_chunk));
    if (parts <= 1 || th_.empty()) { if (n) fn(0, n); return; }
    auto job = std::make_shared<Job>();
    job->fn = &fn; job->n = n; job->parts = parts;
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = job;
      ++gen_;
    }
    cv_.notify_all();
    work(*job);
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [&] { return job->done.load() == job->parts; });
    job_.reset();
  }

 private:
  struct Job {
    const std::function<void(uint32_t, uint32_t)>* fn = nullptr;
    uint32_t n = 0, parts = 0;
    std::atomic<uint32_t> next{0}, done{0};
  };
  void work(Job& j) {
    for (;;) {
      const uint32_t p = j.next.fetch_add(1);
      if (p >= j.parts) return;
      const uint32_t lo = (uint32_t)((uint64_t)j.n * p / j.parts), hi = (uint32_t)((uint64_t)j.n * (p + 1) / j.parts);
      (*j.fn)(lo, hi);
      if (j.done.fetch_add(1) + 1 == j.parts) {
        std::lock_guard<std::mutex> g(m_);
        done_cv_.notify_all();
      }
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        j = job_;
      }
      if (j) work(*j);
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::shared_ptr<Job> job_;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// ------------------------------------------------------------------ parallel stable counting sort
// Items [0, n) with key(i) in [0, K) (UINT32_MAX = drop) are scattered by emit(pos, i) into key
// order, arrival order kept inside each key: per-chunk histograms (contiguous chunks), one
// exclusive scan over (key, chunk), per-chunk scatter.  Returns the number of items kept;
// starts (optional, K + 1 entries) receives each key's first position.
template <class KeyF, class EmitF>
uint32_t counting_sort(WorkerPool& pool, uint32_t n, uint32_t K, KeyF key, EmitF emit, uint32_t* starts = nullptr) {
  const uint32_t P = std::max<uint32_t>(1, std::min<uint32_t>(pool.size() * 2, n / 8192));
  std::vector<uint32_t> hist((size_t)P * K, 0);
  auto range = [&](uint32_t p, uint32_t& lo, uint32_t& hi) {
    lo = (uint32_t)((uint64_t)n * p / P); hi = (uint32_t)((uint64_t)n * (p + 1) / P);
  };
  pool.parallel_for(P, [&](uint32_t p0, uint32_t p1) {
    for (uint32_t p = p0; p < p1; ++p) {
      uint32_t lo, hi;
      range(p, lo, hi);
      uint32_t* hp = hist.data() + (size_t)p * K;
      for (uint32_t i = lo; i < hi; ++i) {
        const uint32_t k = key(i);
        if (k != UINT32_MAX) hp[k]++;
      }
    }
  }, 1);
  uint32_t run = 0;
  for (uint32_t k = 0; k < K; ++k) {
    if (starts) starts[k] = run;
    for (uint32_t p = 0; p < P; ++p) {
      uint32_t& c = hist[(size_t)p * K + k];
      const uint32_t t = c;
      c = run;
      run += t;
    }
  }
  if (starts) starts[K] = run;
  pool.parallel_for(P, [&](uint32_t p0, uint32_t p1) {
    for (uint32_t p = p0; p < p1; ++p) {
      uint32_t lo, hi;
      range(p, lo, hi);
      uint32_t* hp = hist.data() + (size_t)p * K;
      for (uint32_t i = lo; i < hi; ++i) {
        const uint32_t k = key(i);
        if (k != UINT32_MAX) emit(hp[k]++, i);
      }
    }
  }, 1);
  return run;
}

// ------------------------------------------------------------------ TxHash -> set id
class TxTable {
 public:
  explicit TxTable(uint64_t seed = 0x7478666c6f77ULL) : seed_(seed) { rehash(1024); }
  uint64_t hash(const uint8_t* k, uint32_t n) const { return hash_bytes(k, n, seed_); }
  // id of key (hash h = hash(k, n)), or UINT32_MAX
  uint32_t find(const uint8_t* k, uint32_t n, uint64_t h) const {
    for (uint64_t i = h & mask_;; i = (i + 1) & mask_) {
      const Slot& s = slots_[i];
      if (!s.id1) return UINT32_MAX;
      if (s.h == h && len_[s.id1 - 1] == n && !memcmp(arena_.data() + off_[s.id1 - 1], k, n)) return s.id1 - 1;
    }
  }
  // id of key, inserting it with the next id when absent (*created = true); UINT32_MAX when
  // absent and the table already holds `limit` keys
  uint32_t intern(const uint8_t* k, uint32_t n, uint64_t h, bool* created, uint32_t limit = UINT32_MAX) {
    uint64_t i = h & mask_;
    for (;; i = (i + 1) & mask_) {
      const Slot& s = slots_[i];
      if (!s.id1) break;
      if (s.h == h && len_[s.id1 - 1] == n && !memcmp(arena_.data() + off_[s.id1 - 1], k, n)) {
        *created = false;
        return s.id1 - 1;
      }
    }
    *created = false;
    if (off_.size() >= limit) return UINT32_MAX;
    const uint32_t id = (uint32_t)off_.size();
    off_.push_back(arena_.size());
    len_.push_back(n);
    arena_.insert(arena_.end(), k, k + n);
    slots_[i] = Slot{h, id + 1};
    *created = true;
    if ((uint64_t)(id + 1) * 2 > mask_ + 1) rehash((mask_ + 1) * 2);
    return id;
  }
  uint32_t size() const { return (uint32_t)off_.size(); }
  void clear() {
    off_.clear(); len_.clear(); arena_.clear();
    slots_.clear();
    rehash(1024);
  }

 private:
  struct Slot { uint64_t h; uint32_t id1; };
  void rehash(uint64_t cap) {
    std::vector<Slot> ns(cap, Slot{0, 0});
    const uint64_t m = cap - 1;
    for (const Slot& s : slots_) {
      if (!s.id1) continue;
      uint64_t i = s.h & m;
      while (ns[i].id1) i = (i + 1) & m;
      ns[i] = s;
    }
    slots_.swap(ns);
    mask_ = m;
  }
  uint64_t seed_;
  std::vector<Slot> slots_;
  uint64_t mask_ = 0;
  std::vector<uint64_t> off_;
  std::vector<uint32_t> len_;
  std::vector<uint8_t> arena_;
};

// ------------------------------------------------------------------ address -> validator
class AddrTable {
 public:
  void build(const uint8_t* addrs20, uint32_t n) {
    uint64_t cap = 16;
    while (cap < (uint64_t)n * 4) cap *= 2;
    mask_ = cap - 1;
    slots_.assign(cap, UINT32_MAX);
    keys_.assign(addrs20, addrs20 + (size_t)n * 20);
    for (uint32_t v = 0; v < n; ++v) {
      uint64_t i = hash_bytes(addrs20 + 20 * (size_t)v, 20, kSeed) & mask_;
      bool dup = false;
      for (; slots_[i] != UINT32_MAX; i = (i + 1) & mask_)
        if (!memcmp(keys_.data() + 20 * (size_t)slots_[i], addrs20 + 20 * (size_t)v, 20)) { dup = true; break; }
      if (!dup) slots_[i] = v;   // first index wins for a repeated address
    }
  }
  uint32_t find(const uint8_t* a) const {
    if (slots_.empty()) return UINT32_MAX;
    for (uint64_t i = hash_bytes(a, 20, kSeed) & mask_; slots_[i] != UINT32_MAX; i = (i + 1) & mask_)
      if (!memcmp(keys_.data() + 20 * (size_t)slots_[i], a, 20)) return slots_[i];
    return UINT32_MAX;
  }
  void clear() { slots_.clear(); keys_.clear(); }

 private:
  static constexpr uint64_t kSeed = 0x61646472ULL;
  std::vector<uint32_t> slots_;
  std::vector<uint8_t> keys_;
  uint64_t mask_ = 0;
};

}  // namespace txv_host
