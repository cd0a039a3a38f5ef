// host_pack.hpp — the host side of batch admission, built for 64k..1M-vote batches:
//
//   * WorkerPool: persistent threads + parallel_for over vote ranges (the staging copies of a
//     batch into pinned memory, the verify-only packs).
//   * AddrTable: 20-byte validator address -> validator index (ValidatorSet.GetByAddress,
//     tendermint, called at types/vote_set.go:102); its slots are uploaded for the device
//     lookup of the AddVote path (kernels_flow.hip) and used directly by the verify-only paths.
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
#include <system_error>
#include <thread>
#include <vector>

#include "txv_hash.h"

namespace txv_host {

// ------------------------------------------------------------------ hashing
inline uint64_t load64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
inline uint64_t mix64(uint64_t x) {
  x ^= x >> 32; x *= 0xd6e8feb86659fd93ULL; x ^= x >> 32; x *= 0xd6e8feb86659fd93ULL; x ^= x >> 32;
  return x;
}
// the same function the device uses for the set table and the validator address table
inline uint64_t hash_bytes(const uint8_t* p, uint32_t n, uint64_t seed) {
  return txv_hash::hash_chunks(n, seed, [&](uint32_t i) {
    uint64_t t = 0;
    memcpy(&t, p + i, std::min<uint32_t>(8, n - i));
    return t;
  });
}

// ------------------------------------------------------------------ worker pool
class WorkerPool {
 public:
  explicit WorkerPool(unsigned n) {
    // a thread that cannot be created (EAGAIN under a process/thread limit) leaves a smaller
    // pool; parallel_for runs inline with none
    for (unsigned t = 1; t < n; ++t) {
      try {
        th_.emplace_back([this] { loop(); });
      } catch (const std::system_error&) {
        break;
      }
    }
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
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
  // Each call is its own Job and several threads may call at once (e.g. the pool's CheckTx
  // beside txv_submit_votes' staging): idle workers take chunks of any job that has some left,
  // and every caller drains its own job, so no call waits on another's.
  void parallel_for(uint32_t n, const std::function<void(uint32_t, uint32_t)>& fn, uint32_t min_chunk = 2048) {
    const uint32_t parts = std::min<uint32_t>(size() * 4, std::max<uint32_t>(1, n / min_chunk));
    if (parts <= 1 || th_.empty()) { if (n) fn(0, n); return; }
    auto job = std::make_shared<Job>();
    job->fn = &fn; job->n = n; job->parts = parts;
    {
      std::lock_guard<std::mutex> g(m_);
      jobs_.push_back(job);
    }
    cv_.notify_all();
    work(*job);
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [&] { return job->done.load() == job->parts; });
    for (size_t i = 0; i < jobs_.size(); ++i)
      if (jobs_[i] == job) { jobs_.erase(jobs_.begin() + (ptrdiff_t)i); break; }
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
  // a job with chunks left (under m_)
  std::shared_ptr<Job> pick() const {
    for (const auto& j : jobs_)
      if (j->next.load() < j->parts) return j;
    return nullptr;
  }
  void loop() {
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || (j = pick()) != nullptr; });
        if (stop_) return;
      }
      work(*j);
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::shared_ptr<Job>> jobs_;   // jobs whose callers have not returned yet
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
  // the open-addressing slots (validator index or UINT32_MAX), mirrored on the device
  const std::vector<uint32_t>& slots() const { return slots_; }
  uint64_t mask() const { return mask_; }
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
