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
#include <chrono>
#include <cstdlib>
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
// Persistent threads; a parallel_for posts its chunks in one of kSlots job slots and the caller
// takes part.  Claiming a chunk is one CAS on the slot's (sequence, next chunk) word -- no mutex on
// the hot path: with a mutex the 15 woken workers of every pass queued on it one futex hand-off
// after another (tens of microseconds per pass, ~8 passes per CheckTx batch).  A worker that runs
// out of chunks spins for TXV_HOST_SPIN_US (default 200 us: the passes of one CheckTx batch or one
// staging follow each other within microseconds), then sleeps on a condition variable.
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
    stop_.store(true);
    {
      std::lock_guard<std::mutex> g(m_);
      gen_.fetch_add(1);
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
  // Several threads may call at once (e.g. the pool's CheckTx beside txv_submit_votes' staging):
  // each call has its own slot, idle workers take chunks of any slot, and every caller drains its
  // own job, so no call waits on another's.  With every slot taken the call runs inline.
  void parallel_for(uint32_t n, const std::function<void(uint32_t, uint32_t)>& fn, uint32_t min_chunk = 2048) {
    const uint32_t parts = std::min<uint32_t>(std::min<uint32_t>(size() * 4, 0xffff), std::max<uint32_t>(1, n / min_chunk));
    if (parts <= 1 || th_.empty()) { if (n) fn(0, n); return; }
    Slot* s = nullptr;
    for (auto& c : slots_) {
      bool f = false;
      if (c.owned.compare_exchange_strong(f, true)) { s = &c; break; }
    }
    if (!s) { fn(0, n); return; }
    s->fn = &fn; s->n = n;
    s->done.store(0, std::memory_order_relaxed);
    const uint64_t seq = (s->state.load(std::memory_order_relaxed) >> 32) + 1;
    s->state.store(seq << 32 | (uint64_t)parts << 16, std::memory_order_release);   // published: chunk 0 is next
    gen_.fetch_add(1);
    if (sleepers_.load()) {
      std::lock_guard<std::mutex> g(m_);
      cv_.notify_all();
    }
    while (claim_run(*s)) {}
    // the other threads' chunks are usually a few microseconds behind: spin before sleeping
    for (auto t0 = std::chrono::steady_clock::now(); s->done.load(std::memory_order_acquire) != parts;) {
      cpu_relax();
      if (std::chrono::steady_clock::now() - t0 > spin_) {
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [&] { return s->done.load() == parts; });
        break;
      }
    }
    s->owned.store(false, std::memory_order_release);
  }

 private:
  static constexpr int kSlots = 8;
  struct Slot {
    // (sequence << 32) | (parts << 16) | next chunk: the CAS that claims a chunk checks all three
    // (a separate parts word could be the next job's while this word still names the last one)
    std::atomic<uint64_t> state{0};
    std::atomic<uint32_t> done{0};
    std::atomic<bool> owned{false};            // a caller is using the slot
    const std::function<void(uint32_t, uint32_t)>* fn = nullptr;
    uint32_t n = 0;
  };
  // claim the slot's next chunk and run it; false when none is left.  A claimed chunk keeps the
  // job alive (its caller waits for done == parts), so fn / n / parts are read after the CAS.
  bool claim_run(Slot& s) {
    uint64_t v = s.state.load(std::memory_order_acquire);
    for (;;) {
      const uint32_t nx = (uint32_t)(v & 0xffff), parts = (uint32_t)(v >> 16) & 0xffff;
      if (nx >= parts || (v >> 32) == 0) return false;
      if (s.state.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel, std::memory_order_acquire)) {
        const uint32_t n = s.n;
        const uint32_t lo = (uint32_t)((uint64_t)n * nx / parts), hi = (uint32_t)((uint64_t)n * (nx + 1) / parts);
        (*s.fn)(lo, hi);
        if (s.done.fetch_add(1, std::memory_order_acq_rel) + 1 == parts) {
          std::lock_guard<std::mutex> g(m_);
          done_cv_.notify_all();
        }
        return true;
      }
    }
  }
  bool run_any() {
    bool any = false;
    for (auto& s : slots_)
      while (claim_run(s)) any = true;
    return any;
  }
  static void cpu_relax() {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
  void loop() {
    for (;;) {
      const uint64_t g0 = gen_.load();
      if (run_any()) continue;
      for (auto t0 = std::chrono::steady_clock::now(); gen_.load(std::memory_order_acquire) == g0;) {
        cpu_relax();
        if (std::chrono::steady_clock::now() - t0 > spin_) {
          std::unique_lock<std::mutex> lk(m_);
          sleepers_.fetch_add(1);
          cv_.wait(lk, [&] { return stop_.load() || gen_.load() != g0; });
          sleepers_.fetch_sub(1);
          break;
        }
      }
      if (stop_.load()) return;
    }
  }
  std::vector<std::thread> th_;
  Slot slots_[kSlots];
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::atomic<bool> stop_{false};
  std::atomic<unsigned> sleepers_{0};        // workers waiting on cv_
  std::atomic<uint64_t> gen_{0};             // jobs posted so far
  std::chrono::microseconds spin_{spin_us()};
  static unsigned spin_us() {                // TXV_HOST_SPIN_US (default 200, 0 = sleep at once)
    const char* e = getenv("TXV_HOST_SPIN_US");
    return e ? (unsigned)std::max(0, atoi(e)) : 200u;
  }
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
