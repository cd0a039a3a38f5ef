// Stress of txv_host::WorkerPool (host_pack.hpp): 1-3 caller threads posting parallel_for jobs
// back to back, checking every chunk ran exactly once; a hang shows as a timeout.
// hipcc -O2 -std=c++17 -x hip tools/debug/workerpool_stress.cpp -o /tmp/wps/stress && /tmp/wps/stress 16 2 200000
#include "../../go-txflow_amd/csrc/host_pack.hpp"

#include <cstdio>
#include <cstdlib>

int main(int argc, char** argv) {
  const unsigned nt = argc > 1 ? atoi(argv[1]) : 16, callers = argc > 2 ? atoi(argv[2]) : 2;
  const int iters = argc > 3 ? atoi(argv[3]) : 100000;
  txv_host::WorkerPool pool(nt);
  std::atomic<long> bad{0};
  std::vector<std::thread> th;
  std::atomic<long> prog[8] = {};
  std::atomic<bool> fin{false};
  std::thread watch([&] {   // progress once a second: a caller stuck in parallel_for stops counting
    while (!fin.load()) {
      std::this_thread::sleep_for(std::chrono::seconds(1));
      fprintf(stderr, "progress");
      for (unsigned c = 0; c < callers; ++c) fprintf(stderr, " %ld", prog[c].load());
      fprintf(stderr, "\n");
#ifdef TXV_STRESS_DUMP   // built with -Dprivate=public: the slots' words
      for (auto& sl : pool.slots_) {
        const uint64_t v = sl.state.load();
        fprintf(stderr, "  slot seq %llu next %u parts %u done %u owned %d n %u\n", (unsigned long long)(v >> 32),
                (unsigned)(v & 0xffff), (unsigned)(v >> 16) & 0xffff, sl.done.load(), (int)sl.owned.load(), sl.n);
      }
      fprintf(stderr, "  sleepers %u gen %llu\n", pool.sleepers_.load(), (unsigned long long)pool.gen_.load());
#endif
    }
  });
  for (unsigned c = 0; c < callers; ++c)
    th.emplace_back([&, c] {
      std::vector<std::atomic<int>> hit(64);
      for (int it = 0; it < iters; ++it) {
        const uint32_t n = 1 + (uint32_t)((it * 2654435761u + c) % 64);
        for (uint32_t i = 0; i < n; ++i) hit[i].store(0);
        pool.parallel_for(n, [&](uint32_t lo, uint32_t hi) {
          for (uint32_t i = lo; i < hi; ++i) hit[i].fetch_add(1);
        }, 1);
        for (uint32_t i = 0; i < n; ++i)
          if (hit[i].load() != 1) bad.fetch_add(1);
        prog[c].store(it);
      }
    });
  for (auto& t : th) t.join();
  fin.store(true);
  watch.join();
  printf("done, bad=%ld\n", bad.load());
  return bad.load() != 0;
}
