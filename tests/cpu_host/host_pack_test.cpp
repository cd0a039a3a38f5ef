// CPU test of go-txflow_amd/csrc/host_pack.hpp (the host pack's worker pool and lookup tables);
// built by tests/test_host_pack.py with -fsanitize=thread (pool) / address,undefined (tables).
#include "../../go-txflow_amd/csrc/host_pack.hpp"
#include <cstdio>
#include <map>
#include <random>
#include <string>

using namespace txv_host;

static int fail(const char* what, long a, long b) { printf("FAIL %s: %ld vs %ld\n", what, a, b); return 1; }

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 300;
  // pool: back-to-back jobs of varying size; every index visited exactly once per job
  {
    WorkerPool pool(16);
    std::vector<uint32_t> hits(100000);
    for (int it = 0; it < iters; ++it) {
      const uint32_t n = 1 + (uint32_t)((it * 7919u) % 99999u);
      std::fill(hits.begin(), hits.begin() + n, 0u);
      pool.parallel_for(n, [&](uint32_t lo, uint32_t hi) { for (uint32_t i = lo; i < hi; ++i) hits[i]++; }, 512);
      for (uint32_t i = 0; i < n; ++i) if (hits[i] != 1) return fail("pool hit count", i, hits[i]);
    }
  }
  // hash_bytes (txv_hash.h, shared with the device set table): chunk-wise definition, tail bytes
  // beyond the key never matter, never 0
  {
    std::mt19937_64 rng(7);
    for (int it = 0; it < 20000; ++it) {
      const uint32_t len = (uint32_t)(rng() % 80);
      std::vector<uint8_t> a(len + 16), b(len + 16);
      for (auto& x : a) x = (uint8_t)rng();
      b = a;
      for (uint32_t j = len; j < len + 16; ++j) b[j] = (uint8_t)rng();   // different bytes after the key
      const uint64_t seed = rng();
      const uint64_t ha = hash_bytes(a.data(), len, seed), hb = hash_bytes(b.data(), len, seed);
      if (ha != hb || !ha) return fail("hash tail", (long)len, 0);
      uint64_t h = seed ^ (0x9e3779b97f4a7c15ULL * (uint64_t)(len + 1));
      uint32_t i = 0;
      for (; i + 8 <= len; i += 8) { uint64_t w; memcpy(&w, a.data() + i, 8); h = txv_hash::mix64(h ^ w) + 0x9e3779b97f4a7c15ULL; }
      if (i < len) { uint64_t t = 0; memcpy(&t, a.data() + i, len - i); h = txv_hash::mix64(h ^ t ^ ((uint64_t)(len - i) << 56)); }
      if ((txv_hash::mix64(h) | 1ull) != ha) return fail("hash def", (long)len, 1);
    }
  }
  // AddrTable: exact 20-byte match, first index wins on a repeated address, misses
  {
    std::mt19937_64 rng(9);
    std::vector<uint8_t> addrs(20 * 1000);
    for (auto& b : addrs) b = (uint8_t)rng();
    memcpy(addrs.data() + 20 * 999, addrs.data() + 20 * 5, 20);
    AddrTable a;
    a.build(addrs.data(), 1000);
    for (uint32_t v = 0; v < 999; ++v) if (a.find(addrs.data() + 20 * v) != v) return fail("addr find", v, a.find(addrs.data() + 20 * v));
    if (a.find(addrs.data() + 20 * 999) != 5) return fail("addr dup", a.find(addrs.data() + 20 * 999), 5);
    uint8_t miss[20];
    memcpy(miss, addrs.data(), 20);
    miss[19] ^= 1;
    if (a.find(miss) != UINT32_MAX) return fail("addr miss", 0, 1);
  }
  // counting_sort: stable by key, dropped keys skipped, key starts
  {
    WorkerPool pool(8);
    std::mt19937_64 rng(11);
    for (int it = 0; it < 4; ++it) {
      const uint32_t n = (uint32_t)(rng() % 120000), K = 1 + (uint32_t)(rng() % 700);
      std::vector<uint32_t> key(n);
      for (auto& k : key) k = (rng() % 7 == 0) ? UINT32_MAX : (uint32_t)(rng() % K);
      std::vector<uint32_t> out(n, 0xdead), starts(K + 1);
      const uint32_t m = counting_sort(pool, n, K, [&](uint32_t i) { return key[i]; },
                                       [&](uint32_t p, uint32_t i) { out[p] = i; }, starts.data());
      std::vector<std::vector<uint32_t>> byk(K);
      for (uint32_t i = 0; i < n; ++i) if (key[i] != UINT32_MAX) byk[key[i]].push_back(i);
      uint32_t p = 0;
      for (uint32_t k = 0; k < K; ++k) {
        if (starts[k] != p) return fail("sort starts", starts[k], p);
        for (uint32_t i : byk[k]) if (out[p++] != i) return fail("sort order", out[p - 1], i);
      }
      if (m != p || starts[K] != p) return fail("sort count", m, p);
    }
  }
  printf("ok\n");
  return 0;
}
