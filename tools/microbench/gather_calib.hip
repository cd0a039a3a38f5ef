// FETCH_SIZE calibration for the verify kernels' access pattern (MI355X_MICROARCH.md: "other
// access widths are uncalibrated: calibrate on a known byte count"): every lane gathers one
// table entry of READ bytes (READ/16 x 16-byte loads, as load_entry_w does) at a random entry
// index of a 4 GiB table of STRIDE-byte entries (far beyond the 256 MiB Infinity Cache), so
// every access misses on-die.  The program prints the exact number of distinct 32-byte sectors,
// 64-byte sectors and 128-byte lines the gathers touch plus the 4 MiB index read, and the
// kernel's average time; rocprofv3 --pmc FETCH_SIZE on the same run gives the counter to
// compare.  Three shapes separate the hypotheses "FETCH_SIZE = bytes at 32 B granularity" and
// "FETCH_SIZE = half of the 128 B lines fetched":
//   96 96   (the verify tables today), 128 96 (entries padded to one line), 16 16 (one load).
// Build: hipcc --offload-arch=gfx950 -O3 gather_calib.hip -o gather_calib
// Run:   gather_calib STRIDE READ [TABLE_GIB]   (TABLE_GIB default 4; 64 probes the page-walk cost
//        of a verify-sized table)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int Q>
__global__ void gather(const uint4* __restrict__ table, const uint32_t* __restrict__ idx, uint32_t n, uint32_t stride_q,
                       uint32_t* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint4* e = table + (size_t)idx[i] * stride_q;
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < Q; ++j) { const uint4 v = e[j]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  out[i] = acc;
}

static uint64_t distinct(const std::vector<uint32_t>& idx, uint64_t stride, uint64_t read, uint64_t g) {
  std::vector<uint64_t> s;
  s.reserve(idx.size() * (read / g + 2));
  for (uint32_t v : idx) {
    const uint64_t b = (uint64_t)v * stride;
    for (uint64_t a = b / g; a <= (b + read - 1) / g; ++a) s.push_back(a);
  }
  std::sort(s.begin(), s.end());
  return (uint64_t)(std::unique(s.begin(), s.end()) - s.begin()) * g;
}

int main(int argc, char** argv) {
  const uint32_t stride = argc > 1 ? (uint32_t)atoi(argv[1]) : 96, read = argc > 2 ? (uint32_t)atoi(argv[2]) : 96;
  if (stride % 16 || read % 16 || read > stride || (read != 16 && read != 96)) { fprintf(stderr, "bad shape\n"); return 2; }
  const size_t bytes = (size_t)(argc > 3 ? atoi(argv[3]) : 4) << 30, entries = bytes / stride;
  const uint32_t n = 1u << 20;
  uint4* table; uint32_t *didx, *out;
  CHK(hipMalloc(&table, bytes));
  CHK(hipMemset(table, 1, bytes));
  std::vector<uint32_t> idx(n);
  uint64_t x = 0x9e3779b97f4a7c15ull;
  for (auto& v : idx) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint32_t)(x % entries); }
  CHK(hipMalloc(&didx, n * 4)); CHK(hipMalloc(&out, n * 4));
  CHK(hipMemcpy(didx, idx.data(), n * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  float total = 0.f;
  const int reps = 3;
  for (int r = 0; r < reps; ++r) {
    // flush the Infinity Cache between runs with a 1 GiB write
    CHK(hipMemset(reinterpret_cast<char*>(table) + bytes / 2, 1, 1ull << 30));
    CHK(hipEventRecord(e0, 0));
    if (read == 96)
      hipLaunchKernelGGL(gather<6>, dim3((n + 255) / 256), dim3(256), 0, 0, table, didx, n, stride / 16, out);
    else
      hipLaunchKernelGGL(gather<1>, dim3((n + 255) / 256), dim3(256), 0, 0, table, didx, n, stride / 16, out);
    CHK(hipEventRecord(e1, 0));
    CHK(hipDeviceSynchronize());
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); total += ms;
  }
  printf("{\"lanes\": %u, \"stride\": %u, \"read\": %u, \"table_gib\": %zu, \"algorithmic_bytes\": %llu, \"index_bytes\": %u, "
         "\"distinct_32B_bytes\": %llu, \"distinct_64B_bytes\": %llu, \"distinct_128B_bytes\": %llu, \"kernel_ms\": %.4f}\n",
         n, stride, read, bytes >> 30, (unsigned long long)n * read, n * 4, (unsigned long long)distinct(idx, stride, read, 32),
         (unsigned long long)distinct(idx, stride, read, 64), (unsigned long long)distinct(idx, stride, read, 128),
         total / reps);
  return 0;
}
