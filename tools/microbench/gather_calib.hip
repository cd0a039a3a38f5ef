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
//        of a verify-sized table) [MLANES]
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

// cooperative: 8 lanes load one 128-byte entry (16 B each, one coalesced line per 8 lanes)
__global__ void gather_coop(const uint4* __restrict__ table, const uint32_t* __restrict__ idx, uint32_t n,
                            uint32_t stride_q, uint32_t* out) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if ((t >> 3) >= n) return;
  const uint4 v = table[(size_t)idx[t >> 3] * stride_q + (t & 7)];
  out[t >> 3] = v.x ^ v.y ^ v.z ^ v.w;
}

// the fe10 half-Niels entry's loads (ed25519_dev.h load_entry_w): (x4, x4, x2) at words 0 and 12
// (swapped by a per-lane sign), x2 + x4 + x4 at word 22
__global__ void gather_fe10(const uint32_t* __restrict__ table, const uint32_t* __restrict__ idx, uint32_t n,
                            uint32_t stride_w, uint32_t* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t* e = table + (size_t)idx[i] * stride_w;
  const bool neg = idx[i] & 1;
  const uint4* p4 = reinterpret_cast<const uint4*>(e + (neg ? 12 : 0));
  const uint4* m4 = reinterpret_cast<const uint4*>(e + (neg ? 0 : 12));
  const uint2* d2 = reinterpret_cast<const uint2*>(e + 22);
  const uint4 a = p4[0], b = p4[1], c = m4[0], d = m4[1], f = reinterpret_cast<const uint4*>(d2 + 1)[0],
              g = reinterpret_cast<const uint4*>(d2 + 1)[1];
  const uint2 h = reinterpret_cast<const uint2*>(p4 + 2)[0], k = reinterpret_cast<const uint2*>(m4 + 2)[0], l = d2[0];
  out[i] = a.x ^ b.y ^ c.z ^ d.w ^ f.x ^ g.y ^ h.x ^ k.y ^ l.x ^ a.w ^ b.x ^ c.y ^ d.z ^ f.w ^ g.x;
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
  // read 96: 6 x 16-byte loads; 128: 8 x 16-byte loads; 120: the fe10 entry's 9 loads
  // read 8: the cooperative 128-byte gather (8 lanes per entry)
  if (stride % 16 || read > stride || (read != 16 && read != 96 && read != 128 && read != 120 && read != 8)) { fprintf(stderr, "bad shape\n"); return 2; }
  const size_t bytes = (size_t)(argc > 3 ? atoi(argv[3]) : 4) << 30, entries = bytes / stride;
  const uint32_t n = argc > 4 ? (uint32_t)atoi(argv[4]) << 20 : 1u << 20;
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
    else if (read == 128)
      hipLaunchKernelGGL(gather<8>, dim3((n + 255) / 256), dim3(256), 0, 0, table, didx, n, stride / 16, out);
    else if (read == 8)
      hipLaunchKernelGGL(gather_coop, dim3((8 * n + 255) / 256), dim3(256), 0, 0, table, didx, n, stride / 16, out);
    else if (read == 120)
      hipLaunchKernelGGL(gather_fe10, dim3((n + 255) / 256), dim3(256), 0, 0, (const uint32_t*)table, didx, n, stride / 4, out);
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
