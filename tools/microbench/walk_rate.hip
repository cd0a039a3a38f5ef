// walk_rate.hip — where K1b's table walk spends the time beyond its ALU work (gfx950).
// Runs the shipped walk (double_scalarmult_pf<24, 20, 2> from kernels_verify.hip: cooperative
// LDS-DMA gathers, entries read from LDS, signed digits on the fly) over production-sized
// tables (an 11.8 GB radix-2^24 base table + 100 x 872 MB radix-2^20 validator tables, contents
// irrelevant for timing), 8 walks per lane at K1b's geometry (512-thread blocks, 2 waves/SIMD):
//   mode hbm    random 253-bit scalars: every entry a random line of ~99 GB (HBM, TLB misses)
//   mode l2     scalars whose every digit is < 64: all entries within a few hundred KB (L2 hits)
// Compare with tools/microbench/fe10_rate (the same additions with the entry in registers).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../go-txflow_amd/csrc -I../../include walk_rate.hip -o walk_rate
#include "../../go-txflow_amd/csrc/kernels_verify.hip"

#include <cstdio>
#include <random>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int kBlock = 512, kWalks = 8, kNScal = 1 << 16;

// group: validators restricted per XCD (blocks b, b+8, ... share an XCD): 0 = any of the 100,
// g > 0 = XCD x walks only validators [x g, x g + g) (a validator-grouped work list)
__global__ void __launch_bounds__(kBlock, 2) k_pfwalk(const uint32_t* tb, const uint32_t* ta, uint32_t n_val,
                                                      const uint32_t* scal, uint32_t* out, uint32_t group) {
  __shared__ uint4 pf[kBlock / 64][2 * 8 * 64];
  // the wave's buffer from a wave-uniform (scalar) index: the LDS-DMA destination goes to M0
  uint4* wbuf = pf[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
  const uint32_t gid = blockIdx.x * kBlock + threadIdx.x;
  uint32_t acc = 0;
#pragma unroll 1
  for (int r = 0; r < kWalks; ++r) {
    const uint32_t q = (gid * kWalks + r) & (kNScal - 1);
    uint32_t s[8], k[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[j] = scal[(size_t)j * kNScal + q]; k[j] = scal[(size_t)(8 + j) * kNScal + q]; }
    const uint32_t h = gid * 2654435761u + r * 40503u;
    const uint32_t va = group ? ((blockIdx.x % 8) * group + (h >> 8) % group) % n_val : (h >> 8) % n_val;
    const ge_ext R = k1b_walk<24, 20, 2>(tb, ta, va, s, k, wbuf);   // TXV_K1B_REGSTAGE picks the walk
    acc ^= R.X.v[0] ^ R.Y.v[1] ^ R.Z.v[2];
  }
  out[gid] = acc;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const uint32_t n_val = 100;
  uint32_t *tb, *ta, *scal, *out;
  const size_t tbw = Tab<24>::kWords, taw = Tab<20>::kWords;
  CHK(hipMalloc(&tb, tbw * 4));
  CHK(hipMalloc(&ta, taw * 4 * n_val));
  CHK(hipMemset(tb, 0x11, 1 << 20));
  CHK(hipMalloc(&scal, (size_t)16 * kNScal * 4));
  CHK(hipMalloc(&out, (size_t)cus * kBlock * 4));
  std::mt19937_64 rng(7);
  std::vector<uint32_t> h((size_t)16 * kNScal);
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  printf("{\"walks\": %d, \"results\": [\n", cus * kBlock * kWalks);
  const int modes[4] = {0, 1, 0, 0};
  const uint32_t groups[4] = {0, 0, 12, 1};
  const char* names[4] = {"hbm", "l2", "hbm_xcd_grouped12", "hbm_xcd_grouped1"};
  for (int mi = 0; mi < 4; ++mi) {
    const int mode = modes[mi];
    for (int q = 0; q < kNScal; ++q) {
      uint32_t s[8] = {0}, k[8] = {0};
      if (mode == 0) {
        for (int j = 0; j < 8; ++j) { s[j] = (uint32_t)rng(); k[j] = (uint32_t)rng(); }
        s[7] &= 0x1fffffffu; k[7] &= 0x1fffffffu;
      } else {   // every window's digit in [0, 64): W = 24 for s, 20 for k
        for (int p = 0; p < 11; ++p) { const uint32_t v = rng() & 63; const int bit = 24 * p; s[bit / 32] |= v << (bit % 32); if (bit % 32 > 26 && bit / 32 < 7) s[bit / 32 + 1] |= v >> (32 - bit % 32); }
        for (int p = 0; p < 13; ++p) { const uint32_t v = rng() & 63; const int bit = 20 * p; k[bit / 32] |= v << (bit % 32); if (bit % 32 > 26 && bit / 32 < 7) k[bit / 32 + 1] |= v >> (32 - bit % 32); }
      }
      for (int j = 0; j < 8; ++j) { h[(size_t)j * kNScal + q] = s[j]; h[(size_t)(8 + j) * kNScal + q] = k[j]; }
    }
    CHK(hipMemcpy(scal, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      CHK(hipEventRecord(a));
      hipLaunchKernelGGL(k_pfwalk, dim3(cus), dim3(kBlock), 0, 0, tb, ta, n_val, scal, out, groups[mi]);
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      if (rep && ms < best) best = ms;
    }
    const double walks = (double)cus * kBlock * kWalks;
    printf("%s {\"mode\": \"%s\", \"ms\": %.4f, \"walks_per_s\": %.4e, \"additions_per_s\": %.4e}\n", mi ? "," : " ",
           names[mi], best, walks / (best * 1e-3), 23 * walks / (best * 1e-3));
    if (mi == 0) {   // the same launch 40 times back to back (sustained load: clocks under power limits)
      CHK(hipEventRecord(a));
      for (int rep = 0; rep < 40; ++rep)
        hipLaunchKernelGGL(k_pfwalk, dim3(cus), dim3(kBlock), 0, 0, tb, ta, n_val, scal, out, groups[mi]);
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      printf(", {\"mode\": \"hbm_sustained40\", \"ms\": %.4f}\n", ms / 40);
    }
  }
  printf("]}\n");
  return 0;
}
