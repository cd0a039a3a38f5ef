// fe10_rate.hip — pure-ALU ceiling of K1b's table walk on gfx950: the mixed addition
// (ge10_madd_rd, 7 fe10 multiplies) with its entry already in registers, no memory traffic,
// at 1..8 waves per SIMD.  Compare with K1b's achieved additions/s (23 per vote) to split
// its time into ALU issue vs everything else (gathers, LDS reads, digits, tail).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../go-txflow_amd/csrc fe10_rate.hip -o fe10_rate
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "ge.h"

using namespace txv;

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ADDS = 2048;

template <int MODE>
__global__ void __launch_bounds__(256) k_walk(uint32_t* out, uint32_t seed) {
  fe10 qp, qm, qd;
  ge10_ext P;
  for (int i = 0; i < 10; ++i) {
    const uint32_t m = TXV_M10(i);
    qp.v[i] = (seed * 2654435761u + threadIdx.x * 97u + i) & m;
    qm.v[i] = (seed * 40503u + threadIdx.x * 31u + 7u * i) & m;
    qd.v[i] = (seed ^ (threadIdx.x * 131u + 3u * i)) & m;
    P.X.v[i] = (seed + i * 5u + threadIdx.x) & m;
    P.Y.v[i] = (seed * 3u + i) & m;
    P.Z.v[i] = (i == 0);
    P.T.v[i] = (seed * 7u + i * 11u) & m;
  }
#pragma unroll 1
  for (int t = 0; t < ADDS; ++t) {
    if (MODE == 0) {
      P = ge10_madd_rd(P, [&](int role) { return role == 0 ? qp : role == 1 ? qm : qd; }, (t & 1) != 0, [] {});
    } else {
      // the multiplies alone: 7 dependent-free products per step, same operand shapes
      P.X = fe10_mul(P.X, qp);
      P.Y = fe10_mul(P.Y, qm);
      P.Z = fe10_mul(P.Z, qd);
      P.T = fe10_mul(P.T, qp);
      P.X = fe10_mul(P.X, P.Y);
      P.Y = fe10_mul(P.Y, P.Z);
      P.Z = fe10_mul(P.Z, P.T);
    }
    qp.v[t & 7] ^= 1u;   // keep the entry live per iteration
  }
  uint32_t r = 0;
  for (int i = 0; i < 10; ++i) r ^= P.X.v[i] ^ P.Y.v[i] ^ P.Z.v[i] ^ P.T.v[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint32_t* d;
  CHK(hipMalloc(&d, (size_t)cus * 8 * 256 * 4));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  printf("{\"cus\": %d, \"adds_per_lane\": %d, \"results\": [\n", cus, ADDS);
  bool first = true;
  for (int mode = 0; mode < 2; ++mode) {
    for (int wps : {1, 2, 3, 4, 6, 8}) {
      const int blocks = cus * wps;   // 256-thread blocks = one wave per SIMD each
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        CHK(hipEventRecord(a));
        if (mode == 0) hipLaunchKernelGGL(k_walk<0>, dim3(blocks), dim3(256), 0, 0, d, 7u + rep);
        else hipLaunchKernelGGL(k_walk<1>, dim3(blocks), dim3(256), 0, 0, d, 7u + rep);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (rep && ms < best) best = ms;
      }
      const double adds = (double)blocks * 256 * ADDS;
      printf("%s {\"mode\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"additions_per_s\": %.4e, "
             "\"mults_per_s\": %.4e}\n", first ? " " : ",", mode == 0 ? "madd" : "7mul", wps, best,
             adds / (best * 1e-3), 7 * adds / (best * 1e-3));
      first = false;
    }
  }
  printf("]}\n");
  return 0;
}
