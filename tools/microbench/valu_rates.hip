// Integer-VALU issue-rate microbenchmark for gfx950 (MI355X).
// Measures wave-instruction throughput of the integer ops a 255-bit field
// multiply is built from, relative to a full-rate v_add_u32, so the roofline
// peak P used by bench.py is measured on the box rather than assumed.
// Build: hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

// 8 independent chains per lane; each asm statement is one instruction.
#define BODY8(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

__global__ void k_add(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3u + 1u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_addco(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3u + 1u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[i]) : "v"(b) : "vcc");
    BODY8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_addc(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3u + 1u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a[i]) : "v"(b) : "vcc");
    BODY8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mullo(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3u + 1u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mulhi(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3u + 1u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul24(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3u + 1u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mad64(uint32_t* out, uint32_t seed) {
  uint64_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3u + 1u, c = seed ^ 0x1234567u;
#define S(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c) : "vcc");
  for (int it = 0; it < ITERS; ++it) { BODY8(S) }
#undef S
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= (uint32_t)a[i] ^ (uint32_t)(a[i] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_fma64(uint32_t* out, uint32_t seed) {
  double a[8];
  for (int i = 0; i < 8; ++i) a[i] = (double)(seed + threadIdx.x + i);
  double b = 0.999, c = 1e-3;
#define S(i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
  for (int it = 0; it < ITERS; ++it) { BODY8(S) }
#undef S
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= (uint32_t)a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_fma32(uint32_t* out, uint32_t seed) {
  float a[8];
  for (int i = 0; i < 8; ++i) a[i] = (float)(seed + threadIdx.x + i);
  float b = 0.999f, c = 1e-3f;
#define S(i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
  for (int it = 0; it < ITERS; ++it) { BODY8(S) }
#undef S
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= (uint32_t)a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_lshr64(uint32_t* out, uint32_t seed) {
  uint64_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t sh = 3;
#define S(i) asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(a[i]) : "v"(sh));
  for (int it = 0; it < ITERS; ++it) { BODY8(S) }
#undef S
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= (uint32_t)a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_alignbit(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3u + 1u;
#define S(i) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(b));
  for (int it = 0; it < ITERS; ++it) { BODY8(S) }
#undef S
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}


// generic 8-chain kernel: STMT(i) is one instruction per chain
#define KERN(NAME, DECL, STMT)                                                        \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                                \
    uint32_t a[8]; uint64_t q[8];                                                      \
    for (int i = 0; i < 8; ++i) { a[i] = seed + threadIdx.x + i; q[i] = a[i] * 0x9e37ull; } \
    uint32_t b = seed * 3u + 1u, c = seed ^ 0x9e3779b9u;                               \
    uint64_t b64 = (uint64_t)b * 77u;                                                  \
    DECL                                                                               \
    for (int it = 0; it < ITERS; ++it) { BODY8(STMT) }                                \
    uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i] ^ (uint32_t)q[i] ^ (uint32_t)(q[i] >> 32); \
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                    \
  }

#define S_MADS(i) asm volatile("v_mad_u64_u32 %0, s[%2:%3], %1, %1, %0" : "+v"(q[i]) : "v"(b), "n"(2 * i + 20), "n"(2 * i + 21) : "s20","s21","s22","s23","s24","s25","s26","s27","s28","s29","s30","s31","s32","s33","s34","s35");
KERN(k_mad64_sgprs, , S_MADS)
#define S_ADDCOS(i) asm volatile("v_add_co_u32 %0, s[%2:%3], %0, %1" : "+v"(a[i]) : "v"(b), "n"(2 * i + 20), "n"(2 * i + 21) : "s20","s21","s22","s23","s24","s25","s26","s27","s28","s29","s30","s31","s32","s33","s34","s35");
KERN(k_addco_sgprs, , S_ADDCOS)
#define S_LSHLADD(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[i]) : "v"(b64));
KERN(k_lshladd64, , S_LSHLADD)
#define S_ADD3(i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
KERN(k_add3, , S_ADD3)
#define S_MAD24(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
KERN(k_mad24, , S_MAD24)
#define S_MULHI24(i) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
KERN(k_mulhi24, , S_MULHI24)
#define S_DOT2(i) asm volatile("v_dot2_u32_u16 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c));
KERN(k_dot2u16, , S_DOT2)
#define S_DOT4(i) asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c));
KERN(k_dot4u8, , S_DOT4)
#define S_XOR(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
KERN(k_xor, , S_XOR)
#define S_MOV(i) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(a[(i + 1) & 7]));
KERN(k_mov, , S_MOV)
#define S_CND(i) asm volatile("v_cndmask_b32 %0, %0, %1, s[20:21]" : "+v"(a[i]) : "v"(b) : "s20", "s21");
KERN(k_cndmask, , S_CND)
#define S_MADLO(i) asm volatile("v_mad_u64_u32 %0, s[20:21], %1, %1, %0" : "+v"(q[i]) : "v"(b) : "s20", "s21");
KERN(k_mad64_same_sgpr, , S_MADLO)
#define S_MOV64(i) asm volatile("v_mov_b64 %0, %1" : "=v"(q[i]) : "v"(q[(i + 1) & 7]));
KERN(k_mov64, , S_MOV64)
#define S_ADDU64(i) asm volatile("v_lshl_add_u64 %0, %1, 1, %0" : "+v"(q[i]) : "v"(b64));
KERN(k_lshladd64_sh1, , S_ADDU64)
// field-mul shaped pair: mad (carry to cc_i) then addc of that carry into an overflow word
#define S_PAIR(i) asm volatile("v_mad_u64_u32 %0, s[%3:%4], %2, %2, %0\n\tv_addc_co_u32 %1, s[%3:%4], %1, 0, s[%3:%4]" : "+v"(q[i]), "+v"(a[i]) : "v"(b), "n"(2 * (i & 3) + 20), "n"(2 * (i & 3) + 21) : "s20","s21","s22","s23","s24","s25","s26","s27");
KERN(k_madaddc_pair, , S_PAIR)

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  const int block = 256, blocks = cus * 8;  // 8 waves/SIMD worth of work
  uint32_t* out; CHK(hipMalloc(&out, (size_t)blocks * block * 4));
  struct { const char* name; kfn f; } ks[] = {
    {"v_add_u32", k_add}, {"v_add_co_u32", k_addco}, {"v_addc_co_u32", k_addc},
    {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi}, {"v_mul_u32_u24", k_mul24},
    {"v_mad_u64_u32", k_mad64}, {"v_fma_f32", k_fma32}, {"v_fma_f64", k_fma64},
    {"v_lshrrev_b64", k_lshr64}, {"v_alignbit_b32", k_alignbit},
    {"v_mad_u64_u32 (8 carry SGPR pairs)", k_mad64_sgprs}, {"v_mad_u64_u32 (one carry SGPR pair)", k_mad64_same_sgpr},
    {"v_add_co_u32 (8 carry SGPR pairs)", k_addco_sgprs}, {"v_lshl_add_u64 (shift 0)", k_lshladd64},
    {"v_lshl_add_u64 (shift 1)", k_lshladd64_sh1}, {"v_add3_u32", k_add3}, {"v_mad_u32_u24", k_mad24},
    {"v_mul_hi_u32_u24", k_mulhi24}, {"v_dot2_u32_u16", k_dot2u16}, {"v_dot4_u32_u8", k_dot4u8},
    {"v_xor_b32", k_xor}, {"v_mov_b32", k_mov}, {"v_mov_b64", k_mov64}, {"v_cndmask_b32", k_cndmask},
    {"mad+addc pair (counts 2 insts)", k_madaddc_pair},
  };
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  double base = 0;
  printf("{\"cus\": %d, \"clock_khz\": %d, \"results\": [\n", cus, prop.clockRate);
  for (size_t i = 0; i < sizeof(ks) / sizeof(ks[0]); ++i) {
    hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(block), 0, 0, out, 7u);  // warm
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(block), 0, 0, out, 7u + r);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
    }
    double wave_insts = (double)blocks * (block / 64) * ITERS * 8.0;
    double lane_ops_per_s = wave_insts * 64.0 / (best * 1e-3);
    if (i == 0) base = lane_ops_per_s;
    printf("  {\"inst\": \"%s\", \"ms\": %.4f, \"lane_ops_per_s\": %.4e, \"rate_vs_v_add_u32\": %.4f}%s\n",
           ks[i].name, best, lane_ops_per_s, lane_ops_per_s / base,
           i + 1 < sizeof(ks) / sizeof(ks[0]) ? "," : "");
  }
  printf("]}\n");
  CHK(hipFree(out));
  return 0;
}
