// fe.h — GF(2^255 - 19) arithmetic for CDNA4 (gfx950), 8 x 32-bit limbs, radix 2^32.
//
// Design (MI355X-first):
//   * One lane = one field element in 8 VGPRs.  Values are kept "weakly reduced":
//     any value in [0, 2^256) represents itself mod p; only encodings are canonical.
//   * Multiply = 8x8 product scanning.  Each partial product is ONE v_mad_u64_u32
//     (32x32 -> 64 multiply with a 64-bit addend) whose carry-out (VOP3b SGPR-pair sdst)
//     is folded into a third accumulator word by one v_addc_co_u32: 2 VALU ops per
//     partial product, 64 half-rate mads per multiply.  2^256 = 38 (mod p) folds the top.
//   * Carries between separate asm statements travel in explicit SGPR-pair operands
//     (the compiler tracks them as values), never through an implicit VCC.
//
// The __host__ branch of each primitive exists only so tests/cpu_emu can run the very
// same kernel source on the host to localise logic bugs; the product library never calls
// device math on the host (libtxvote has no CPU verify path).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#define TXV_HD __host__ __device__ __forceinline__

// Scheduling fence: keeps the compiler from interleaving independent field multiplies,
// which buys ILP at the cost of registers; with >= 4 waves per SIMD latency is hidden by
// the other waves instead (DESIGN.md §K1 register budget).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(TXV_SCHED_FENCE_OFF)   // _OFF: experiment builds
#define TXV_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define TXV_SCHED_FENCE() ((void)0)
#endif

namespace txv {

// ---------------------------------------------------------------- carry primitives
// c is an SGPR lane mask on the device; 0/1 on the host emulation.
TXV_HD void add_cc(uint32_t& r, uint64_t& c, uint32_t x, uint32_t y) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("v_add_co_u32 %0, %1, %2, %3" : "=v"(r), "=s"(c) : "v"(x), "v"(y));
#else
  r = x + y; c = r < x;
#endif
}
TXV_HD void addc_cc(uint32_t& r, uint64_t& c, uint32_t x, uint32_t y, uint64_t ci) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("v_addc_co_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(c) : "v"(x), "v"(y), "s"(ci));
#else
  uint64_t t = (uint64_t)x + y + (ci ? 1u : 0u); r = (uint32_t)t; c = t >> 32;
#endif
}
// r = x + y + ci, carry-out discarded
TXV_HD uint32_t addc_last(uint32_t x, uint32_t y, uint64_t ci) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r; uint64_t c;
  asm("v_addc_co_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(c) : "v"(x), "v"(y), "s"(ci));
  return r;
#else
  return x + y + (ci ? 1u : 0u);
#endif
}
TXV_HD void sub_cc(uint32_t& r, uint64_t& c, uint32_t x, uint32_t y) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("v_sub_co_u32 %0, %1, %2, %3" : "=v"(r), "=s"(c) : "v"(x), "v"(y));
#else
  r = x - y; c = x < y;
#endif
}
TXV_HD void subb_cc(uint32_t& r, uint64_t& c, uint32_t x, uint32_t y, uint64_t ci) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("v_subb_co_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(c) : "v"(x), "v"(y), "s"(ci));
#else
  uint64_t t = (uint64_t)x - y - (ci ? 1u : 0u); r = (uint32_t)t; c = (t >> 63) & 1u;
#endif
}
// {acc, ovf} += a * b   (96-bit column accumulator)
TXV_HD void mac(uint64_t& acc, uint32_t& ovf, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_addc_co_u32 %1, %2, %1, 0, %2"
      : "+v"(acc), "+v"(ovf), "=&s"(cc) : "v"(a), "v"(b));
#else
  unsigned __int128 t = (unsigned __int128)a * b + acc;
  acc = (uint64_t)t; ovf += (uint32_t)(t >> 64);
#endif
}
// per-lane select on a carry mask: c[lane] ? a : b
TXV_HD uint32_t sel_c(uint64_t c, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(c));
  return r;
#else
  return c ? a : b;
#endif
}
TXV_HD uint64_t mul64(uint32_t a, uint32_t b) { return (uint64_t)a * b; }
TXV_HD uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

// ---------------------------------------------------------------- field elements
struct fe { uint32_t v[8]; };

TXV_HD fe fe_zero() { fe r; for (int i = 0; i < 8; ++i) r.v[i] = 0; return r; }
TXV_HD fe fe_one() { fe r = fe_zero(); r.v[0] = 1; return r; }

#if defined(__HIP_DEVICE_COMPILE__)
#include "fe_asm.h"
#endif

// reduce a 512-bit product t[16] to [0, 2^256) using 2^256 = 38 (mod p)
TXV_HD fe fe_reduce512(const uint32_t t[16]) {
  uint64_t p[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) p[i] = mad64(t[8 + i], 38u, (uint64_t)t[i]);
  fe r; uint64_t c;
  r.v[0] = (uint32_t)p[0];
  add_cc(r.v[1], c, (uint32_t)p[1], (uint32_t)(p[0] >> 32));
#pragma unroll
  for (int i = 2; i < 8; ++i) addc_cc(r.v[i], c, (uint32_t)p[i], (uint32_t)(p[i - 1] >> 32), c);
  uint32_t top = addc_last((uint32_t)(p[7] >> 32), 0u, c);          // <= 39
  uint64_t f = mad64(top, 38u, (uint64_t)r.v[0]);
  r.v[0] = (uint32_t)f;
  add_cc(r.v[1], c, r.v[1], (uint32_t)(f >> 32));
#pragma unroll
  for (int i = 2; i < 8; ++i) addc_cc(r.v[i], c, r.v[i], 0u, c);
  // a final carry means r wrapped to a tiny value: add 38 once more (cannot carry again)
  r.v[0] += sel_c(c, 38u, 0u);
  return r;
}

// Product scanning with the reduction folded into the high columns: as soon as column
// k >= 8 is complete its word is multiplied by 38 and added into result word k-8, so the
// upper half of the 512-bit product is never held in registers.
TXV_HD fe fe_mul(const fe& a, const fe& b) {
  fe r;
#if defined(__HIP_DEVICE_COMPILE__)
  fe_mul_dev(r, a, b);   // the same column scan + fold as one asm block (fe_asm.h)
  return r;
#else
  uint64_t acc = 0; uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
#pragma unroll
    for (int i = 0; i <= k; ++i) mac(acc, ovf, a.v[i], b.v[k - i]);
    r.v[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
    ovf = 0;
  }
  uint32_t fc = 0;   // fold carry (<= 39)
#pragma unroll
  for (int k = 8; k < 16; ++k) {
    if (k < 15) {
#pragma unroll
      for (int i = k - 7; i <= 7; ++i) mac(acc, ovf, a.v[i], b.v[k - i]);
    }
    const uint32_t w = (uint32_t)acc;
    if (k < 15) { acc = (acc >> 32) | ((uint64_t)ovf << 32); ovf = 0; }
    uint64_t f = mad64(w, 38u, (uint64_t)r.v[k - 8] + fc);
    r.v[k - 8] = (uint32_t)f;
    fc = (uint32_t)(f >> 32);
  }
  // r += 38 * fc, then a possible final wrap
  uint64_t c;
  uint64_t f = mad64(fc, 38u, (uint64_t)r.v[0]);
  r.v[0] = (uint32_t)f;
  add_cc(r.v[1], c, r.v[1], (uint32_t)(f >> 32));
#pragma unroll
  for (int i = 2; i < 8; ++i) addc_cc(r.v[i], c, r.v[i], 0u, c);
  r.v[0] += sel_c(c, 38u, 0u);
  return r;
#endif
}

TXV_HD fe fe_sq(const fe& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe r;
  fe_sq_dev(r, a);
  return r;
#else
  // off-diagonal triangle U = sum_{i<j} a_i a_j 2^(32(i+j))
  uint32_t u[16];
  uint64_t acc = 0; uint32_t ovf = 0;
  u[0] = 0;
#pragma unroll
  for (int k = 1; k < 14; ++k) {
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); 2 * i < k; ++i) mac(acc, ovf, a.v[i], a.v[k - i]);
    u[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
    ovf = 0;
  }
  u[14] = (uint32_t)acc;
  u[15] = (uint32_t)(acc >> 32);
  // t = 2U + sum a_i^2 2^(64 i)
  uint32_t t[16];
  uint64_t c;
  uint64_t d = mul64(a.v[0], a.v[0]);
  t[0] = (uint32_t)d;                                       // u[0] = 0
  add_cc(t[1], c, (u[1] << 1), (uint32_t)(d >> 32));
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    d = mul64(a.v[i], a.v[i]);
    uint32_t s0 = (u[2 * i] << 1) | (u[2 * i - 1] >> 31);
    uint32_t s1 = (u[2 * i + 1] << 1) | (u[2 * i] >> 31);
    addc_cc(t[2 * i], c, s0, (uint32_t)d, c);
    addc_cc(t[2 * i + 1], c, s1, (uint32_t)(d >> 32), c);
  }
  return fe_reduce512(t);
#endif
}

TXV_HD fe fe_sqn(fe a, int n) {
#pragma nounroll
  for (int i = 0; i < n; ++i) a = fe_sq(a);
  return a;
}

TXV_HD fe fe_add(const fe& a, const fe& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe r;
  fe_add_dev(r, a, b);
  return r;
#else
  fe r; uint64_t c;
  add_cc(r.v[0], c, a.v[0], b.v[0]);
#pragma unroll
  for (int i = 1; i < 8; ++i) addc_cc(r.v[i], c, a.v[i], b.v[i], c);
  // wrap: + 38 * carry
  uint32_t w = sel_c(c, 38u, 0u);
  add_cc(r.v[0], c, r.v[0], w);
#pragma unroll
  for (int i = 1; i < 8; ++i) addc_cc(r.v[i], c, r.v[i], 0u, c);
  r.v[0] += sel_c(c, 38u, 0u);   // second wrap leaves r tiny: no further carry
  return r;
#endif
}

TXV_HD fe fe_sub(const fe& a, const fe& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe r;
  fe_sub_dev(r, a, b);
  return r;
#else
  fe r; uint64_t c;
  sub_cc(r.v[0], c, a.v[0], b.v[0]);
#pragma unroll
  for (int i = 1; i < 8; ++i) subb_cc(r.v[i], c, a.v[i], b.v[i], c);
  // borrow means r = a - b + 2^256 = (a - b) + 38 (mod p) too large by 38: subtract 38
  uint32_t w = sel_c(c, 38u, 0u);
  sub_cc(r.v[0], c, r.v[0], w);
#pragma unroll
  for (int i = 1; i < 8; ++i) subb_cc(r.v[i], c, r.v[i], 0u, c);
  r.v[0] -= sel_c(c, 38u, 0u);   // second borrow leaves r near 2^256: no further borrow
  return r;
#endif
}

TXV_HD fe fe_dbl(const fe& a) { return fe_add(a, a); }
TXV_HD fe fe_neg(const fe& a) { return fe_sub(fe_zero(), a); }

// canonical representative in [0, p)
TXV_HD fe fe_canon(const fe& a) {
  fe r = a; uint64_t c;
  // fold bit 255: r = low255 + 19 * bit255   (< 2^255 + 19)
  uint32_t top = r.v[7] >> 31;
  r.v[7] &= 0x7fffffffu;
  add_cc(r.v[0], c, r.v[0], top * 19u);
#pragma unroll
  for (int i = 1; i < 8; ++i) addc_cc(r.v[i], c, r.v[i], 0u, c);
  // conditional subtract p: t = r + 19; if t >= 2^255 then r = t - 2^255
  fe t;
  add_cc(t.v[0], c, r.v[0], 19u);
#pragma unroll
  for (int i = 1; i < 8; ++i) addc_cc(t.v[i], c, r.v[i], 0u, c);
  bool ge = (t.v[7] >> 31) != 0;
  t.v[7] &= 0x7fffffffu;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = ge ? t.v[i] : r.v[i];
  return r;
}

TXV_HD bool fe_iszero(const fe& a) {
  fe c = fe_canon(a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= c.v[i];
  return o == 0;
}
TXV_HD uint32_t fe_parity(const fe& a) { return fe_canon(a).v[0] & 1u; }
TXV_HD fe fe_select(bool s, const fe& a, const fe& b) {   // s ? a : b
  fe r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = s ? a.v[i] : b.v[i];
  return r;
}

// z^(2^250 - 1) and z^11: shared prefix of the p-2 and (p-5)/8 exponent chains
TXV_HD void fe_pow2501(fe& out250, fe& z11, const fe& z) {
  fe z2 = fe_sq(z);
  fe z8 = fe_sqn(z2, 2);
  fe z9 = fe_mul(z8, z);
  z11 = fe_mul(z9, z2);
  fe z_5_0 = fe_mul(fe_sq(z11), z9);
  fe z_10_0 = fe_mul(fe_sqn(z_5_0, 5), z_5_0);
  fe z_20_0 = fe_mul(fe_sqn(z_10_0, 10), z_10_0);
  fe z_40_0 = fe_mul(fe_sqn(z_20_0, 20), z_20_0);
  fe z_50_0 = fe_mul(fe_sqn(z_40_0, 10), z_10_0);
  fe z_100_0 = fe_mul(fe_sqn(z_50_0, 50), z_50_0);
  fe z_200_0 = fe_mul(fe_sqn(z_100_0, 100), z_100_0);
  out250 = fe_mul(fe_sqn(z_200_0, 50), z_50_0);
}
TXV_HD fe fe_invert(const fe& z) {
  fe t, z11; fe_pow2501(t, z11, z);
  return fe_mul(fe_sqn(t, 5), z11);        // 2^255 - 21 = p - 2
}
TXV_HD fe fe_pow22523(const fe& z) {
  fe t, z11; fe_pow2501(t, z11, z);
  return fe_mul(fe_sqn(t, 2), z);          // 2^252 - 3 = (p - 5) / 8
}

// little-endian 32-byte load with bit 255 cleared (ref10 FeFromBytes semantics)
TXV_HD fe fe_from_words_255(const uint32_t w[8]) {
  fe r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = w[i];
  r.v[7] &= 0x7fffffffu;
  return r;
}

// constants (little-endian 32-bit limbs)
TXV_HD fe fe_const_d() {
  fe r; const uint32_t k[8] = {0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du,
                               0x7779e898u, 0x8cc74079u, 0x2b6ffe73u, 0x52036ceeu};
  for (int i = 0; i < 8; ++i) r.v[i] = k[i];
  return r;
}
TXV_HD fe fe_const_d2() {
  fe r; const uint32_t k[8] = {0x26b2f159u, 0xebd69b94u, 0x8283b156u, 0x00e0149au,
                               0xeef3d130u, 0x198e80f2u, 0x56dffce7u, 0x2406d9dcu};
  for (int i = 0; i < 8; ++i) r.v[i] = k[i];
  return r;
}
TXV_HD fe fe_const_sqrtm1() {
  fe r; const uint32_t k[8] = {0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u,
                               0x3dfbd7a7u, 0x2b4d0099u, 0x4fc1df0bu, 0x2b832480u};
  for (int i = 0; i < 8; ++i) r.v[i] = k[i];
  return r;
}

}  // namespace txv
