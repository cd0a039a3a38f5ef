// fe10.h — GF(2^255 - 19) in 10 unsigned limbs of radix 2^25.5 (26, 25, 26, 25, ... bits) for the
// table walk of K1b (ge.h ge10_madd), the dominant kernel.
//
// Why a second representation (DESIGN.md §K1b field arithmetic): on gfx950 every integer op a
// radix-2^32 multiply needs (v_mad_u64_u32, v_add_co/addc) issues at ~0.55 of the rate of a plain
// v_add_u32 / v_and_b32 / v_lshrrev_b32 (profiles/r01/valu_rates.json), and the radix-2^32
// product scan spends one carry add per partial product.  With 25.5-bit limbs the 100 partial
// products accumulate carry-free in 64-bit column sums (each ONE v_mad_u64_u32, the running
// column carry riding in as the first product's addend), additions and subtractions are 10
// carry-free fast-class adds, and the reduction is one 64-bit shift + mask per column.
//
// Limb i sits at bit offset o(i) = 25 i + ceil(i / 2); o(i) + o(j) = o(i + j) + [i, j both odd],
// and 2^(o(k + 10)) = 2^255 2^(o(k)) = 19 2^(o(k)) (mod p).
//
// Bounds (all unsigned, checked in tests/cpu_emu against 2^255 - 19 arithmetic):
//   "carried"  output of fe10_mul / fe10_carry: limb i < 2^w(i), limb 1 < 2^25 + 2^18
//   fe10_mul(f, g) needs f_i < 4 * 2^w(i) and g_i < 3 * 2^w(i) (so 19 g_i < 2^32); every column
//              sum then stays below 2^62.6
//   fe10_add(a, b) of carried a, b: < 2 * 2^w       fe10_sub(a, b) = a - b + 2p, b carried:
//              < a + 2 * 2^w  (3 * 2^w for carried a)
// The device code is plain C++: the compiler turns (u64) a * b + acc into v_mad_u64_u32 and
// allocates the registers (no asm blocks, so no hazard nops between them).
#pragma once
#include "fe.h"

namespace txv {

struct fe10 { uint32_t v[10]; };

#define TXV_W10(i) (((i) & 1) ? 25 : 26)
#define TXV_M10(i) (((i) & 1) ? 0x1ffffffu : 0x3ffffffu)

// 2p in limb form: (2^26 - 19) * 2 for limb 0, 2 (2^w - 1) elsewhere
TXV_HD uint32_t fe10_2p(int i) { return i == 0 ? 0x7ffffdau : ((i & 1) ? 0x3fffffeu : 0x7fffffeu); }

TXV_HD fe10 fe10_zero() { fe10 r; for (int i = 0; i < 10; ++i) r.v[i] = 0; return r; }
TXV_HD fe10 fe10_one() { fe10 r = fe10_zero(); r.v[0] = 1; return r; }

TXV_HD fe10 fe10_add(const fe10& a, const fe10& b) {
  fe10 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = a.v[i] + b.v[i];
  return r;
}
// a - b + 2p (b carried)
TXV_HD fe10 fe10_sub(const fe10& a, const fe10& b) {
  fe10 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = (a.v[i] + fe10_2p(i)) - b.v[i];
  return r;
}
// neg ? 2p - a : a   (a carried; result < 2 * 2^w), branch-free per lane
TXV_HD fe10 fe10_cneg(const fe10& a, bool neg) {
  const uint32_t m = neg ? 0xffffffffu : 0u;
  fe10 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = (a.v[i] ^ m) + (m & (fe10_2p(i) + 1u));   // ~a + 1 + 2p = 2p - a
  return r;
}

// one sequential carry pass over 32-bit limbs (any limbs < 2^32 - 2^7): carried output
TXV_HD fe10 fe10_carry(const fe10& a) {
  fe10 r = a;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t t = r.v[i] + c;
    c = t >> TXV_W10(i);
    r.v[i] = t & TXV_M10(i);
  }
  const uint32_t t = r.v[0] + 19u * c;   // c < 2^8
  r.v[0] = t & 0x3ffffffu;
  r.v[1] += t >> 26;
  return r;
}

// cin + sum_{i<10} a_i b_i: on the device ONE asm block of 10 chained v_mad_u64_u32 with the
// carry-in as the first addend (left to itself the compiler sums the 10 columns independently
// and adds each carry with an extra v_lshl_add_u64, holding 10 accumulator pairs live)
#ifndef TXV_FE10_MUL
#define TXV_FE10_MUL 1
#endif
TXV_HD uint64_t fe10_col(uint64_t cin, const uint32_t a[10], const uint32_t b[10]) {
#if defined(__HIP_DEVICE_COMPILE__) && TXV_FE10_MUL == 2
  // two interleaved 5-product chains (independent until the final add)
  uint64_t x, y, cc;
  asm("v_mad_u64_u32 %0, %2, %3, %13, %23\n\t"
      "v_mad_u64_u32 %1, %2, %4, %14, 0\n\t"
      "v_mad_u64_u32 %0, %2, %5, %15, %0\n\t"
      "v_mad_u64_u32 %1, %2, %6, %16, %1\n\t"
      "v_mad_u64_u32 %0, %2, %7, %17, %0\n\t"
      "v_mad_u64_u32 %1, %2, %8, %18, %1\n\t"
      "v_mad_u64_u32 %0, %2, %9, %19, %0\n\t"
      "v_mad_u64_u32 %1, %2, %10, %20, %1\n\t"
      "v_mad_u64_u32 %0, %2, %11, %21, %0\n\t"
      "v_mad_u64_u32 %1, %2, %12, %22, %1\n\t"
      "v_lshl_add_u64 %0, %0, 0, %1"
      : "=&v"(x), "=&v"(y), "=&s"(cc)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]), "v"(a[9]),
        "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]), "v"(b[8]), "v"(b[9]),
        "v"(cin));
  return x;
#elif defined(__HIP_DEVICE_COMPILE__) && TXV_FE10_MUL == 1
  uint64_t acc, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %12, %22\n\t"
      "v_mad_u64_u32 %0, %1, %3, %13, %0\n\t"
      "v_mad_u64_u32 %0, %1, %4, %14, %0\n\t"
      "v_mad_u64_u32 %0, %1, %5, %15, %0\n\t"
      "v_mad_u64_u32 %0, %1, %6, %16, %0\n\t"
      "v_mad_u64_u32 %0, %1, %7, %17, %0\n\t"
      "v_mad_u64_u32 %0, %1, %8, %18, %0\n\t"
      "v_mad_u64_u32 %0, %1, %9, %19, %0\n\t"
      "v_mad_u64_u32 %0, %1, %10, %20, %0\n\t"
      "v_mad_u64_u32 %0, %1, %11, %21, %0"
      : "=&v"(acc), "=&s"(cc)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]), "v"(a[9]),
        "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]), "v"(b[8]), "v"(b[9]),
        "v"(cin));
  return acc;
#else
  uint64_t acc = cin;
  for (int i = 0; i < 10; ++i) acc += (uint64_t)a[i] * b[i];
  return acc;
#endif
}

// h = f * g (mod p), carried.  Column k collects f_i g_j over i + j = k (doubled when i and j
// are both odd, i.e. i odd and k even) and, times 19, over i + j = k + 10; the column's carry into
// k + 1 is the first addend of column k + 1, the carry out of column 9 wraps into limb 0 times 19.
TXV_HD fe10 fe10_mul(const fe10& f, const fe10& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int j = 1; j < 10; ++j) g19[j] = 19u * g.v[j];
#pragma unroll
  for (int i = 0; i < 10; ++i) f2[i] = (i & 1) ? f.v[i] + f.v[i] : f.v[i];
  g19[0] = 0;
  fe10 h;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    uint32_t a[10], b[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      a[i] = ((i & 1) && !(k & 1)) ? f2[i] : f.v[i];
      b[i] = i <= k ? g.v[k - i] : g19[k + 10 - i];
    }
    acc = fe10_col(acc, a, b);
    h.v[k] = (uint32_t)acc & TXV_M10(k);
    acc >>= TXV_W10(k);
  }
  // acc < 2^39: limb 0 += 19 acc, then one carry into limb 1
  const uint64_t t = (uint64_t)(uint32_t)acc * 19u + h.v[0] + ((uint64_t)((uint32_t)(acc >> 32) * 19u) << 32);
  h.v[0] = (uint32_t)t & 0x3ffffffu;
  h.v[1] += (uint32_t)(t >> 26);
  return h;
}

// Two independent products with their column chains interleaved.  fe10_mul is ONE dependency
// chain of 100 v_mad_u64_u32 (each column's carry is the next column's first addend), and a wave
// issues it with nothing else to fill the mad's latency; two products in one asm block per column
// (the mads of both chains alternating) give every mad an independent neighbour, at no extra
// instruction (unlike splitting one column into two chains, which costs a 64-bit add per column).
TXV_HD void fe10_col2(uint64_t c1, const uint32_t a[10], const uint32_t b[10], uint64_t c2, const uint32_t x[10],
                      const uint32_t y[10], uint64_t& o1, uint64_t& o2) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t p, q, cc;
  asm("v_mad_u64_u32 %0, %2, %3, %13, %43\n\t"
      "v_mad_u64_u32 %1, %2, %23, %33, %44\n\t"
      "v_mad_u64_u32 %0, %2, %4, %14, %0\n\t"
      "v_mad_u64_u32 %1, %2, %24, %34, %1\n\t"
      "v_mad_u64_u32 %0, %2, %5, %15, %0\n\t"
      "v_mad_u64_u32 %1, %2, %25, %35, %1\n\t"
      "v_mad_u64_u32 %0, %2, %6, %16, %0\n\t"
      "v_mad_u64_u32 %1, %2, %26, %36, %1\n\t"
      "v_mad_u64_u32 %0, %2, %7, %17, %0\n\t"
      "v_mad_u64_u32 %1, %2, %27, %37, %1\n\t"
      "v_mad_u64_u32 %0, %2, %8, %18, %0\n\t"
      "v_mad_u64_u32 %1, %2, %28, %38, %1\n\t"
      "v_mad_u64_u32 %0, %2, %9, %19, %0\n\t"
      "v_mad_u64_u32 %1, %2, %29, %39, %1\n\t"
      "v_mad_u64_u32 %0, %2, %10, %20, %0\n\t"
      "v_mad_u64_u32 %1, %2, %30, %40, %1\n\t"
      "v_mad_u64_u32 %0, %2, %11, %21, %0\n\t"
      "v_mad_u64_u32 %1, %2, %31, %41, %1\n\t"
      "v_mad_u64_u32 %0, %2, %12, %22, %0\n\t"
      "v_mad_u64_u32 %1, %2, %32, %42, %1"
      : "=&v"(p), "=&v"(q), "=&s"(cc)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]), "v"(a[9]),
        "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]), "v"(b[8]), "v"(b[9]),
        "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]), "v"(x[8]), "v"(x[9]),
        "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]), "v"(y[4]), "v"(y[5]), "v"(y[6]), "v"(y[7]), "v"(y[8]), "v"(y[9]),
        "v"(c1), "v"(c2));
  o1 = p;
  o2 = q;
#else
  uint64_t p = c1, q = c2;
  for (int i = 0; i < 10; ++i) {
    p += (uint64_t)a[i] * b[i];
    q += (uint64_t)x[i] * y[i];
  }
  o1 = p;
  o2 = q;
#endif
}

// h1 = f1 * g1, h2 = f2 * g2 (mod p), carried: fe10_mul twice, same bounds, columns interleaved
TXV_HD void fe10_mul2(const fe10& f1, const fe10& g1, const fe10& f2, const fe10& g2, fe10& h1, fe10& h2) {
  uint32_t g19a[10], f2a[10], g19b[10], f2b[10];
#pragma unroll
  for (int j = 1; j < 10; ++j) {
    g19a[j] = 19u * g1.v[j];
    g19b[j] = 19u * g2.v[j];
  }
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    f2a[i] = (i & 1) ? f1.v[i] + f1.v[i] : f1.v[i];
    f2b[i] = (i & 1) ? f2.v[i] + f2.v[i] : f2.v[i];
  }
  g19a[0] = g19b[0] = 0;
  fe10 r1, r2;
  uint64_t acc1 = 0, acc2 = 0;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    uint32_t a[10], b[10], x[10], y[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const bool dbl = (i & 1) && !(k & 1);
      a[i] = dbl ? f2a[i] : f1.v[i];
      x[i] = dbl ? f2b[i] : f2.v[i];
      b[i] = i <= k ? g1.v[k - i] : g19a[k + 10 - i];
      y[i] = i <= k ? g2.v[k - i] : g19b[k + 10 - i];
    }
    fe10_col2(acc1, a, b, acc2, x, y, acc1, acc2);
    r1.v[k] = (uint32_t)acc1 & TXV_M10(k);
    r2.v[k] = (uint32_t)acc2 & TXV_M10(k);
    acc1 >>= TXV_W10(k);
    acc2 >>= TXV_W10(k);
  }
  const uint64_t t1 = (uint64_t)(uint32_t)acc1 * 19u + r1.v[0] + ((uint64_t)((uint32_t)(acc1 >> 32) * 19u) << 32);
  const uint64_t t2 = (uint64_t)(uint32_t)acc2 * 19u + r2.v[0] + ((uint64_t)((uint32_t)(acc2 >> 32) * 19u) << 32);
  r1.v[0] = (uint32_t)t1 & 0x3ffffffu;
  r1.v[1] += (uint32_t)(t1 >> 26);
  r2.v[0] = (uint32_t)t2 & 0x3ffffffu;
  r2.v[1] += (uint32_t)(t2 >> 26);
  h1 = r1;
  h2 = r2;
}

// fully carried: every limb < 2^w(i), value < 2^255 (+ the value itself may still be >= p)
TXV_HD fe10 fe10_strict(const fe10& a) {
  fe10 r = fe10_carry(a);
  uint32_t c = 0;
#pragma unroll
  for (int i = 1; i < 10; ++i) {
    const uint32_t t = r.v[i] + c;
    c = t >> TXV_W10(i);
    r.v[i] = t & TXV_M10(i);
  }
  // a carry out of limb 9 here means the value wrapped past 2^255: add 19; the upper limbs are
  // then (near) zero, so limb 0's own carry stops in limb 1
  const uint32_t t = r.v[0] + 19u * c;
  r.v[0] = t & 0x3ffffffu;
  r.v[1] += t >> 26;
  return r;
}

// radix-2^32 (weakly reduced, < 2^256) -> carried limbs (limb 0 may exceed 2^26 by 19 when bit 255
// was set; every bound above has the slack)
TXV_HD fe10 fe10_from_fe(const fe& a) {
  fe10 r;
  const uint32_t top = a.v[7] >> 31;          // bit 255 = 19 (mod p)
  int bit = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int w = bit >> 5, s = bit & 31;
    uint32_t x = a.v[w] >> s;
    if (s + TXV_W10(i) > 32 && w < 7) x |= a.v[w + 1] << (32 - s);
    r.v[i] = x & TXV_M10(i);
    bit += TXV_W10(i);
  }
  r.v[0] += 19u * top;
  return r;
}

// limbs -> radix-2^32 (< 2^255 + 19: weakly reduced)
TXV_HD fe fe_from_fe10(const fe10& a) {
  const fe10 s = fe10_strict(a);
  fe r;
#pragma unroll
  for (int w = 0; w < 8; ++w) r.v[w] = 0;
  int bit = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int w = bit >> 5, sh = bit & 31;
    r.v[w] |= s.v[i] << sh;
    if (sh + TXV_W10(i) > 32 && w < 7) r.v[w + 1] |= s.v[i] >> (32 - sh);
    bit += TXV_W10(i);
  }
  return r;
}

}  // namespace txv
