// sc.h — scalars mod L = 2^252 + 27742317777372353535851937790883648493 on 32-bit limbs.
//
// x/crypto ed25519.Verify (external) needs two scalar steps:
//   ScReduce:  k = SHA-512(R || A || M) mod L       -> sc_reduce512 (Barrett, b = 2^32)
//   ScMinimal: reject unless s < L                   -> sc_lt_L
// Signed radix-16 recoding (digits in [-8, 7]) drives the fixed-base table walk in ge.h.
// Any exact reduction yields the same canonical k, so bit parity only requires exactness.
#pragma once
#include "fe.h"

namespace txv {

struct sc { uint32_t v[8]; };

TXV_HD uint32_t L_limb(int i) {
  // L little-endian 32-bit limbs
  return i == 0 ? 0x5cf5d3edu : i == 1 ? 0x5812631au : i == 2 ? 0xa2f79cd6u : i == 3 ? 0x14def9deu
       : i == 7 ? 0x10000000u : 0u;
}
TXV_HD uint32_t MU_limb(int i) {
  // floor(2^512 / L), 9 limbs
  return i == 0 ? 0x0a2c131bu : i == 1 ? 0xed9ce5a3u : i == 2 ? 0x086329a7u : i == 3 ? 0x2106215du
       : i == 4 ? 0xffffffebu : i == 8 ? 0xfu : 0xffffffffu;
}

// s < L ?  (ScMinimal semantics)
TXV_HD bool sc_lt_L(const uint32_t s[8]) {
  // borrow of s - L tells s < L
  uint32_t d; uint64_t c;
  sub_cc(d, c, s[0], L_limb(0));
#pragma unroll
  for (int i = 1; i < 8; ++i) subb_cc(d, c, s[i], L_limb(i), c);
  return addc_last(0u, 0u, c) != 0u;
}

// x (16 limbs, < 2^512) mod L   — HAC 14.42 with b = 2^32, k = 8
TXV_HD sc sc_reduce512(const uint32_t x[16]) {
  // q1 = x >> 224 (9 limbs); q2 = q1 * mu; q3 = q2 >> 288
  uint32_t q3[9];
  {
    uint64_t acc = 0; uint32_t ovf = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
#pragma unroll
      for (int i = (k > 8 ? k - 8 : 0); i <= (k < 8 ? k : 8); ++i) mac(acc, ovf, x[7 + i], MU_limb(k - i));
      if (k >= 9) q3[k - 9] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)ovf << 32);
      ovf = 0;
    }
    q3[8] = (uint32_t)acc;
  }
  // r2 = (q3 * L) mod 2^288
  uint32_t r2[9];
  {
    uint64_t acc = 0; uint32_t ovf = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
#pragma unroll
      for (int i = 0; i <= k; ++i) {
        if (L_limb(k - i) != 0u && k - i < 8) mac(acc, ovf, q3[i], L_limb(k - i));
      }
      r2[k] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)ovf << 32);
      ovf = 0;
    }
  }
  // r = x[0..8] - r2  (mod 2^288)
  uint32_t r[9]; uint64_t c;
  sub_cc(r[0], c, x[0], r2[0]);
#pragma unroll
  for (int i = 1; i < 9; ++i) subb_cc(r[i], c, x[i], r2[i], c);
  // at most two conditional subtractions of L
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    uint32_t t[9];
    sub_cc(t[0], c, r[0], L_limb(0));
#pragma unroll
    for (int i = 1; i < 9; ++i) subb_cc(t[i], c, r[i], i < 8 ? L_limb(i) : 0u, c);
    bool lt = addc_last(0u, 0u, c) != 0u;   // r < L
#pragma unroll
    for (int i = 0; i < 9; ++i) r[i] = lt ? r[i] : t[i];
  }
  sc out;
#pragma unroll
  for (int i = 0; i < 8; ++i) out.v[i] = r[i];
  return out;
}

// (signed radix-2^W recoding lives in ed25519_dev.h: sc_recode<W>, sc_digit<W>)

}  // namespace txv
