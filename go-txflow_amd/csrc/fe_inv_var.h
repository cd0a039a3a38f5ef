// fe_inv_var.h — variable-time inverse in GF(2^255 - 19) by Bernstein–Yang divsteps
// ("Fast constant-time gcd computation and modular inversion", 2019), in the variable-time
// form with 30-divstep batches on signed 30-bit limbs.
//
// Why: x/crypto's encode(R') needs 1/Z once per verified vote; the Fermat chain (254 squarings
// + 11 multiplies, fe_invert) is ~32k VALU instructions per lane, and under SIMD its cost per
// vote only falls with more votes per lane (split mode).  Verification works
// on public data, so a variable-time inverse is admissible: each 30-divstep batch is ~10
// 32-bit ops per divstep on one word, then one 2x2 matrix applied to (f, g) and (d, e) with
// 9-limb signed 32x32->64 multiply-adds.  Result: canonical z^-1 mod p (0 for z = 0), the
// same value fe_invert returns after fe_canon.
#pragma once
#include "fe.h"

namespace txv {

struct s30 { int32_t v[9]; };   // value = sum v[i] 2^(30 i); v[0..7] in [0, 2^30), v[8] signed

constexpr int32_t kM30 = 0x3FFFFFFF;
// p = 2^255 - 19 in signed-30 limbs
TXV_HD int32_t p30(int i) { return i == 0 ? 0x3FFFFFED : (i == 8 ? 0x7FFF : 0x3FFFFFFF); }
// p^-1 mod 2^30 (Newton from p0 = -19 mod 2^30)
constexpr uint32_t inv30_p() {
  uint32_t p0 = 0x3FFFFFEDu, x = p0;
  for (int i = 0; i < 5; ++i) x *= 2u - p0 * x;
  return x & 0x3FFFFFFFu;
}
constexpr uint32_t kPInv30 = inv30_p();
static_assert((0x3FFFFFEDu * kPInv30 & 0x3FFFFFFFu) == 1u, "p^-1 mod 2^30");

// f^-1 mod 256 for odd f (Newton: exact mod 8, then mod 64, mod 4096)
TXV_HD uint32_t inv256_odd(uint32_t f) {
  uint32_t x = f;
  x *= 2u - f * x;
  x *= 2u - f * x;
  return x;
}

// 30 divsteps on the low words of f (odd) and g; t = transition matrix scaled by 2^30
TXV_HD int32_t divsteps30_var(int32_t eta, uint32_t f, uint32_t g, int32_t t[4]) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  int i = 30;
  for (;;) {
    const int zeros = __builtin_ctz(g | (0xFFFFFFFFu << i));
    g >>= zeros; u <<= zeros; v <<= zeros; eta -= zeros; i -= zeros;
    if (i == 0) break;
    if (eta < 0) {   // delta > 0: (f, g) <- (g, -f)
      uint32_t tmp;
      eta = -eta;
      tmp = f; f = g; g = 0u - tmp;
      tmp = u; u = q; q = 0u - tmp;
      tmp = v; v = r; r = 0u - tmp;
    }
    // cancel up to min(eta + 1, i) low bits of g at once (at most 8)
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = (0xFFFFFFFFu >> (32 - limit)) & 255u;
    const uint32_t w = (g * inv256_odd(f)) & m;   // g - w f = 0 mod 2^limit
    g -= f * w; q -= u * w; r -= v * w;
  }
  t[0] = (int32_t)u; t[1] = (int32_t)v; t[2] = (int32_t)q; t[3] = (int32_t)r;
  return eta;
}

// (f, g) <- t (f, g) / 2^30 (exact division by construction).  All 9 limbs, fully unrolled:
// shrinking the length as f, g lose bits (as CPU implementations do) would index the limb
// arrays dynamically, which puts them in scratch memory on the GPU.
TXV_HD void update_fg30(s30& f, s30& g, const int32_t t[4]) {
  const int64_t u = t[0], v = t[1], q = t[2], r = t[3];
  int64_t cf = u * f.v[0] + v * g.v[0], cg = q * f.v[0] + r * g.v[0];
  cf >>= 30; cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    cf += u * f.v[i] + v * g.v[i];
    cg += q * f.v[i] + r * g.v[i];
    f.v[i - 1] = (int32_t)cf & kM30; g.v[i - 1] = (int32_t)cg & kM30;
    cf >>= 30; cg >>= 30;
  }
  f.v[8] = (int32_t)cf; g.v[8] = (int32_t)cg;
}

// (d, e) <- t (d, e) / 2^30 mod p, kept in (-2p, p): multiples of p are added so the low
// 30 bits cancel (d, e enter in (-2p, p); the sign corrections keep the bound)
TXV_HD void update_de30(s30& d, s30& e, const int32_t t[4]) {
  const int64_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
  int32_t md = (t[0] & sd) + (t[1] & se);
  int32_t me = (t[2] & sd) + (t[3] & se);
  int64_t cd = u * d.v[0] + v * e.v[0], ce = q * d.v[0] + r * e.v[0];
  md -= (int32_t)((kPInv30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)kM30);
  me -= (int32_t)((kPInv30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)kM30);
  cd += (int64_t)p30(0) * md; ce += (int64_t)p30(0) * me;
  cd >>= 30; ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    cd += u * d.v[i] + v * e.v[i] + (int64_t)p30(i) * md;
    ce += q * d.v[i] + r * e.v[i] + (int64_t)p30(i) * me;
    d.v[i - 1] = (int32_t)cd & kM30; e.v[i - 1] = (int32_t)ce & kM30;
    cd >>= 30; ce >>= 30;
  }
  d.v[8] = (int32_t)cd; e.v[8] = (int32_t)ce;
}

TXV_HD void s30_carry(s30& a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) { a.v[i + 1] += a.v[i] >> 30; a.v[i] &= kM30; }
}
TXV_HD void s30_add_p_if(s30& a, int32_t mask) {
#pragma unroll
  for (int i = 0; i < 9; ++i) a.v[i] += p30(i) & mask;
  s30_carry(a);
}

// batches_out (host tests): the 30-divstep batches run, or -1 if g had not reached 0 at the cap
TXV_HD fe fe_invert_var_n(const fe& z, int& batches_out) {
  const fe c = fe_canon(z);
  s30 f, g, d, e;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int bit = 30 * i, w = bit >> 5, off = bit & 31;
    uint32_t x = c.v[w] >> off;
    if (off > 2 && w + 1 < 8) x |= c.v[w + 1] << (32 - off);
    g.v[i] = (int32_t)(x & (uint32_t)kM30);
    f.v[i] = p30(i);
    d.v[i] = 0;
    e.v[i] = 0;
  }
  e.v[0] = 1;
  int32_t eta = -1;
  int32_t t[4];
  // <= 25 batches for 255-bit inputs (Bernstein–Yang bound: 724 divsteps); the cap only
  // guarantees termination
  batches_out = -1;
#pragma unroll 1
  for (int it = 0; it < 32; ++it) {
    eta = divsteps30_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    update_de30(d, e, t);
    update_fg30(f, g, t);
    int32_t any = 0;
#pragma unroll
    for (int j = 0; j < 9; ++j) any |= g.v[j];
    if (!any) { batches_out = it + 1; break; }
  }
  // f = +-1: z^-1 = d * f, brought from (-2p, p) into [0, p)
  const int32_t neg = f.v[8] >> 31;
  s30_add_p_if(d, d.v[8] >> 31);
#pragma unroll
  for (int i = 0; i < 9; ++i) d.v[i] = (d.v[i] ^ neg) - neg;
  s30_carry(d);
  s30_add_p_if(d, d.v[8] >> 31);
  fe out;
  uint64_t acc = 0;
  int nbits = 0, k = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    acc |= (uint64_t)(uint32_t)d.v[i] << nbits;
    nbits += 30;
    if (nbits >= 32 && k < 8) { out.v[k++] = (uint32_t)acc; acc >>= 32; nbits -= 32; }
  }
  while (k < 8) { out.v[k++] = (uint32_t)acc; acc >>= 32; }
  return out;
}
TXV_HD fe fe_invert_var(const fe& z) {
  int batches;
  return fe_invert_var_n(z, batches);
}

}  // namespace txv
