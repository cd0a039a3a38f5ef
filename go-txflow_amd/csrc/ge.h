// ge.h — edwards25519 group law (a = -1, d = -121665/121666) in extended coordinates.
//
// Formulas are the complete HWCD (Hisil-Wong-Carter-Dawson 2008) ones: the unified
// addition is exact for every pair of curve points, including the identity, torsion and
// small-order points that the adversarial validator set contains,
// so [s]B + [k](-A) comes out as the same group element x/crypto computes and its
// canonical encoding is bit-identical (Appendix A.1 step 6).
//
// Precomputed table entries are half-Niels triples ((y+x)/2, (y-x)/2, d*x*y) in fe10 limbs,
// 128 bytes each (ge10_madd below); a mixed add costs 7 field multiplies.
#pragma once
#include "fe.h"
#include "fe10.h"

namespace txv {

struct ge_ext { fe X, Y, Z, T; };
struct ge_niels { fe ypx, ymx, xy2d; };

TXV_HD ge_ext ge_identity() {
  ge_ext r; r.X = fe_zero(); r.Y = fe_one(); r.Z = fe_one(); r.T = fe_zero(); return r;
}

// ---------------------------------------------------------------- table walk (K1b)
// The fixed-base tables hold each multiple Q = (x, y) as a HALF-Niels entry
//   qp = (y + x) / 2, qm = (y - x) / 2, qd = d x y        (mod p, canonical, fe10 limbs)
// With them the mixed addition below computes (E, H, G, F) = 1/2 of HWCD's
// (B - A, B + A, 2Z + 2d T x y, 2Z - 2d T x y), so (X3, Y3, Z3, T3) = 1/4 of the HWCD sum: the
// same projective point, and no doubling of Z -- which keeps every operand inside fe10_mul's
// bounds without a carry pass.  7 multiplies, 6 carry-free adds/subs, one conditional negation.
struct ge10_ext { fe10 X, Y, Z, T; };

// P + Q or P - Q: the caller passes (qp, qm) already swapped for -Q (the swap is an address
// choice when loading); neg negates qd's product
TXV_HD ge10_ext ge10_madd(const ge10_ext& p, const fe10& qp, const fe10& qm, const fe10& qd, bool neg) {
  // C first: T and qd die before the other products (register peak, 4 waves/SIMD at 128 VGPRs)
  const fe10 C = fe10_cneg(fe10_mul(p.T, qd), neg);
  TXV_SCHED_FENCE();
  const fe10 A = fe10_mul(fe10_sub(p.Y, p.X), qm);
  TXV_SCHED_FENCE();
  const fe10 B = fe10_mul(fe10_add(p.Y, p.X), qp);
  TXV_SCHED_FENCE();
  const fe10 E = fe10_sub(B, A), H = fe10_add(B, A);
  const fe10 G = fe10_add(p.Z, C), F = fe10_sub(p.Z, C);
  ge10_ext r;
  r.X = fe10_mul(F, E);
  TXV_SCHED_FENCE();
  r.Y = fe10_mul(H, G);
  TXV_SCHED_FENCE();
  r.Z = fe10_mul(F, G);
  TXV_SCHED_FENCE();
  r.T = fe10_mul(H, E);
  TXV_SCHED_FENCE();
  return r;
}

// the same addition with the entry read piecewise right before each use (rd(0) = qp, rd(1) = qm,
// rd(2) = qd, already swapped for -Q): only one of them is live at a time, which keeps the
// prefetching K1b walk inside 128 VGPRs; mid() runs once all three are read (the walk issues its
// next prefetch there, into the buffer just read)
// kT = false: the last addition of a walk (its T is never read)
// TXV_MUL_PAIRS=1: the 7 products as interleaved pairs (fe10_mul2).  Measured equal (589 vs 592M
// votes/s, profiles/r02) and 20 VGPRs more (218 vs 198), which leaves no room for a K1a wave
// beside two K1b waves on a SIMD: off by default
#ifndef TXV_MUL_PAIRS
#define TXV_MUL_PAIRS 0
#endif
template <bool kT = true, class Rd, class Mid>
TXV_HD ge10_ext ge10_madd_rd(const ge10_ext& p, Rd rd, bool neg, Mid mid) {
#if TXV_MUL_PAIRS
  // the 7 products as 3 interleaved pairs + 1 (fe10_mul2): (C, A), B, (X3, Y3), (Z3, T3)
  fe10 Cm, A;
  fe10_mul2(p.T, rd(2), fe10_sub(p.Y, p.X), rd(1), Cm, A);
  const fe10 C = fe10_cneg(Cm, neg);
  TXV_SCHED_FENCE();
  const fe10 B = fe10_mul(fe10_add(p.Y, p.X), rd(0));
  TXV_SCHED_FENCE();
  mid();
  const fe10 E = fe10_sub(B, A), H = fe10_add(B, A);
  const fe10 G = fe10_add(p.Z, C), F = fe10_sub(p.Z, C);
  ge10_ext r;
  fe10_mul2(F, E, H, G, r.X, r.Y);
  TXV_SCHED_FENCE();
  if (kT) {
    fe10_mul2(F, G, H, E, r.Z, r.T);
    TXV_SCHED_FENCE();
  } else {
    r.Z = fe10_mul(F, G);
    TXV_SCHED_FENCE();
    r.T = fe10_zero();
  }
  return r;
#else
  const fe10 C = fe10_cneg(fe10_mul(p.T, rd(2)), neg);
  TXV_SCHED_FENCE();
  const fe10 A = fe10_mul(fe10_sub(p.Y, p.X), rd(1));
  TXV_SCHED_FENCE();
  const fe10 B = fe10_mul(fe10_add(p.Y, p.X), rd(0));
  TXV_SCHED_FENCE();
  mid();
  const fe10 E = fe10_sub(B, A), H = fe10_add(B, A);
  const fe10 G = fe10_add(p.Z, C), F = fe10_sub(p.Z, C);
  // E and G are the g operands (the ones fe10_mul multiplies by 19) of two products each, so
  // their 19x limbs are computed once
  ge10_ext r;
  r.X = fe10_mul(F, E);
  TXV_SCHED_FENCE();
  r.Y = fe10_mul(H, G);
  TXV_SCHED_FENCE();
  r.Z = fe10_mul(F, G);
  TXV_SCHED_FENCE();
  if (kT) {
    r.T = fe10_mul(H, E);
    TXV_SCHED_FENCE();
  } else {
    r.T = fe10_zero();
  }
  return r;
#endif
}

// the entry's own point (Z = 1): x = qp - qm, y = qp + qm, T = x y
TXV_HD ge10_ext ge10_from_entry(const fe10& qp, const fe10& qm) {
  ge10_ext r;
  r.X = fe10_carry(fe10_sub(qp, qm));
  r.Y = fe10_carry(fe10_add(qp, qm));
  r.Z = fe10_one();
  r.T = fe10_mul(r.X, r.Y);
  return r;
}

// P + Q for two extended points in fe10 (add-2008-hwcd-3, a = -1, k = 2d): 9 multiplies; the
// lane-quad combine of the split K1b (txv_k_scalarmult_split).  Inputs carried (fe10_mul outputs
// or ge10_from_entry), output carried.  Operand bounds: Y - X < 3 * 2^w (g ok), Y + X < 2 * 2^w;
// D = 2 Z1 Z2 carried once more, so F = D - C < 3 * 2^w and G = D + C < 2 * 2^w; E = B - A
// < 3 * 2^w is only ever the g operand, F only the f operand.
TXV_HD ge10_ext ge10_add(const ge10_ext& p, const ge10_ext& q) {
  const fe10 A = fe10_mul(fe10_sub(p.Y, p.X), fe10_sub(q.Y, q.X));
  const fe10 B = fe10_mul(fe10_add(p.Y, p.X), fe10_add(q.Y, q.X));
  const fe10 C = fe10_mul(fe10_mul(p.T, q.T), fe10_from_fe(fe_const_d2()));
  const fe10 Zz = fe10_mul(p.Z, q.Z);
  const fe10 D = fe10_carry(fe10_add(Zz, Zz));
  const fe10 E = fe10_sub(B, A), H = fe10_add(B, A), G = fe10_add(D, C), F = fe10_sub(D, C);
  ge10_ext r;
  r.X = fe10_mul(F, E);
  r.Y = fe10_mul(H, G);
  r.Z = fe10_mul(F, G);
  r.T = fe10_mul(H, E);
  return r;
}

// (p + 1) / 2
TXV_HD fe fe_const_half() {
  fe r; const uint32_t k[8] = {0xfffffff7u, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                               0xffffffffu, 0xffffffffu, 0xffffffffu, 0x3fffffffu};
  for (int i = 0; i < 8; ++i) r.v[i] = k[i];
  return r;
}

// table entry words: qp at 0..9, qm at 12..21 (both 16-byte aligned, so the sign swap is an
// address offset), qd at 22..31; words 10, 11 zero.  32 words = one 128-byte line.
constexpr int kEntryWords = 32;
constexpr int kEntryQm = 12;
constexpr int kEntryQd = 22;

TXV_HD void entry_words(uint32_t e[kEntryWords], const fe& ypx, const fe& ymx, const fe& xy2d) {
  const fe h = fe_const_half();
  const fe10 qp = fe10_from_fe(fe_canon(fe_mul(ypx, h)));
  const fe10 qm = fe10_from_fe(fe_canon(fe_mul(ymx, h)));
  const fe10 qd = fe10_from_fe(fe_canon(fe_mul(xy2d, h)));
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    e[i] = qp.v[i];
    e[kEntryQm + i] = qm.v[i];
    e[kEntryQd + i] = qd.v[i];
  }
  e[10] = 0;
  e[11] = 0;
}
// the identity's entry (y + x = y - x = 1, 2dxy = 0)
TXV_HD void entry_identity(uint32_t e[kEntryWords]) { entry_words(e, fe_one(), fe_one(), fe_zero()); }

// extended + extended (add-2008-hwcd-3), used by the table builder
TXV_HD ge_ext ge_add(const ge_ext& p, const ge_ext& q) {
  fe A = fe_mul(fe_sub(p.Y, p.X), fe_sub(q.Y, q.X));
  fe B = fe_mul(fe_add(p.Y, p.X), fe_add(q.Y, q.X));
  fe C = fe_mul(fe_mul(p.T, q.T), fe_const_d2());
  fe D = fe_dbl(fe_mul(p.Z, q.Z));
  fe E = fe_sub(B, A), H = fe_add(B, A), G = fe_add(D, C), F = fe_sub(D, C);
  ge_ext r;
  r.X = fe_mul(E, F); r.Y = fe_mul(G, H); r.Z = fe_mul(F, G); r.T = fe_mul(E, H);
  return r;
}

// dbl-2008-hwcd with a = -1
TXV_HD ge_ext ge_dbl(const ge_ext& p) {
  fe A = fe_sq(p.X), B = fe_sq(p.Y), C = fe_dbl(fe_sq(p.Z));
  fe AB = fe_add(A, B);
  fe E = fe_sub(fe_sq(fe_add(p.X, p.Y)), AB);   // 2XY
  fe G = fe_sub(B, A);
  fe H = fe_neg(AB);
  fe F = fe_sub(G, C);
  ge_ext r;
  r.X = fe_mul(E, F); r.Y = fe_mul(G, H); r.Z = fe_mul(F, G); r.T = fe_mul(E, H);
  return r;
}

// canonical 32-byte encoding as 8 little-endian words: y with bit 255 = parity(x), given 1/Z
TXV_HD void ge_encode_zinv(uint32_t out[8], const fe& X, const fe& Y, const fe& zi) {
  fe x = fe_canon(fe_mul(X, zi));
  fe y = fe_canon(fe_mul(Y, zi));
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = y.v[i];
  out[7] |= (x.v[0] & 1u) << 31;
}
TXV_HD void ge_encode(uint32_t out[8], const ge_ext& p) { ge_encode_zinv(out, p.X, p.Y, fe_invert(p.Z)); }

// ref10 ExtendedGroupElement.FromBytes (x/crypto@c2843e01d9a2):
// y = low 255 bits (y >= p accepted), reject only if (y^2-1)/(dy^2+1) has no square root,
// negate x when parity(x) != bit 255 (x = 0 with bit 255 set is accepted).
TXV_HD bool ge_decode(ge_ext& h, const uint32_t w[8]) {
  fe one = fe_one();
  h.Y = fe_from_words_255(w);
  h.Z = one;
  fe u = fe_sq(h.Y);
  fe v = fe_mul(u, fe_const_d());
  u = fe_sub(u, one);
  v = fe_add(v, one);
  fe v3 = fe_mul(fe_sq(v), v);
  fe x = fe_mul(fe_mul(fe_sq(v3), v), u);        // u v^7
  x = fe_pow22523(x);
  x = fe_mul(fe_mul(x, v3), u);                  // u v^3 (u v^7)^((p-5)/8)
  fe vxx = fe_mul(fe_sq(x), v);
  bool ok = true;
  if (!fe_iszero(fe_sub(vxx, u))) {
    if (!fe_iszero(fe_add(vxx, u))) ok = false;
    x = fe_mul(x, fe_const_sqrtm1());
  }
  if (fe_parity(x) != (w[7] >> 31)) x = fe_neg(x);
  h.X = x;
  h.T = fe_mul(x, h.Y);
  return ok;
}

// affine Niels form of an extended point given 1/Z
TXV_HD ge_niels ge_to_niels(const ge_ext& p, const fe& zinv) {
  fe x = fe_mul(p.X, zinv), y = fe_mul(p.Y, zinv);
  ge_niels n;
  n.ypx = fe_canon(fe_add(y, x));
  n.ymx = fe_canon(fe_sub(y, x));
  n.xy2d = fe_canon(fe_mul(fe_mul(x, y), fe_const_d2()));
  return n;
}

}  // namespace txv
