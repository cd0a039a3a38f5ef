// ge.h — edwards25519 group law (a = -1, d = -121665/121666) in extended coordinates.
//
// Formulas are the complete HWCD (Hisil-Wong-Carter-Dawson 2008) ones: the unified
// addition is exact for every pair of curve points, including the identity, torsion and
// small-order points that the adversarial validator set contains,
// so [s]B + [k](-A) comes out as the same group element x/crypto computes and its
// canonical encoding is bit-identical (Appendix A.1 step 6).
//
// Precomputed table entries are "affine Niels" triples (y+x, y-x, 2d*x*y), canonical,
// 96 bytes each; a mixed add costs 7 field multiplies.
#pragma once
#include "fe.h"

namespace txv {

struct ge_ext { fe X, Y, Z, T; };
struct ge_niels { fe ypx, ymx, xy2d; };

TXV_HD ge_ext ge_identity() {
  ge_ext r; r.X = fe_zero(); r.Y = fe_one(); r.Z = fe_one(); r.T = fe_zero(); return r;
}

// P + s*Q where Q is an affine Niels point and s = -1 when neg (swap y+x/y-x, negate 2dxy)
TXV_HD ge_ext ge_madd(const ge_ext& p, const ge_niels& q, bool neg) {
  fe qp = fe_select(neg, q.ymx, q.ypx);
  fe qm = fe_select(neg, q.ypx, q.ymx);
  fe A = fe_mul(fe_sub(p.Y, p.X), qm);
  TXV_SCHED_FENCE();
  fe B = fe_mul(fe_add(p.Y, p.X), qp);
  TXV_SCHED_FENCE();
  fe E = fe_sub(B, A), H = fe_add(B, A);
  fe C = fe_mul(p.T, q.xy2d);
  TXV_SCHED_FENCE();
  fe D = fe_dbl(p.Z);
  fe Gp = fe_add(D, C), Fm = fe_sub(D, C);
  fe G = fe_select(neg, Fm, Gp), F = fe_select(neg, Gp, Fm);
  ge_ext r;
  r.X = fe_mul(E, F);
  TXV_SCHED_FENCE();
  r.Y = fe_mul(G, H);
  TXV_SCHED_FENCE();
  r.Z = fe_mul(F, G);
  TXV_SCHED_FENCE();
  r.T = fe_mul(E, H);
  TXV_SCHED_FENCE();
  return r;
}

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
