/*
 * ed25519.c — CPU restatement of golang.org/x/crypto/ed25519.Verify as pinned by
 * go-txflow (x/crypto v0.0.0-20190308221718-c2843e01d9a2, go.sum:153; external,
 * not present in /root/reference).  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Call chain in the reference: types/tx_vote.go:115 -> tendermint
 * PubKeyEd25519.VerifyBytes (len(sig)!=64 -> false) -> ed25519.Verify.
 * The acceptance rules restated here are SURVEY.md Appendix A.1:
 *   1. sig[63] & 0xE0 != 0                       -> reject
 *   2. A = ref10 FromBytes(pub): y = low 255 bits (y >= p accepted, used mod p),
 *      x from sqrt((y^2-1)/(dy^2+1)) via the (p-5)/8 power and sqrt(-1) fix-up,
 *      reject only if no root; if parity(x) != bit255 negate x (x=0 with bit255=1 accepted)
 *   3. k = SHA-512(R || pub || M) mod L           (ScReduce)
 *   4. s = sig[32:64]; reject unless s < L        (ScMinimal)
 *   5. R' = [k](-A) + [s]B                        (GeDoubleScalarMultVartime; exact group law)
 *   6. accept iff canonical encode(R') == sig[0:32] byte-for-byte (R never decoded)
 * Field arithmetic: radix 2^51, 5 x 64-bit limbs with 128-bit products.  The double
 * scalar multiplication follows the reference algorithm's shape (width-5 signed digits,
 * 8 odd multiples of A and B, shared doublings) so the CPU baseline times the same work.
 */
#include "oracle.h"
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[5]; } fe;
#define M51 ((1ULL << 51) - 1)

static const fe FE_D = {{0x34dca135978a3ULL, 0x1a8283b156ebdULL, 0x5e7a26001c029ULL, 0x739c663a03cbbULL, 0x52036cee2b6ffULL}};
static const fe FE_D2 = {{0x69b9426b2f159ULL, 0x35050762add7aULL, 0x3cf44c0038052ULL, 0x6738cc7407977ULL, 0x2406d9dc56dffULL}};
static const fe FE_SQRTM1 = {{0x61b274a0ea0b0ULL, 0xd5a5fc8f189dULL, 0x7ef5e9cbd0c60ULL, 0x78595a6804c9eULL, 0x2b8324804fc1dULL}};
static const fe FE_BX = {{0x62d608f25d51aULL, 0x412a4b4f6592aULL, 0x75b7171a4b31dULL, 0x1ff60527118feULL, 0x216936d3cd6e5ULL}};
static const fe FE_BY = {{0x6666666666658ULL, 0x4ccccccccccccULL, 0x1999999999999ULL, 0x3333333333333ULL, 0x6666666666666ULL}};

static inline void fe_0(fe* h) { memset(h, 0, sizeof *h); }
static inline void fe_1(fe* h) { memset(h, 0, sizeof *h); h->v[0] = 1; }

static inline void fe_carry(fe* h) {
  uint64_t c;
  c = h->v[0] >> 51; h->v[0] &= M51; h->v[1] += c;
  c = h->v[1] >> 51; h->v[1] &= M51; h->v[2] += c;
  c = h->v[2] >> 51; h->v[2] &= M51; h->v[3] += c;
  c = h->v[3] >> 51; h->v[3] &= M51; h->v[4] += c;
  c = h->v[4] >> 51; h->v[4] &= M51; h->v[0] += 19 * c;
  c = h->v[0] >> 51; h->v[0] &= M51; h->v[1] += c;
}

static inline void fe_add(fe* h, const fe* f, const fe* g) {
  for (int i = 0; i < 5; ++i) h->v[i] = f->v[i] + g->v[i];
  fe_carry(h);
}
/* f - g computed as f + 4p - g; inputs are carried (limbs < 2^52) */
static inline void fe_sub(fe* h, const fe* f, const fe* g) {
  h->v[0] = f->v[0] + 0x1FFFFFFFFFFFB4ULL - g->v[0];
  h->v[1] = f->v[1] + 0x1FFFFFFFFFFFFCULL - g->v[1];
  h->v[2] = f->v[2] + 0x1FFFFFFFFFFFFCULL - g->v[2];
  h->v[3] = f->v[3] + 0x1FFFFFFFFFFFFCULL - g->v[3];
  h->v[4] = f->v[4] + 0x1FFFFFFFFFFFFCULL - g->v[4];
  fe_carry(h);
}
static inline void fe_neg(fe* h, const fe* f) { fe z; fe_0(&z); fe_sub(h, &z, f); }

static void fe_mul(fe* h, const fe* f, const fe* g) {
  const uint64_t *a = f->v, *b = g->v;
  uint64_t b1 = 19 * b[1], b2 = 19 * b[2], b3 = 19 * b[3], b4 = 19 * b[4];
  u128 r0 = (u128)a[0] * b[0] + (u128)a[1] * b4 + (u128)a[2] * b3 + (u128)a[3] * b2 + (u128)a[4] * b1;
  u128 r1 = (u128)a[0] * b[1] + (u128)a[1] * b[0] + (u128)a[2] * b4 + (u128)a[3] * b3 + (u128)a[4] * b2;
  u128 r2 = (u128)a[0] * b[2] + (u128)a[1] * b[1] + (u128)a[2] * b[0] + (u128)a[3] * b4 + (u128)a[4] * b3;
  u128 r3 = (u128)a[0] * b[3] + (u128)a[1] * b[2] + (u128)a[2] * b[1] + (u128)a[3] * b[0] + (u128)a[4] * b4;
  u128 r4 = (u128)a[0] * b[4] + (u128)a[1] * b[3] + (u128)a[2] * b[2] + (u128)a[3] * b[1] + (u128)a[4] * b[0];
  uint64_t c;
  r1 += (uint64_t)(r0 >> 51); uint64_t h0 = (uint64_t)r0 & M51;
  r2 += (uint64_t)(r1 >> 51); uint64_t h1 = (uint64_t)r1 & M51;
  r3 += (uint64_t)(r2 >> 51); uint64_t h2 = (uint64_t)r2 & M51;
  r4 += (uint64_t)(r3 >> 51); uint64_t h3 = (uint64_t)r3 & M51;
  c = (uint64_t)(r4 >> 51); uint64_t h4 = (uint64_t)r4 & M51;
  h0 += 19 * c; c = h0 >> 51; h0 &= M51; h1 += c;
  h->v[0] = h0; h->v[1] = h1; h->v[2] = h2; h->v[3] = h3; h->v[4] = h4;
}
static inline void fe_sq(fe* h, const fe* f) { fe_mul(h, f, f); }

static void fe_frombytes(fe* h, const uint8_t s[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; ++i) {
    uint64_t v = 0;
    for (int j = 7; j >= 0; --j) v = (v << 8) | s[8 * i + j];
    w[i] = v;
  }
  h->v[0] = w[0] & M51;
  h->v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
  h->v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
  h->v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
  h->v[4] = (w[3] >> 12) & M51;  /* bit 255 dropped: ref10 FeFromBytes ignores it */
}

/* canonical (fully reduced) little-endian encoding */
static void fe_tobytes(uint8_t s[32], const fe* f) {
  fe h = *f;
  fe_carry(&h);
  fe_carry(&h);
  uint64_t q = (h.v[0] + 19) >> 51;
  q = (h.v[1] + q) >> 51;
  q = (h.v[2] + q) >> 51;
  q = (h.v[3] + q) >> 51;
  q = (h.v[4] + q) >> 51;   /* q = 1 iff h >= p */
  h.v[0] += 19 * q;
  uint64_t c;
  c = h.v[0] >> 51; h.v[0] &= M51; h.v[1] += c;
  c = h.v[1] >> 51; h.v[1] &= M51; h.v[2] += c;
  c = h.v[2] >> 51; h.v[2] &= M51; h.v[3] += c;
  c = h.v[3] >> 51; h.v[3] &= M51; h.v[4] += c;
  h.v[4] &= M51;
  uint64_t w[4];
  w[0] = h.v[0] | (h.v[1] << 51);
  w[1] = (h.v[1] >> 13) | (h.v[2] << 38);
  w[2] = (h.v[2] >> 26) | (h.v[3] << 25);
  w[3] = (h.v[3] >> 39) | (h.v[4] << 12);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

static int fe_isnegative(const fe* f) { uint8_t s[32]; fe_tobytes(s, f); return s[0] & 1; }
static int fe_isnonzero(const fe* f) {
  uint8_t s[32]; fe_tobytes(s, f);
  uint8_t r = 0; for (int i = 0; i < 32; ++i) r |= s[i];
  return r != 0;
}

static void fe_sqn(fe* h, const fe* f, int n) { *h = *f; for (int i = 0; i < n; ++i) fe_sq(h, h); }

/* z^(2^250 - 1) and z^11 — shared prefix of the inversion and (p-5)/8 chains */
static void fe_pow2501(fe* out250, fe* z11, const fe* z) {
  fe z2, z8, z9, t0, t1, z_5_0, z_10_0, z_20_0, z_50_0, z_100_0;
  fe_sq(&z2, z);
  fe_sqn(&z8, &z2, 2);
  fe_mul(&z9, &z8, z);
  fe_mul(z11, &z9, &z2);
  fe_sq(&t0, z11);
  fe_mul(&z_5_0, &t0, &z9);                 /* 2^5 - 1 */
  fe_sqn(&t0, &z_5_0, 5);  fe_mul(&z_10_0, &t0, &z_5_0);     /* 2^10 - 1 */
  fe_sqn(&t0, &z_10_0, 10); fe_mul(&z_20_0, &t0, &z_10_0);   /* 2^20 - 1 */
  fe_sqn(&t0, &z_20_0, 20); fe_mul(&t1, &t0, &z_20_0);       /* 2^40 - 1 */
  fe_sqn(&t0, &t1, 10);    fe_mul(&z_50_0, &t0, &z_10_0);    /* 2^50 - 1 */
  fe_sqn(&t0, &z_50_0, 50); fe_mul(&z_100_0, &t0, &z_50_0);  /* 2^100 - 1 */
  fe_sqn(&t0, &z_100_0, 100); fe_mul(&t1, &t0, &z_100_0);    /* 2^200 - 1 */
  fe_sqn(&t0, &t1, 50);    fe_mul(out250, &t0, &z_50_0);     /* 2^250 - 1 */
}
static void fe_invert(fe* h, const fe* z) {
  fe t250, z11, t;
  fe_pow2501(&t250, &z11, z);
  fe_sqn(&t, &t250, 5);
  fe_mul(h, &t, &z11);                      /* 2^255 - 21 = p - 2 */
}
static void fe_pow22523(fe* h, const fe* z) {
  fe t250, z11, t;
  fe_pow2501(&t250, &z11, z);
  fe_sqn(&t, &t250, 2);
  fe_mul(h, &t, z);                         /* 2^252 - 3 = (p-5)/8 */
}

/* ---------------- group: twisted Edwards a = -1, extended coordinates ---------------- */
typedef struct { fe X, Y, Z; } ge_p2;
typedef struct { fe X, Y, Z, T; } ge_p3;
typedef struct { fe X, Y, Z, T; } ge_p1p1;       /* (E, H, G, F): X3=E*F, Y3=G*H, Z3=F*G, T3=E*H */
typedef struct { fe YpX, YmX, Z, T2d; } ge_cached;

static void p1p1_to_p2(ge_p2* r, const ge_p1p1* p) {
  fe_mul(&r->X, &p->X, &p->T); fe_mul(&r->Y, &p->Y, &p->Z); fe_mul(&r->Z, &p->Z, &p->T);
}
static void p1p1_to_p3(ge_p3* r, const ge_p1p1* p) {
  fe_mul(&r->X, &p->X, &p->T); fe_mul(&r->Y, &p->Y, &p->Z); fe_mul(&r->Z, &p->Z, &p->T);
  fe_mul(&r->T, &p->X, &p->Y);
}
static void p3_to_cached(ge_cached* r, const ge_p3* p) {
  fe_add(&r->YpX, &p->Y, &p->X); fe_sub(&r->YmX, &p->Y, &p->X);
  r->Z = p->Z; fe_mul(&r->T2d, &p->T, &FE_D2);
}
static void p3_to_p2(ge_p2* r, const ge_p3* p) { r->X = p->X; r->Y = p->Y; r->Z = p->Z; }
static void p2_0(ge_p2* r) { fe_0(&r->X); fe_1(&r->Y); fe_1(&r->Z); }

/* dbl-2008-hwcd, a = -1 */
static void ge_dbl(ge_p1p1* r, const ge_p2* p) {
  fe A, B, C, S, t;
  fe_sq(&A, &p->X); fe_sq(&B, &p->Y); fe_sq(&C, &p->Z); fe_add(&C, &C, &C);
  fe_add(&t, &p->X, &p->Y); fe_sq(&S, &t);
  fe AB; fe_add(&AB, &A, &B);
  fe_sub(&r->X, &S, &AB);          /* E = 2XY */
  fe_sub(&r->Z, &B, &A);           /* G = B - A */
  fe_neg(&r->Y, &AB);              /* H = -A - B */
  fe_sub(&r->T, &r->Z, &C);        /* F = G - C */
}
/* add-2008-hwcd-3 with a cached operand; sign = +1 add, -1 subtract */
static void ge_addsub(ge_p1p1* r, const ge_p3* p, const ge_cached* q, int neg) {
  fe A, B, C, D, t;
  fe_sub(&t, &p->Y, &p->X); fe_mul(&A, &t, neg ? &q->YpX : &q->YmX);
  fe_add(&t, &p->Y, &p->X); fe_mul(&B, &t, neg ? &q->YmX : &q->YpX);
  fe_mul(&C, &p->T, &q->T2d);
  fe_mul(&D, &p->Z, &q->Z); fe_add(&D, &D, &D);
  fe_sub(&r->X, &B, &A);                 /* E */
  fe_add(&r->Y, &B, &A);                 /* H */
  if (!neg) { fe_add(&r->Z, &D, &C); fe_sub(&r->T, &D, &C); }   /* G, F */
  else      { fe_sub(&r->Z, &D, &C); fe_add(&r->T, &D, &C); }
}

static void ge_p2_tobytes(uint8_t s[32], const ge_p2* p) {
  fe zi, x, y;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi); fe_mul(&y, &p->Y, &zi);
  fe_tobytes(s, &y);
  s[31] ^= (uint8_t)(fe_isnegative(&x) << 7);
}

/* ref10 ExtendedGroupElement.FromBytes semantics (Appendix A.1 step 3) */
static int ge_frombytes(ge_p3* h, const uint8_t s[32]) {
  fe u, v, v3, vxx, check, one;
  fe_1(&one);
  fe_frombytes(&h->Y, s);
  fe_1(&h->Z);
  fe_sq(&u, &h->Y);
  fe_mul(&v, &u, &FE_D);
  fe_sub(&u, &u, &one);             /* u = y^2 - 1 */
  fe_add(&v, &v, &one);             /* v = d y^2 + 1 */
  fe_sq(&v3, &v); fe_mul(&v3, &v3, &v);          /* v^3 */
  fe_sq(&h->X, &v3); fe_mul(&h->X, &h->X, &v); fe_mul(&h->X, &h->X, &u);  /* u v^7 */
  fe_pow22523(&h->X, &h->X);
  fe_mul(&h->X, &h->X, &v3); fe_mul(&h->X, &h->X, &u);                  /* u v^3 (u v^7)^((p-5)/8) */
  fe_sq(&vxx, &h->X); fe_mul(&vxx, &vxx, &v);
  fe_sub(&check, &vxx, &u);
  if (fe_isnonzero(&check)) {
    fe_add(&check, &vxx, &u);
    if (fe_isnonzero(&check)) return 0;
    fe_mul(&h->X, &h->X, &FE_SQRTM1);
  }
  if (fe_isnegative(&h->X) != (s[31] >> 7)) fe_neg(&h->X, &h->X);
  fe_mul(&h->T, &h->X, &h->Y);
  return 1;
}

/* width-5 signed-digit recoding: r[i] in {0, +-1, +-3, ..., +-15}, sum r[i] 2^i = a (a < 2^256) */
static void recode_w5(int8_t r[257], const uint8_t a[32]) {
  uint32_t k[9];
  for (int i = 0; i < 8; ++i) k[i] = (uint32_t)a[4 * i] | ((uint32_t)a[4 * i + 1] << 8) | ((uint32_t)a[4 * i + 2] << 16) | ((uint32_t)a[4 * i + 3] << 24);
  k[8] = 0;
  memset(r, 0, 257);
  for (int i = 0; i < 257; ++i) {
    /* k is the remaining value shifted right by i */
    if (k[0] & 1) {
      int d = (int)(k[0] & 31);
      if (d > 16) d -= 32;
      r[i] = (int8_t)d;
      /* k -= d */
      if (d > 0) {
        uint64_t bor = (uint64_t)d;
        for (int j = 0; j < 9 && bor; ++j) { uint64_t t = (uint64_t)k[j] - bor; k[j] = (uint32_t)t; bor = (t >> 63) & 1; }
      } else {
        uint64_t car = (uint64_t)(-d);
        for (int j = 0; j < 9 && car; ++j) { uint64_t t = (uint64_t)k[j] + car; k[j] = (uint32_t)t; car = t >> 32; }
      }
    }
    for (int j = 0; j < 8; ++j) k[j] = (k[j] >> 1) | (k[j + 1] << 31);
    k[8] >>= 1;
  }
}

static ge_cached BI[8];
static int BI_ready = 0;

static void ge_base_p3(ge_p3* B) {
  B->X = FE_BX; B->Y = FE_BY; fe_1(&B->Z); fe_mul(&B->T, &FE_BX, &FE_BY);
}

static void odd_multiples(ge_cached out[8], const ge_p3* P) {
  ge_p3 cur = *P, twoP; ge_p1p1 t; ge_p2 p2;
  p3_to_p2(&p2, P); ge_dbl(&t, &p2); p1p1_to_p3(&twoP, &t);
  ge_cached twoPc; p3_to_cached(&twoPc, &twoP);
  p3_to_cached(&out[0], &cur);
  for (int i = 1; i < 8; ++i) {
    ge_addsub(&t, &cur, &twoPc, 0); p1p1_to_p3(&cur, &t);
    p3_to_cached(&out[i], &cur);
  }
}

static void init_base(void) {
  if (BI_ready) return;
  ge_p3 B; ge_base_p3(&B);
  odd_multiples(BI, &B);
  __atomic_store_n(&BI_ready, 1, __ATOMIC_RELEASE);
}

/* r = [a]A + [b]B (variable time) */
static void ge_double_scalarmult(ge_p2* r, const uint8_t a[32], const ge_p3* A, const uint8_t b[32]) {
  int8_t as[257], bs[257];
  ge_cached Ai[8];
  ge_p1p1 t; ge_p3 u;
  init_base();
  recode_w5(as, a); recode_w5(bs, b);
  odd_multiples(Ai, A);
  p2_0(r);
  int i = 256;
  while (i >= 0 && !as[i] && !bs[i]) --i;
  for (; i >= 0; --i) {
    ge_dbl(&t, r);
    if (as[i] > 0) { p1p1_to_p3(&u, &t); ge_addsub(&t, &u, &Ai[as[i] / 2], 0); }
    else if (as[i] < 0) { p1p1_to_p3(&u, &t); ge_addsub(&t, &u, &Ai[(-as[i]) / 2], 1); }
    if (bs[i] > 0) { p1p1_to_p3(&u, &t); ge_addsub(&t, &u, &BI[bs[i] / 2], 0); }
    else if (bs[i] < 0) { p1p1_to_p3(&u, &t); ge_addsub(&t, &u, &BI[(-bs[i]) / 2], 1); }
    p1p1_to_p2(r, &t);
  }
}

/* ---------------- scalars mod L = 2^252 + 27742317777372353535851937790883648493 ---------------- */
static const uint64_t L64[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};
static const uint64_t MU64[5] = {0xed9ce5a30a2c131bULL, 0x2106215d086329a7ULL, 0xffffffffffffffebULL,
                                 0xffffffffffffffffULL, 0xfULL};   /* floor(2^512 / L) */

/* Barrett reduction of a 512-bit little-endian value x[8] (HAC 14.42, b = 2^64, k = 4) */
static void barrett(uint64_t out[4], const uint64_t x[8]) {
  uint64_t q1[5], q2[10] = {0}, r2[5] = {0}, r[5];
  for (int i = 0; i < 5; ++i) q1[i] = x[3 + i];
  for (int i = 0; i < 5; ++i) {
    u128 c = 0;
    for (int j = 0; j < 5; ++j) {
      c += (u128)q1[i] * MU64[j] + q2[i + j];
      q2[i + j] = (uint64_t)c; c >>= 64;
    }
    q2[i + 5] = (uint64_t)c;
  }
  const uint64_t* q3 = q2 + 5;   /* q2 >> 320, 5 limbs */
  for (int i = 0; i < 5; ++i) {   /* (q3 * L) mod 2^320 */
    u128 c = 0;
    for (int j = 0; i + j < 5; ++j) {
      c += (u128)q3[i] * (j < 4 ? L64[j] : 0) + r2[i + j];
      r2[i + j] = (uint64_t)c; c >>= 64;
    }
  }
  u128 bor = 0;
  for (int i = 0; i < 5; ++i) {   /* r = x mod 2^320 - r2 (mod 2^320) */
    u128 t = (u128)x[i] - r2[i] - bor;
    r[i] = (uint64_t)t; bor = (t >> 64) & 1;
  }
  for (int it = 0; it < 3; ++it) {   /* while r >= L: r -= L */
    int ge = 0;
    if (r[4]) ge = 1;
    else {
      ge = 1;
      for (int i = 3; i >= 0; --i) { if (r[i] != L64[i]) { ge = r[i] > L64[i]; break; } }
    }
    if (!ge) break;
    bor = 0;
    for (int i = 0; i < 5; ++i) {
      u128 t = (u128)r[i] - (i < 4 ? L64[i] : 0) - bor;
      r[i] = (uint64_t)t; bor = (t >> 64) & 1;
    }
  }
  for (int i = 0; i < 4; ++i) out[i] = r[i];
}

static void load64_le(uint64_t* w, const uint8_t* s, int n) {
  for (int i = 0; i < n; ++i) {
    uint64_t v = 0;
    for (int j = 7; j >= 0; --j) v = (v << 8) | s[8 * i + j];
    w[i] = v;
  }
}
static void store64_le(uint8_t* s, const uint64_t* w, int n) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 8; ++j) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

void orc_sc_reduce64(const uint8_t in[64], uint8_t out[32]) {
  uint64_t x[8], r[4];
  load64_le(x, in, 8);
  barrett(r, x);
  store64_le(out, r, 4);
}

int orc_sc_minimal(const uint8_t s[32]) {
  uint64_t w[4]; load64_le(w, s, 4);
  for (int i = 3; i >= 0; --i) { if (w[i] != L64[i]) return w[i] < L64[i]; }
  return 0;   /* s == L */
}

/* out = (a*b + c) mod L; a, b, c are 256-bit little-endian */
static void sc_muladd(uint8_t out[32], const uint8_t a[32], const uint8_t b[32], const uint8_t c[32]) {
  uint64_t A[4], B[4], C[4], X[8] = {0}, r[4];
  load64_le(A, a, 4); load64_le(B, b, 4); load64_le(C, c, 4);
  for (int i = 0; i < 4; ++i) {
    u128 car = 0;
    for (int j = 0; j < 4; ++j) {
      car += (u128)A[i] * B[j] + X[i + j];
      X[i + j] = (uint64_t)car; car >>= 64;
    }
    X[i + 4] = (uint64_t)car;
  }
  u128 car = 0;
  for (int i = 0; i < 8; ++i) { car += (u128)X[i] + (i < 4 ? C[i] : 0); X[i] = (uint64_t)car; car >>= 64; }
  barrett(r, X);
  store64_le(out, r, 4);
}

/* ---------------- public API ---------------- */
int orc_ed25519_decode_ok(const uint8_t pub[32]) { ge_p3 A; return ge_frombytes(&A, pub); }

int orc_ed25519_verify(const uint8_t pub[32], const uint8_t* msg, size_t msg_len,
                       const uint8_t* sig, size_t sig_len) {
  if (sig_len != 64) return 0;                 /* tendermint PubKeyEd25519.VerifyBytes */
  if (sig[63] & 0xE0) return 0;
  ge_p3 A;
  if (!ge_frombytes(&A, pub)) return 0;
  fe_neg(&A.X, &A.X); fe_neg(&A.T, &A.T);      /* -A */
  uint8_t buf_small[512];
  uint8_t* buf = buf_small;
  size_t tot = 64 + msg_len;
  uint8_t* heap = 0;
  if (tot > sizeof buf_small) { heap = (uint8_t*)__builtin_malloc(tot); buf = heap; }
  memcpy(buf, sig, 32); memcpy(buf + 32, pub, 32); if (msg_len) memcpy(buf + 64, msg, msg_len);
  uint8_t h[64], k[32];
  orc_sha512(buf, tot, h);
  if (heap) __builtin_free(heap);
  orc_sc_reduce64(h, k);
  if (!orc_sc_minimal(sig + 32)) return 0;
  ge_p2 R; uint8_t chk[32];
  ge_double_scalarmult(&R, k, &A, sig + 32);
  ge_p2_tobytes(chk, &R);
  return memcmp(chk, sig, 32) == 0;
}

static void scalarmult_base(uint8_t out[32], const uint8_t k[32]) {
  ge_p3 B; ge_base_p3(&B);
  uint8_t zero[32] = {0};
  ge_p2 R;
  ge_double_scalarmult(&R, zero, &B, k);
  ge_p2_tobytes(out, &R);
}
void orc_scalarmult_base(const uint8_t k[32], uint8_t out[32]) { scalarmult_base(out, k); }

int orc_scalarmult(const uint8_t k[32], const uint8_t p_enc[32], uint8_t out[32]) {
  ge_p3 P; if (!ge_frombytes(&P, p_enc)) return 0;
  uint8_t zero[32] = {0};
  ge_p2 R; ge_double_scalarmult(&R, k, &P, zero);
  ge_p2_tobytes(out, &R);
  return 1;
}
int orc_point_canonical(const uint8_t p_enc[32], uint8_t out[32]) {
  ge_p3 P; if (!ge_frombytes(&P, p_enc)) return 0;
  ge_p2 R; p3_to_p2(&R, &P); ge_p2_tobytes(out, &R);
  return 1;
}

static void expand_seed(const uint8_t seed[32], uint8_t a[32], uint8_t prefix[32]) {
  uint8_t h[64];
  orc_sha512(seed, 32, h);
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  memcpy(a, h, 32); memcpy(prefix, h + 32, 32);
}

void orc_ed25519_pubkey(const uint8_t seed[32], uint8_t pub[32]) {
  uint8_t a[32], prefix[32];
  expand_seed(seed, a, prefix);
  scalarmult_base(pub, a);
}

void orc_ed25519_sign(const uint8_t seed[32], const uint8_t* msg, size_t msg_len, uint8_t sig[64]) {
  uint8_t a[32], prefix[32], pub[32], h[64], r[32], k[32];
  expand_seed(seed, a, prefix);
  scalarmult_base(pub, a);
  size_t tot = 64 + msg_len;
  uint8_t* buf = (uint8_t*)__builtin_malloc(tot);
  memcpy(buf + 32, prefix, 32); if (msg_len) memcpy(buf + 64, msg, msg_len);
  orc_sha512(buf + 32, 32 + msg_len, h);
  orc_sc_reduce64(h, r);
  scalarmult_base(sig, r);                       /* R */
  memcpy(buf, sig, 32); memcpy(buf + 32, pub, 32);
  orc_sha512(buf, tot, h);
  orc_sc_reduce64(h, k);
  sc_muladd(sig + 32, k, a, r);                  /* S = k*a + r mod L */
  __builtin_free(buf);
}
