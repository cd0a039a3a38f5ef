// emu.hip — TEST-ONLY host emulation of the device math in go-txflow_amd/csrc.
//
// Compiles the very same __host__ __device__ headers (fe.h, sc.h, sha2.h, ge.h,
// ed25519_dev.h) for the host so logic errors in the kernel source can be localised on a
// machine without a GPU.  It is not linked into libtxvote.so and the product never calls it.
#include "../../go-txflow_amd/csrc/ed25519_dev.h"
#include "../../go-txflow_amd/csrc/fe_inv_var.h"
#include "../../go-txflow_amd/csrc/wire_dev.h"
#include <cstring>
#include <vector>

using namespace txv;

static void build_table(std::vector<uint32_t>& tab, const uint32_t w[8], bool* ok_out) {
  tab.assign(kTableWords, 0);
  ge_ext A;
  bool ok = ge_decode(A, w);
  if (ok_out) *ok_out = ok;
  for (int pos = 0; pos < 64; ++pos) {
    ge_ext P = A;
    for (int i = 0; i < 4 * pos; ++i) P = ge_dbl(P);
    ge_ext M[8];
    M[0] = P;
    M[1] = ge_dbl(P);
    for (int j = 2; j < 8; ++j) M[j] = ge_add(M[j - 1], P);
    uint32_t* out = tab.data() + pos * kTabEntries * kEntryWords;
    for (int j = 0; j < 8; ++j) {
      ge_niels n = ge_to_niels(M[j], fe_invert(M[j].Z));
      entry_words(out + (j + 1) * kEntryWords, n.ypx, n.ymx, n.xy2d);
    }
    entry_identity(out);
  }
}

template <int W>
static int digits_w(const uint32_t* s_in, int mode, int32_t* out) {
  constexpr int n = Tab<W>::kPositions;
  if (mode == 0) {          // the walks' streaming digits (table_digit)
    uint32_t s[8], c = 0;
    for (int i = 0; i < 8; ++i) s[i] = s_in[i];
    for (int pos = 0; pos < n; ++pos) out[pos] = table_digit<W>(s, c, pos);
  } else {                  // the split kernel's all-at-once digits
    int d[n];
    signed_digits<W, n>(s_in, d);
    for (int pos = 0; pos < n; ++pos) out[pos] = d[pos];
  }
  return n;
}

extern "C" {

// digits of scalar s for table window w (20, 21, 24, 26); returns the number of positions
int emu_digits(int w, const uint32_t* s, int mode, int32_t* out) {
  switch (w) {
    case 20: return digits_w<20>(s, mode, out);
    case 21: return digits_w<21>(s, mode, out);
    case 24: return digits_w<24>(s, mode, out);
    case 26: return digits_w<26>(s, mode, out);
    default: return -1;
  }
}

int emu_fe(const uint32_t* a, const uint32_t* b, uint32_t* out, int op) {
  fe x, y, r;
  for (int j = 0; j < 8; ++j) { x.v[j] = a[j]; y.v[j] = b[j]; }
  switch (op) {
    case 0: r = fe_mul(x, y); break;
    case 1: r = fe_sq(x); break;
    case 2: r = fe_add(x, y); break;
    case 3: r = fe_sub(x, y); break;
    case 4: r = fe_canon(x); break;
    case 5: r = fe_invert(x); break;
    case 7: r = fe_invert_var(x); break;
    default: {
      uint32_t t[16];
      for (int j = 0; j < 8; ++j) { t[j] = x.v[j]; t[8 + j] = y.v[j]; }
      sc s = sc_reduce512(t);
      for (int j = 0; j < 8; ++j) r.v[j] = s.v[j];
    }
  }
  for (int j = 0; j < 8; ++j) out[j] = r.v[j];
  return 0;
}

// divstep inverse with its batch count (-1: g had not reached 0 within the 32-batch cap)
int emu_inv_var(const uint32_t* a, uint32_t* out) {
  fe x;
  for (int j = 0; j < 8; ++j) x.v[j] = a[j];
  int batches;
  const fe r = fe_invert_var_n(x, batches);
  for (int j = 0; j < 8; ++j) out[j] = r.v[j];
  return batches;
}
// batch counts of n inputs (32-byte little-endian each), for the search in the test
void emu_inv_var_counts(const uint32_t* a, int n, int32_t* counts) {
  for (int i = 0; i < n; ++i) {
    fe x;
    for (int j = 0; j < 8; ++j) x.v[j] = a[8 * i + j];
    fe_invert_var_n(x, counts[i]);
  }
}

// fe10 primitives on raw limbs (op 0 mul, 1 add, 2 sub, 3 cneg, 4 carry, 5 strict, 6 from radix
// 2^32 (8 words in), 7 to radix 2^32 (8 words out), 8 madd on (X,Y,Z,T) + entry words)
int emu_fe10(const uint32_t* a, const uint32_t* b, uint32_t* out, int op) {
  fe10 x, y, r;
  for (int j = 0; j < 10; ++j) { x.v[j] = a[j]; y.v[j] = b[j]; }
  switch (op) {
    case 0: r = fe10_mul(x, y); break;
    case 1: r = fe10_add(x, y); break;
    case 2: r = fe10_sub(x, y); break;
    case 3: r = fe10_cneg(x, true); break;
    case 4: r = fe10_carry(x); break;
    case 5: r = fe10_strict(x); break;
    case 6: {
      fe f;
      for (int j = 0; j < 8; ++j) f.v[j] = a[j];
      r = fe10_from_fe(f);
      break;
    }
    case 7: {
      fe f = fe_from_fe10(x);
      for (int j = 0; j < 8; ++j) out[j] = f.v[j];
      return 0;
    }
    case 9: {   // fe10_mul2(x, y, y, x): both products, out[0..9] and out[10..19]
      fe10 r2;
      fe10_mul2(x, y, y, x, r, r2);
      for (int j = 0; j < 10; ++j) out[10 + j] = r2.v[j];
      break;
    }
    default: return -1;
  }
  for (int j = 0; j < 10; ++j) out[j] = r.v[j];
  return 0;
}
// one table addition through ge10_madd: p = X,Y,Z,T (40 limbs), e = 32 entry words, out 40 limbs
int emu_ge10_madd(const uint32_t* p, const uint32_t* e, int neg, uint32_t* out) {
  ge10_ext P;
  for (int j = 0; j < 10; ++j) { P.X.v[j] = p[j]; P.Y.v[j] = p[10 + j]; P.Z.v[j] = p[20 + j]; P.T.v[j] = p[30 + j]; }
  fe10 qp, qm, qd;
  load_entry_w<4>(e, 0, 0, neg != 0, qp, qm, qd);
  P = ge10_madd(P, qp, qm, qd, neg != 0);
  for (int j = 0; j < 10; ++j) { out[j] = P.X.v[j]; out[10 + j] = P.Y.v[j]; out[20 + j] = P.Z.v[j]; out[30 + j] = P.T.v[j]; }
  return 0;
}
// the same addition through the walk's form (entry read piecewise, product pairs), kT = 0 for the
// last addition of a walk (T not computed)
int emu_ge10_madd_rd(const uint32_t* p, const uint32_t* e, int neg, uint32_t* out, int kT) {
  ge10_ext P;
  for (int j = 0; j < 10; ++j) { P.X.v[j] = p[j]; P.Y.v[j] = p[10 + j]; P.Z.v[j] = p[20 + j]; P.T.v[j] = p[30 + j]; }
  fe10 q[3];
  load_entry_w<4>(e, 0, 0, neg != 0, q[0], q[1], q[2]);
  auto rd = [&](int role) { return q[role]; };
  auto mid = [] {};
  P = kT ? ge10_madd_rd<true>(P, rd, neg != 0, mid) : ge10_madd_rd<false>(P, rd, neg != 0, mid);
  for (int j = 0; j < 10; ++j) { out[j] = P.X.v[j]; out[10 + j] = P.Y.v[j]; out[20 + j] = P.Z.v[j]; out[30 + j] = P.T.v[j]; }
  return 0;
}
// entry words of the affine point (x, y) (radix 2^32 in, canonical)
int emu_entry(const uint32_t* x, const uint32_t* y, uint32_t* e) {
  fe X, Y;
  for (int j = 0; j < 8; ++j) { X.v[j] = x[j]; Y.v[j] = y[j]; }
  ge_ext P; P.X = X; P.Y = Y; P.Z = fe_one(); P.T = fe_mul(X, Y);
  ge_niels n = ge_to_niels(P, fe_one());
  entry_words(e, n.ypx, n.ymx, n.xy2d);
  return 0;
}

// kernel-K1 logic for one vote; msg given as raw bytes
int emu_verify(const uint8_t pub[32], const uint8_t* msg, uint32_t len, const uint8_t* sig, uint32_t sig_len) {
  static std::vector<uint32_t> btab;
  if (btab.empty()) {
    uint32_t bw[8];
    base_point_words(bw);
    build_table(btab, bw, nullptr);
  }
  if (sig_len != 64) return 0;
  uint32_t s[16], pw[8];
  memcpy(s, sig, 64);
  memcpy(pw, pub, 32);
  std::vector<uint32_t> atab;
  bool dok;
  build_table(atab, pw, &dok);
  if ((s[15] & 0xE0000000u) || !dok || !sc_lt_L(s + 8)) return 0;
  uint64_t pre[8];
  for (int j = 0; j < 4; ++j) {
    pre[j] = be64_from_le32(s[2 * j], s[2 * j + 1]);
    pre[4 + j] = be64_from_le32(pw[2 * j], pw[2 * j + 1]);
  }
  const uint32_t nw = (len + 7) / 8;
  std::vector<uint64_t> words(nw + 1, 0);
  for (uint32_t i = 0; i < len; ++i) words[i / 8] |= (uint64_t)msg[i] << (56 - 8 * (i % 8));
  MsgView m{words.data(), 1, nw, len};
  uint32_t dig[16];
  sha512_prefixed(dig, pre, 8, m);
  sc k = sc_reduce512(dig);
  ge_ext R = double_scalarmult_fixed(btab.data(), atab.data(), s + 8, k.v, true);
  uint32_t enc[8];
  ge_encode(enc, R);
  return memcmp(enc, s, 32) == 0;
}


// TxVoteMessage decode through wire_dev.h (txv_k_decode_msgs' parser and row copies, global-memory
// form): the message sits at byte `shift` (0..3) of a word buffer.  Returns the TXV_WIRE_* status;
// i64: height, ts_sec; u32: ts_nanos, txhash_off, txhash_len, addr_len, sig_off, sig_len;
// rows: TxKey 8 words, address 5, signature 16.
static uint64_t fast_hits = 0;
uint64_t emu_wire_fast_hits() { return fast_hits; }
// general parser only (the oracle-independent reference for the fast path)
int emu_wire_decode_general(const uint8_t* msg, uint32_t len, uint32_t disamb, uint32_t prefix) {
  using namespace txv::wire;
  Parsed o{};
  return len ? (int)parse_msg(msg, len, disamb, prefix, o) : 3;
}
int emu_wire_decode(const uint8_t* msg, uint32_t len, uint32_t max_msg, uint32_t disamb, uint32_t prefix,
                    uint32_t shift, int64_t* i64, uint32_t* u32, uint32_t* rows) {
  using namespace txv::wire;
  std::vector<uint32_t> words((len + shift + 3) / 4 + 24, 0xA5A5A5A5u);   // kernel: 128 B padding
  uint8_t* bytes = reinterpret_cast<uint8_t*>(words.data());
  memcpy(bytes + shift, msg, len);
  Parsed o{};
  uint32_t st = len == 0 ? 3u : (len > max_msg ? 1u : 4u);
  if (st == 4u) {   // as the kernel: fast path, else the general parser (fast_hits counts the former)
    if (fast_msg((const uint32_t*)words.data(), shift, len, prefix, o)) { st = 0; ++fast_hits; }
    else { o = Parsed{}; st = parse_msg((const uint8_t*)(bytes + shift), len, disamb, prefix, o); }
  }
  if (st != 0) o = Parsed{};
  memset(rows, 0, 29 * 4);
  const uint32_t an = o.addr_len < 20 ? o.addr_len : 20u, sn = o.sig_len < 64 ? o.sig_len : 64u;
  if (o.has_key) copy_row<8>((const uint32_t*)words.data(), shift + o.key_off, 32u, rows);
  if (an) copy_row<5>((const uint32_t*)words.data(), shift + o.addr_off, an, rows + 8);
  if (sn) copy_row<16>((const uint32_t*)words.data(), shift + o.sig_off, sn, rows + 13);
  i64[0] = o.height; i64[1] = o.sec;
  u32[0] = (uint32_t)o.nanos; u32[1] = o.th_off; u32[2] = o.th_len; u32[3] = o.addr_len; u32[4] = o.sig_off;
  u32[5] = o.sig_len;
  return (int)st;
}

}  // extern "C"
