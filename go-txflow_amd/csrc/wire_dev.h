// wire_dev.h — the TxVoteMessage amino decoder run by txv_k_decode_msgs (kernels_wire.hip), as
// __host__ __device__ code so tests/cpu_emu can run the same source on the host.  Rules: go-amino
// v0.15.1 (external) as restated in oracle/wire.c's header; statuses are include/txvote.h's TXV_WIRE_*.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#define TXV_WIRE_HD __host__ __device__ __forceinline__

namespace txv {
namespace wire {

TXV_WIRE_HD int clz64(uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __clzll((long long)v);
#else
  return __builtin_clzll(v);
#endif
}

TXV_WIRE_HD int ctz64(uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ffsll((unsigned long long)v) - 1;
#else
  return __builtin_ctzll(v);
#endif
}

// (hi:lo) >> sh, 0 < sh < 32
TXV_WIRE_HD uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh);
#endif
}

constexpr uint32_t TYP_VARINT = 0, TYP_8BYTE = 1, TYP_BYTES = 2, TYP_4BYTE = 5;
constexpr int64_t kMinSec = -62135596800LL, kMaxSec = 253402300800LL;

// Go binary.Uvarint over b[p, end): bytes read, 0 = error (truncated or overflow)
template <typename B>
TXV_WIRE_HD uint32_t uvarint(B b, uint32_t p, uint32_t end, uint64_t& v) {
  uint64_t x = 0;
#pragma unroll 1
  for (uint32_t i = 0; i < 10; ++i) {
    if (p + i >= end) return 0;
    const uint32_t c = b[p + i];
    if (c < 0x80u) {
      if (i == 9 && c > 1u) return 0;
      v = x | ((uint64_t)c << (7 * i));
      return i + 1;
    }
    x |= (uint64_t)(c & 0x7fu) << (7 * i);
  }
  return 0;
}

TXV_WIRE_HD uint32_t uvarint_size(uint64_t v) {
  return v ? (uint32_t)((64 - clz64(v) + 6) / 7) : 1u;
}

template <typename B>
TXV_WIRE_HD uint32_t field_key(B b, uint32_t p, uint32_t end, uint32_t& num, uint32_t& typ) {
  uint64_t v;
  const uint32_t k = uvarint(b, p, end, v);
  if (!k || (v >> 3) > ((1u << 29) - 1u)) return 0;
  num = (uint32_t)(v >> 3);
  typ = (uint32_t)v & 7u;
  return k;
}

// DecodeByteSlice: bytes read (0 = error), body at [body, body + blen)
template <typename B>
TXV_WIRE_HD uint32_t byte_slice(B b, uint32_t p, uint32_t end, uint32_t& body, uint32_t& blen) {
  uint64_t cnt;
  const uint32_t k = uvarint(b, p, end, cnt);
  if (!k || cnt > (uint64_t)(end - p - k)) return 0;   // also rejects count >= 2^63
  body = p + k;
  blen = (uint32_t)cnt;
  return k + (uint32_t)cnt;
}

template <typename B>
TXV_WIRE_HD uint32_t skip_any(B b, uint32_t p, uint32_t end, uint32_t typ) {
  uint64_t v;
  uint32_t x, y;
  switch (typ) {
    case TYP_VARINT: return uvarint(b, p, end, v);
    case TYP_8BYTE: return end - p >= 8 ? 8u : 0u;
    case TYP_BYTES: return byte_slice(b, p, end, x, y);
    case TYP_4BYTE: return end - p >= 4 ? 4u : 0u;
    default: return 0;
  }
}

// skip strictly increasing extra fields up to end; false on error
template <typename B>
TXV_WIRE_HD bool skip_rest(B b, uint32_t p, uint32_t end, uint32_t last) {
#pragma unroll 1
  while (p < end) {
    uint32_t num, typ;
    const uint32_t k = field_key(b, p, end, num, typ);
    if (!k || num <= last) return false;
    last = num;
    p += k;
    const uint32_t a = skip_any(b, p, end, typ);
    if (!a) return false;
    p += a;
  }
  return true;
}

struct Parsed {
  int64_t height, sec;
  int32_t nanos;
  uint32_t th_off, th_len, key_off, addr_off, addr_len, sig_off, sig_len;
  bool has_key;
};

// time.Time body [p, end): consumed bytes, or UINT32_MAX on error
template <typename B>
TXV_WIRE_HD uint32_t time_body(B b, uint32_t p, uint32_t end, int64_t& sec, int32_t& nanos) {
  const uint32_t p0 = p;
  uint32_t num, typ, k;
  uint64_t v;
  if (p < end) {
    if (!(k = field_key(b, p, end, num, typ))) return UINT32_MAX;
    if (num == 1 && typ == TYP_VARINT) {
      p += k;
      if (!(k = uvarint(b, p, end, v))) return UINT32_MAX;
      p += k;
      if ((int64_t)v < kMinSec || (int64_t)v >= kMaxSec) return UINT32_MAX;
      sec = (int64_t)v;
    }
  }
  if (p < end) {
    if (!(k = field_key(b, p, end, num, typ))) return UINT32_MAX;
    if (num == 2 && typ == TYP_VARINT) {
      p += k;
      if (!(k = uvarint(b, p, end, v))) return UINT32_MAX;
      p += k;
      if (v > 999999999ull) return UINT32_MAX;
      nanos = (int32_t)v;
    }
  }
  return p - p0;
}

// TxVote body [p, end) (types/tx_vote.go:48-55); false on an amino error
template <typename B>
TXV_WIRE_HD bool txvote_body(B b, uint32_t p, uint32_t end, Parsed& o) {
  uint32_t last = 0;
#pragma unroll 1
  for (uint32_t f = 1; f <= 6; ++f) {
    if (p == end) continue;
    uint32_t num = 0, typ = 0;
    const uint32_t k = field_key(b, p, end, num, typ);
    if (k && f < num) continue;
    if (!k || num <= last) return false;
    last = num;
    p += k;
    if (num != f || typ != (f == 1 ? TYP_VARINT : TYP_BYTES)) return false;
    uint32_t adv, body, blen;
    if (f == 1) {
      uint64_t v;
      if (!(adv = uvarint(b, p, end, v))) return false;
      o.height = (int64_t)v;
    } else if (f == 4) {
      if (!byte_slice(b, p, end, body, blen)) return false;
      const uint32_t used = time_body(b, body, body + blen, o.sec, o.nanos);
      if (used == UINT32_MAX) return false;
      adv = uvarint_size(blen) + used;
    } else {
      if (f == 3 && end - p < 32) return false;
      if (!(adv = byte_slice(b, p, end, body, blen))) return false;
      if (f == 2) { o.th_off = body; o.th_len = blen; }
      else if (f == 3) { if (blen != 32) return false; o.key_off = body; o.has_key = true; }
      else if (f == 5) { o.addr_off = body; o.addr_len = blen; }
      else { o.sig_off = body; o.sig_len = blen; }
    }
    p += adv;
  }
  return skip_rest(b, p, end, last);
}

// whole message [0, len): TXV_WIRE_OK or TXV_WIRE_ERR_DECODE
template <typename B>
TXV_WIRE_HD uint32_t parse_msg(B b, uint32_t len, uint32_t disamb, uint32_t prefix, Parsed& o) {
  auto word_at = [&](uint32_t p) {
    return (uint32_t)b[p] | ((uint32_t)b[p + 1] << 8) | ((uint32_t)b[p + 2] << 16) | ((uint32_t)b[p + 3] << 24);
  };
  if (len < 4) return 2;
  uint32_t p;
  if (b[0] == 0) {
    if (len < 8 || (word_at(0) & 0xFFFFFF00u) != (disamb << 8) || word_at(4) != prefix) return 2;
    p = 8;
  } else {
    if (word_at(0) != prefix) return 2;
    p = 4;
  }
  uint32_t last = 0;
  if (p < len) {
    uint32_t num = 0, typ = 0;
    const uint32_t k = field_key(b, p, len, num, typ);
    if (!(k && 1 < num)) {
      if (!k || num <= last) return 2;
      last = num;
      p += k;
      if (num != 1 || typ != TYP_BYTES) return 2;
      uint32_t body, blen;
      if (!byte_slice(b, p, len, body, blen)) return 2;
      if (!txvote_body(b, body, body + blen, o)) return 2;
      p += uvarint_size(blen) + blen;
    }
  }
  return skip_rest(b, p, len, last) ? 0u : 2u;
}

// ---- canonical-layout fast path ------------------------------------------------------------
// Straight-line (branch-free) parse of a message laid out the way the reference's encoder writes
// it: 4-byte prefix, key 0x0a, minimal body length ending the message, then the TxVote fields with
// their one-byte canonical keys (0x08 0x12 0x1a 0x22 0x2a 0x32, each present or absent) and a
// canonical time body (0x08 sec, 0x10 nanos, minimal length, fully consumed), nothing else.  It
// reads 8-byte windows (3 aligned words + 2 funnel shifts: one memory round trip per field
// instead of one per byte).  Whenever it returns true, parse_msg would return TXV_WIRE_OK with the
// same fields (every condition above is one the general rules accept the same way); anything else
// returns false and the lane takes parse_msg.  Reads stay within the message + 12 bytes.

// 8 bytes at byte position pos of the word array w
template <typename WP>
TXV_WIRE_HD uint64_t peek8(WP w, uint32_t pos) {
  const uint32_t a = pos >> 2, sh = (pos & 3u) * 8u;
  const uint32_t x0 = w[a], x1 = w[a + 1], x2 = w[a + 2];
  const uint32_t lo = sh ? funnel(x1, x0, sh) : x0, hi = sh ? funnel(x2, x1, sh) : x1;
  return ((uint64_t)hi << 32) | lo;
}

// uvarint in the low bytes of x (bytes beyond `avail` are ignored): byte count, 0 = not terminated
TXV_WIRE_HD uint32_t vint(uint64_t x, uint32_t avail, uint64_t& v) {
  const uint64_t avail_mask = avail >= 8 ? ~0ull : ((1ull << (8 * avail)) - 1);
  const uint64_t term = ~x & 0x8080808080808080ull & avail_mask;
  const uint32_t n = term ? (uint32_t)(ctz64(term) >> 3) + 1u : 0u;
  uint64_t r = x & 0x7F7F7F7F7F7F7F7Full;
  r = (r & 0x007F007F007F007Full) | ((r & 0x7F007F007F007F00ull) >> 1);
  r = (r & 0x00003FFF00003FFFull) | ((r & 0x3FFF00003FFF0000ull) >> 2);
  r = (r & 0x000000000FFFFFFFull) | ((r & 0x0FFFFFFF00000000ull) >> 4);
  v = n >= 8 ? r : (r & ((1ull << (7 * n)) - 1));
  return n;
}

template <typename WP>
TXV_WIRE_HD bool fast_msg(WP w, uint32_t m0, uint32_t len, uint32_t prefix, Parsed& o) {
  bool ok = len >= 7;
  uint64_t x = peek8(w, m0), v;
  ok = ok && (uint32_t)x == prefix && ((x >> 32) & 0xFF) == 0x0Au;
  const uint32_t nb = vint(x >> 40, 3, v);
  ok = ok && nb && nb == uvarint_size(v) && v == (uint64_t)(len - 5 - nb);
  const uint32_t end = len;
  uint32_t q = ok ? 5 + nb : end;
  // advance q past n more bytes, failing (and parking q at end) when they do not fit
  auto adv = [&](bool pres, uint64_t n) {
    const bool fits = n <= (uint64_t)(end - q);
    ok = ok && (!pres || fits);
    q = !pres ? q : (fits ? q + (uint32_t)n : end);
  };
  // 1 Height
  x = peek8(w, m0 + q);
  bool pres = q < end && (x & 0xFF) == 0x08u;
  uint32_t n = vint(x >> 8, 7, v);
  ok = ok && (!pres || n);
  o.height = pres ? (int64_t)v : 0;
  adv(pres, 1 + n);
  // 2 TxHash, 5 ValidatorAddress, 6 Signature share the bytes-field shape
  auto bytes_field = [&](uint32_t key, uint32_t& off, uint32_t& flen) {
    const uint64_t y = peek8(w, m0 + q);
    const bool p = q < end && (y & 0xFF) == key;
    uint64_t l;
    const uint32_t k = vint(y >> 8, 7, l);
    ok = ok && (!p || k);
    adv(p, 1 + k);
    off = p ? q : 0;
    flen = p ? (uint32_t)(l < 0xFFFFFFFFull ? l : 0xFFFFFFFFull) : 0;
    adv(p, l);
  };
  bytes_field(0x12u, o.th_off, o.th_len);
  // 3 TxKey: 0x1a 0x20 + 32 bytes
  x = peek8(w, m0 + q);
  pres = q < end && (x & 0xFFFF) == 0x201Au;
  o.has_key = pres;
  o.key_off = pres ? q + 2 : 0;
  adv(pres, 34);
  // 4 Timestamp: minimal length, canonical body, fully consumed
  x = peek8(w, m0 + q);
  pres = q < end && (x & 0xFF) == 0x22u;
  uint64_t tl;
  n = vint(x >> 8, 7, tl);
  ok = ok && (!pres || (n && n == uvarint_size(tl)));
  adv(pres, 1 + n);
  const uint32_t t0 = q;
  adv(pres, tl);
  const uint32_t te = pres ? q : t0;
  uint32_t t = t0;
  x = peek8(w, m0 + t);
  const bool s_pres = t < te && (x & 0xFF) == 0x08u;
  uint64_t sec;
  n = vint(x >> 8, 7, sec);
  ok = ok && (!s_pres || (n && t + 1 + n <= te && (int64_t)sec >= -62135596800LL && (int64_t)sec < 253402300800LL));
  t = s_pres ? t + 1 + n : t;
  x = peek8(w, m0 + (t < te ? t : te));
  const bool n_pres = t < te && (x & 0xFF) == 0x10u;
  uint64_t ns;
  n = vint(x >> 8, 7, ns);
  ok = ok && (!n_pres || (n && t + 1 + n <= te && ns <= 999999999ull));
  t = n_pres ? t + 1 + n : t;
  ok = ok && t == te;
  o.sec = s_pres ? (int64_t)sec : 0;
  o.nanos = n_pres ? (int32_t)ns : 0;
  bytes_field(0x2Au, o.addr_off, o.addr_len);
  bytes_field(0x32u, o.sig_off, o.sig_len);
  return ok && q == end;
}

// copy `len` bytes (<= 4 * W) from src byte offset o into W output words, zero beyond len.
// Reads W + 1 aligned words unconditionally (all loads in flight at once): the callers guarantee
// 4 readable bytes past every field (LDS slack / >= 16 bytes of padding after the wire buffer).
template <int W, typename WP>
TXV_WIRE_HD void copy_row(WP words, uint32_t o, uint32_t len, uint32_t* out) {
  const uint32_t a = o >> 2, sh = (o & 3u) * 8u;
  uint32_t x[W + 1];
#pragma unroll
  for (int j = 0; j <= W; ++j) x[j] = words[a + j];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    uint32_t v = sh ? funnel(x[j + 1], x[j], sh) : x[j];
    const int valid = (int)len - 4 * j;
    if (valid <= 0) v = 0;
    else if (valid < 4) v &= 0xFFFFFFFFu >> (8 * (4 - valid));
    out[j] = v;
  }
}

}  // namespace wire
}  // namespace txv
