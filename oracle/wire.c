/*
 * wire.c — restatement of the TxVoteMessage wire codec on the ingest path.  TEST INFRASTRUCTURE
 * ONLY (see oracle.h).
 *
 * Reference: Reactor.Receive (txvotepool/reactor.go:170-190) -> decodeMsg (:278-284):
 *   len(bz) > MaxMsgBytes                  -> ErrTxTooLarge (peer stopped)
 *   cdc.UnmarshalBinaryBare(bz, &msg)      msg is the TxpoolMessage interface; the codec
 *                                          (txvotepool/codec.go) registers one concrete,
 *                                          &TxVoteMessage{} as "tendermint/txvotepool/TxVoteMessage"
 *                                          (reactor.go:273-276); TxVoteMessage{Tx types.TxVote} (:288-291)
 *   *TxVoteMessage                         -> CheckTxWithInfo(msg.Tx, ...)
 *   anything else (nil msg)                -> "Unknown message type", ignored
 *
 * The amino rules (go-amino v0.15.1-0.20190603130624-25d5598ed22b, external, not in the container:
 * restated from its published algorithm; beyond round trips of the reference's own encoder and
 * txMessageSize (txvotepool/txvotepool_test.go:301-303) this decoder is PARITY UNPINNED):
 *   interface, bare:   empty -> nil msg, no error.  Else DecodeDisambPrefixBytes: < 4 bytes error;
 *                      first byte 0x00 -> 8-byte disfix (0x00, 3 disambiguation, 4 prefix bytes),
 *                      else 4 prefix bytes; both must name the registered concrete.  disamb/prefix =
 *                      SHA-256(name) with leading zero bytes skipped, 3 bytes, zero bytes skipped,
 *                      4 bytes (nameToDisfix).
 *   top level:         every byte must be consumed (UnmarshalBinaryBare "didn't read all bytes").
 *   struct fields:     for each declared field in order: nothing left -> default; read key
 *                      (uvarint, typ3 = low 3 bits, num <= 2^29-1); key num > field num -> default,
 *                      key re-read for the next field; num <= last seen -> error; num != field num
 *                      -> error; typ3 != the field's -> error; decode the value.  Then the remaining
 *                      bytes as extra fields (num strictly increasing) skipped by typ3: 0 varint,
 *                      1 8 bytes, 2 length-prefixed, 5 4 bytes, else error.
 *   uvarint:           Go binary.Uvarint: overlong encodings accepted, > 10 bytes or a 10th byte > 1
 *                      overflow, running out of bytes is an error.
 *   length-prefixed:   uvarint count; count >= 2^63 or count > remaining -> error.
 *   [32]byte (TxKey):  remaining < 32 -> error; length-prefixed, length must be exactly 32.
 *   int64 (Height):    typ3 varint, uvarint reinterpreted as int64 (no zigzag).
 *   nested struct:     length-prefixed body; the parent advances by UvarintSize(len(body)) (the
 *                      minimal prefix size, not the bytes it read) + what the body decoder consumed
 *                      (decodeReflectBinaryStruct's n accounting).
 *   time.Time body:    [key 1 varint: seconds, uvarint as int64, in [-62135596800, 253402300800)]
 *                      [key 2 varint: nanos <= 999999999]; a different key is left unread (the
 *                      field stays 0); missing -> 0 = the Unix epoch (amino's default time).
 *                      Bytes left unread in the body are NOT an error: they are not counted in the
 *                      parent's advance, so the parent reads them again as its own next key.
 */
#include "oracle.h"
#include <string.h>
#include <time.h>

#define TYP_VARINT 0
#define TYP_8BYTE 1
#define TYP_BYTES 2
#define TYP_4BYTE 5
#define MIN_SEC (-62135596800LL)
#define MAX_SEC (253402300800LL)

typedef struct {
  const uint8_t* base;   /* start of the whole message (offsets are relative to it) */
  int err;
} dctx;

/* Go binary.Uvarint on [p, end): returns bytes read (> 0) or 0 on error */
static size_t get_uvarint(const uint8_t* p, const uint8_t* end, uint64_t* v) {
  uint64_t x = 0;
  unsigned s = 0;
  for (size_t i = 0; p + i < end; ++i) {
    const uint8_t b = p[i];
    if (b < 0x80) {
      if (i > 9 || (i == 9 && b > 1)) return 0;
      *v = x | ((uint64_t)b << s);
      return i + 1;
    }
    if (i >= 9) return 0;   /* 10 continuation bytes: overflow whatever follows */
    x |= (uint64_t)(b & 0x7f) << s;
    s += 7;
  }
  return 0;
}

static size_t uvarint_size(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) { v >>= 7; ++n; }
  return n;
}

static size_t get_key(const uint8_t* p, const uint8_t* end, uint32_t* num, unsigned* typ) {
  uint64_t v;
  const size_t k = get_uvarint(p, end, &v);
  if (!k) return 0;
  if ((v >> 3) > ((1u << 29) - 1)) return 0;
  *num = (uint32_t)(v >> 3);
  *typ = (unsigned)(v & 7);
  return k;
}

/* DecodeByteSlice: returns bytes read and the body [*b, *b + *blen) */
static size_t get_bytes(const uint8_t* p, const uint8_t* end, const uint8_t** b, uint64_t* blen) {
  uint64_t cnt;
  const size_t k = get_uvarint(p, end, &cnt);
  if (!k) return 0;
  if (cnt >> 63) return 0;
  if (cnt > (uint64_t)(end - p - (ptrdiff_t)k)) return 0;
  *b = p + k;
  *blen = cnt;
  return k + (size_t)cnt;
}

/* consumeAny */
static size_t skip_value(const uint8_t* p, const uint8_t* end, unsigned typ) {
  uint64_t v;
  const uint8_t* b;
  switch (typ) {
    case TYP_VARINT: return get_uvarint(p, end, &v);
    case TYP_8BYTE: return end - p >= 8 ? 8 : 0;
    case TYP_BYTES: return get_bytes(p, end, &b, &v);
    case TYP_4BYTE: return end - p >= 4 ? 4 : 0;
    default: return 0;
  }
}

/* time body: returns consumed bytes (may be < len), or (size_t)-1 on error */
static size_t decode_time(const uint8_t* p, const uint8_t* end, int64_t* sec, int32_t* nanos) {
  const uint8_t* q = p;
  uint32_t num;
  unsigned typ;
  uint64_t v;
  size_t k;
  *sec = 0;
  *nanos = 0;
  if (q < end) {
    if (!(k = get_key(q, end, &num, &typ))) return (size_t)-1;
    if (num == 1 && typ == TYP_VARINT) {
      q += k;
      if (!(k = get_uvarint(q, end, &v))) return (size_t)-1;
      q += k;
      if ((int64_t)v < MIN_SEC || (int64_t)v >= MAX_SEC) return (size_t)-1;
      *sec = (int64_t)v;
    }
  }
  if (q < end) {
    if (!(k = get_key(q, end, &num, &typ))) return (size_t)-1;
    if (num == 2 && typ == TYP_VARINT) {
      q += k;
      if (!(k = get_uvarint(q, end, &v))) return (size_t)-1;
      q += k;
      if (v > 999999999ull) return (size_t)-1;
      *nanos = (int32_t)v;
    }
  }
  return (size_t)(q - p);
}

/* TxVote fields (types/tx_vote.go:48-55): 1 Height varint, 2 TxHash bytes, 3 TxKey [32]byte,
 * 4 Timestamp struct, 5 ValidatorAddress bytes, 6 Signature bytes.  Decodes the body
 * [p, end) completely; returns 0 on success. */
static int decode_txvote(dctx* d, const uint8_t* p, const uint8_t* end, orc_wire_vote* o) {
  static const unsigned ftyp[7] = {0, TYP_VARINT, TYP_BYTES, TYP_BYTES, TYP_BYTES, TYP_BYTES, TYP_BYTES};
  uint32_t last = 0;
  for (uint32_t f = 1; f <= 6; ++f) {
    if (p == end) continue;   /* default value (already zeroed) */
    uint32_t num = 0;
    unsigned typ = 0;
    const size_t k = get_key(p, end, &num, &typ);
    if (k && f < num) continue;            /* field absent: re-read the key for the next field */
    if (!k || num <= last) return -1;
    last = num;
    p += k;
    if (num != f || typ != ftyp[f]) return -1;
    const uint8_t* b;
    uint64_t blen, v;
    size_t adv;
    switch (f) {
      case 1:
        if (!(adv = get_uvarint(p, end, &v))) return -1;
        o->height = (int64_t)v;
        break;
      case 3:
        if (end - p < 32) return -1;
        if (!(adv = get_bytes(p, end, &b, &blen)) || blen != 32) return -1;
        memcpy(o->txkey, b, 32);
        break;
      case 4: {
        if (!(get_bytes(p, end, &b, &blen))) return -1;
        const size_t used = decode_time(b, b + blen, &o->ts_sec, &o->ts_nanos);
        if (used == (size_t)-1) return -1;
        adv = uvarint_size(blen) + used;   /* decodeReflectBinaryStruct's n */
        break;
      }
      default:
        if (!(adv = get_bytes(p, end, &b, &blen))) return -1;
        if (f == 2) { o->txhash_off = (uint32_t)(b - d->base); o->txhash_len = (uint32_t)blen; }
        if (f == 5) { o->addr_off = (uint32_t)(b - d->base); o->addr_len = (uint32_t)blen; }
        if (f == 6) { o->sig_off = (uint32_t)(b - d->base); o->sig_len = (uint32_t)blen; }
        break;
    }
    p += adv;
  }
  while (p < end) {   /* extra fields */
    uint32_t num;
    unsigned typ;
    const size_t k = get_key(p, end, &num, &typ);
    if (!k || num <= last) return -1;
    last = num;
    p += k;
    const size_t adv = skip_value(p, end, typ);
    if (!adv) return -1;
    p += adv;
  }
  return 0;
}

void orc_wire_prefix(uint8_t disamb[3], uint8_t prefix[4]) {
  static const char name[] = "tendermint/txvotepool/TxVoteMessage";
  uint8_t h[32];
  orc_sha256((const uint8_t*)name, sizeof name - 1, h);
  size_t i = 0;
  while (h[i] == 0) ++i;
  memcpy(disamb, h + i, 3);
  i += 3;
  while (h[i] == 0) ++i;
  memcpy(prefix, h + i, 4);
}

int orc_wire_decode(const uint8_t* bz, size_t len, uint32_t max_msg_bytes, orc_wire_vote* o) {
  memset(o, 0, sizeof *o);
  if (len > max_msg_bytes) return ORC_WIRE_TOO_LARGE;
  if (len == 0) return ORC_WIRE_NIL;
  uint8_t disamb[3], prefix[4];
  orc_wire_prefix(disamb, prefix);
  dctx d = {bz, 0};
  const uint8_t* p = bz;
  const uint8_t* end = bz + len;
  if (len < 4) return ORC_WIRE_ERR_DECODE;
  if (bz[0] == 0x00) {
    if (len < 8 || memcmp(bz + 1, disamb, 3) || memcmp(bz + 4, prefix, 4)) return ORC_WIRE_ERR_DECODE;
    p += 8;
  } else {
    if (memcmp(bz, prefix, 4)) return ORC_WIRE_ERR_DECODE;
    p += 4;
  }
  /* TxVoteMessage, bare: one field, 1 Tx (struct, length-prefixed) */
  uint32_t last = 0;
  if (p < end) {
    uint32_t num = 0;
    unsigned typ = 0;
    const size_t k = get_key(p, end, &num, &typ);
    if (!(k && 1 < num)) {
      if (!k || num <= last) goto bad;
      last = num;
      p += k;
      if (num != 1 || typ != TYP_BYTES) goto bad;
      const uint8_t* b;
      uint64_t blen;
      if (!get_bytes(p, end, &b, &blen)) goto bad;
      if (decode_txvote(&d, b, b + blen, o)) goto bad;
      p += uvarint_size(blen) + blen;   /* the body decoder consumed all of it */
    }
  }
  while (p < end) {
    uint32_t num;
    unsigned typ;
    const size_t k = get_key(p, end, &num, &typ);
    if (!k || num <= last) goto bad;
    last = num;
    p += k;
    const size_t adv = skip_value(p, end, typ);
    if (!adv) goto bad;
    p += adv;
  }
  return ORC_WIRE_OK;
bad:
  memset(o, 0, sizeof *o);
  return ORC_WIRE_ERR_DECODE;
}

static size_t put_uvarint(uint8_t* out, uint64_t v) {
  size_t n = 0;
  while (v >= 0x80) { if (out) out[n] = (uint8_t)(v | 0x80); ++n; v >>= 7; }
  if (out) out[n] = (uint8_t)v;
  return n + 1;
}

static size_t put_bytes_field(uint8_t* out, uint8_t key, const uint8_t* b, size_t len) {
  if (!len) return 0;
  size_t n = 0;
  if (out) out[n] = key;
  ++n;
  n += put_uvarint(out ? out + n : 0, len);
  if (out) memcpy(out + n, b, len);
  return n + len;
}

/* cdc.MarshalBinaryBare(TxVote) -- also a CommitSig's bytes (types/tx_vote.go:154-159) --
 * field rules as TxVote.Size (types/tx_vote.go:144-150).  out == 0: length only; -1 when amino
 * rejects the timestamp. */
int orc_txvote_encode(int64_t height, const uint8_t* txhash, size_t txhash_len, const uint8_t* txkey,
                      int64_t ts_sec, int32_t ts_nanos, const uint8_t* addr, size_t addr_len,
                      const uint8_t* sig, size_t sig_len, uint8_t* w) {
  if (ts_sec != 0 && (ts_sec < MIN_SEC || ts_sec >= MAX_SEC)) return -1;
  if (ts_nanos < 0 || ts_nanos > 999999999) return -1;
  uint8_t tb[24];
  size_t tl = 0;
  if (ts_sec != 0) { tb[tl++] = 0x08; tl += put_uvarint(tb + tl, (uint64_t)ts_sec); }
  if (ts_nanos != 0) { tb[tl++] = 0x10; tl += put_uvarint(tb + tl, (uint64_t)ts_nanos); }
  static const uint8_t zero32[32];
  size_t n = 0;
  if (height != 0) {
    if (w) w[n] = 0x08;
    n += 1 + put_uvarint(w ? w + n + 1 : 0, (uint64_t)height);
  }
  n += put_bytes_field(w ? w + n : 0, 0x12, txhash, txhash_len);
  if (w) { w[n] = 0x1a; w[n + 1] = 0x20; memcpy(w + n + 2, txkey ? txkey : zero32, 32); }
  n += 34;
  n += put_bytes_field(w ? w + n : 0, 0x22, tb, tl);
  n += put_bytes_field(w ? w + n : 0, 0x2a, addr, addr_len);
  n += put_bytes_field(w ? w + n : 0, 0x32, sig, sig_len);
  return (int)n;
}

int orc_wire_encode(int64_t height, const uint8_t* txhash, size_t txhash_len, const uint8_t* txkey,
                    int64_t ts_sec, int32_t ts_nanos, const uint8_t* addr, size_t addr_len,
                    const uint8_t* sig, size_t sig_len, uint8_t* out, size_t cap) {
  /* 4 prefix bytes of the registered TxVoteMessage, field 1 = the TxVote body */
  const int body = orc_txvote_encode(height, txhash, txhash_len, txkey, ts_sec, ts_nanos, addr, addr_len, sig, sig_len, 0);
  if (body < 0) return -1;
  uint8_t disamb[3], prefix[4];
  orc_wire_prefix(disamb, prefix);
  const size_t total = 4 + 1 + put_uvarint(0, (uint64_t)body) + (size_t)body;
  if (total > cap) return -1;
  memcpy(out, prefix, 4);
  out[4] = 0x0a;
  uint8_t* w = out + 5 + put_uvarint(out + 5, (uint64_t)body);
  orc_txvote_encode(height, txhash, txhash_len, txkey, ts_sec, ts_nanos, addr, addr_len, sig, sig_len, w);
  return (int)total;
}

/* CPU baseline: decode n messages in a loop on one thread; returns seconds */
double orc_wire_decode_many(const uint8_t* wire, const uint64_t* off, const uint32_t* len, uint32_t n,
                            uint32_t max_msg_bytes, uint8_t* status_out, orc_wire_vote* out) {
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (uint32_t i = 0; i < n; ++i) status_out[i] = (uint8_t)orc_wire_decode(wire + off[i], len[i], max_msg_bytes, out + i);
  clock_gettime(CLOCK_MONOTONIC, &b);
  return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}
