/*
 * amino.c — restatement of the go-amino (v0.15.1-0.20190603130624-25d5598ed22b, external)
 * encodings used on the TxVote admission path.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * SignBytes: types/tx_vote.go:83-89 = cdc.MarshalBinaryLengthPrefixed(CanonicalizeTxVote(..))
 *   CanonicalTxVote (types/tx_vote.go:177-183) field order / tags:
 *     1 Height int64 `binary:"fixed64"`   0x09 + 8 B LE        omitted when 0
 *     2 TxHash string                     0x12 + uvarint len   omitted when ""
 *     3 TxKey [32]byte                    0x1a 0x20 + 32 B     never omitted; always zero because
 *                                                             CanonicalizeTxVote (:185-191) does not copy it
 *     4 Timestamp time.Time               0x22 + uvarint len + {0x08 uvarint(uint64(sec))}{0x10 uvarint(nanos)}
 *                                         sub-fields omitted when 0; field omitted when its body is empty
 *     5 ChainID string                    0x2a + uvarint len   omitted when ""
 *   Pinned against types/vote_test.go:62 (the Go zero time encodes as
 *   0x08 0x80 0x92 0xb8 0xc3 0x98 0xfe 0xff 0xff 0xff 0x01).
 * Size: types/tx_vote.go:144-150 = len(cdc.MarshalBinaryBare(TxVote)); TxVote (types/tx_vote.go:48-55)
 *   fields 1 Height (uvarint of uint64(int64), 0x08), 2 TxHash (0x12), 3 TxKey (0x1a, 34 B),
 *   4 Timestamp (0x22), 5 ValidatorAddress (0x2a), 6 Signature (0x32).
 *   Pinned by txvotepool/txvotepool_test.go:102 (Size()==114 for a 20-byte-tx vote).
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

#define AMINO_MIN_SEC (-62135596800LL)
#define AMINO_MAX_SEC (253402300800LL)

static size_t uvarint(uint8_t* out, uint64_t v) {
  size_t n = 0;
  while (v >= 0x80) { if (out) out[n] = (uint8_t)(v | 0x80); ++n; v >>= 7; }
  if (out) out[n] = (uint8_t)v;
  return n + 1;
}

/* encodes the time body (without key/length); returns length, -1 if out of range */
static int time_body(uint8_t* out, int64_t sec, int32_t nanos) {
  size_t n = 0;
  if (sec != 0) {
    if (sec < AMINO_MIN_SEC || sec >= AMINO_MAX_SEC) return -1;
    if (out) out[n] = 0x08;
    n += 1;
    n += uvarint(out ? out + n : 0, (uint64_t)sec);
  }
  if (nanos != 0) {
    if (nanos < 0 || nanos > 999999999) return -1;
    if (out) out[n] = 0x10;
    n += 1;
    n += uvarint(out ? out + n : 0, (uint64_t)(uint32_t)nanos);
  }
  return (int)n;
}

int orc_signbytes(int64_t height, const uint8_t* txhash, size_t txhash_len,
                  int64_t ts_sec, int32_t ts_nanos,
                  const uint8_t* chain_id, size_t chain_len, uint8_t* out, size_t out_cap) {
  uint8_t* body = (uint8_t*)malloc(txhash_len + chain_len + 128);
  size_t n = 0;
  if (!body) return -1;
  if (height != 0) {
    body[n++] = 0x09;
    for (int i = 0; i < 8; ++i) body[n++] = (uint8_t)((uint64_t)height >> (8 * i));
  }
  if (txhash_len) {
    body[n++] = 0x12;
    n += uvarint(body + n, txhash_len);
    memcpy(body + n, txhash, txhash_len); n += txhash_len;
  }
  body[n++] = 0x1a; body[n++] = 0x20;
  memset(body + n, 0, 32); n += 32;
  uint8_t tb[32];
  int tl = time_body(tb, ts_sec, ts_nanos);
  if (tl < 0) { free(body); return -1; }
  if (tl > 0) {
    body[n++] = 0x22;
    n += uvarint(body + n, (uint64_t)tl);
    memcpy(body + n, tb, (size_t)tl); n += (size_t)tl;
  }
  if (chain_len) {
    body[n++] = 0x2a;
    n += uvarint(body + n, chain_len);
    memcpy(body + n, chain_id, chain_len); n += chain_len;
  }
  size_t pl = uvarint(0, n);
  if (pl + n > out_cap) { free(body); return -1; }
  uvarint(out, n);
  memcpy(out + pl, body, n);
  free(body);
  return (int)(pl + n);
}

int orc_txvote_size(int64_t height, size_t txhash_len, int64_t ts_sec, int32_t ts_nanos,
                    size_t addr_len, size_t sig_len) {
  size_t n = 0;
  if (height != 0) n += 1 + uvarint(0, (uint64_t)height);
  if (txhash_len) n += 1 + uvarint(0, txhash_len) + txhash_len;
  n += 34;
  int tl = time_body(0, ts_sec, ts_nanos);
  if (tl < 0) return 0;
  if (tl > 0) n += 1 + uvarint(0, (uint64_t)tl) + (size_t)tl;
  if (addr_len) n += 1 + uvarint(0, addr_len) + addr_len;
  if (sig_len) n += 1 + uvarint(0, sig_len) + sig_len;
  return (int)n;
}
