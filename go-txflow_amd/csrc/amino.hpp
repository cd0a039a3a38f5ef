// amino.hpp — host encoder for the TxVote amino byte strings the hot path hashes.
//
// SignBytes = cdc.MarshalBinaryLengthPrefixed(CanonicalizeTxVote(chainID, vote))
//   (types/tx_vote.go:83-89, CanonicalTxVote :177-183, CanonicalizeTxVote :185-192; encoder is
//   go-amino v0.15.1-0.20190603130624-25d5598ed22b, external).  Field rules:
//   Height fixed64 (0x09, omitted when 0), TxHash (0x12), TxKey (0x1a 0x20 + 32 zero bytes:
//   CanonicalizeTxVote never copies it), Timestamp (0x22, body {0x08 uvarint(uint64 sec)}
//   {0x10 uvarint(nanos)}, sub-fields omitted when 0, whole field omitted when empty),
//   ChainID (0x2a, omitted when empty).  Out-of-range times make amino error -> SignBytes panics.
// Size = len(cdc.MarshalBinaryBare(TxVote)) (types/tx_vote.go:144-150).
// The commit side effects' encodings (TxStore.SaveTx, tx/store.go:83-107; MakeCommit,
// types/vote_set.go:242-259) are built from the same TxVote body.
#pragma once
#include <stdint.h>
#include <string.h>

// the size rules also run on the device (kernels_wire.hip: TxVote.Size() of decoded messages)
#if defined(__HIPCC__)
#define TXV_AHD __host__ __device__ inline
#else
#define TXV_AHD inline
#endif

namespace txv_host {

constexpr int64_t kAminoMinSec = -62135596800LL;   // 0001-01-01T00:00:00Z
constexpr int64_t kAminoMaxSec = 253402300800LL;   // 10000-01-01T00:00:00Z (exclusive)

TXV_AHD uint32_t put_uvarint(uint8_t* out, uint64_t v) {
  uint32_t n = 0;
  while (v >= 0x80) { if (out) out[n] = (uint8_t)(v | 0x80); ++n; v >>= 7; }
  if (out) out[n] = (uint8_t)v;
  return n + 1;
}

// time body length (or -1 when amino rejects the time)
TXV_AHD int time_body(uint8_t* out, int64_t sec, int32_t nanos) {
  uint32_t n = 0;
  if (sec != 0) {
    if (sec < kAminoMinSec || sec >= kAminoMaxSec) return -1;
    if (out) out[n] = 0x08;
    ++n;
    n += put_uvarint(out ? out + n : nullptr, (uint64_t)sec);
  }
  if (nanos != 0) {
    if (nanos < 0 || nanos > 999999999) return -1;
    if (out) out[n] = 0x10;
    ++n;
    n += put_uvarint(out ? out + n : nullptr, (uint64_t)(uint32_t)nanos);
  }
  return (int)n;
}

// SignBytes length (or -1 when amino rejects the time), without encoding
TXV_AHD int sign_bytes_len(int64_t height, uint32_t txhash_len, int64_t sec, int32_t nanos, uint32_t chain_len) {
  const int tl = time_body(nullptr, sec, nanos);
  if (tl < 0) return -1;
  uint64_t body = 0;
  if (height != 0) body += 9;
  if (txhash_len) body += 1 + put_uvarint(nullptr, txhash_len) + txhash_len;
  body += 34;
  if (tl > 0) body += 1 + put_uvarint(nullptr, (uint64_t)tl) + (uint64_t)tl;
  if (chain_len) body += 1 + put_uvarint(nullptr, chain_len) + chain_len;
  return (int)(put_uvarint(nullptr, body) + body);
}

// Writes SignBytes into out (capacity cap).  Returns length, or -1 (amino error / too long).
inline int sign_bytes(uint8_t* out, uint32_t cap, int64_t height, const uint8_t* txhash, uint32_t txhash_len,
                      int64_t sec, int32_t nanos, const uint8_t* chain, uint32_t chain_len) {
  uint8_t tb[24];
  const int tl = time_body(tb, sec, nanos);
  if (tl < 0) return -1;
  uint64_t body = 0;
  if (height != 0) body += 9;
  if (txhash_len) body += 1 + put_uvarint(nullptr, txhash_len) + txhash_len;
  body += 34;
  if (tl > 0) body += 1 + put_uvarint(nullptr, (uint64_t)tl) + (uint64_t)tl;
  if (chain_len) body += 1 + put_uvarint(nullptr, chain_len) + chain_len;
  const uint32_t pl = put_uvarint(nullptr, body);
  if (pl + body > cap) return -1;
  uint8_t* p = out + put_uvarint(out, body);
  if (height != 0) {
    *p++ = 0x09;
    for (int i = 0; i < 8; ++i) *p++ = (uint8_t)((uint64_t)height >> (8 * i));
  }
  if (txhash_len) {
    *p++ = 0x12;
    p += put_uvarint(p, txhash_len);
    memcpy(p, txhash, txhash_len);
    p += txhash_len;
  }
  *p++ = 0x1a; *p++ = 0x20;
  memset(p, 0, 32); p += 32;
  if (tl > 0) {
    *p++ = 0x22;
    p += put_uvarint(p, (uint64_t)tl);
    memcpy(p, tb, (size_t)tl);
    p += tl;
  }
  if (chain_len) {
    *p++ = 0x2a;
    p += put_uvarint(p, chain_len);
    memcpy(p, chain, chain_len);
    p += chain_len;
  }
  return (int)(p - out);
}

TXV_AHD int txvote_size(int64_t height, uint32_t txhash_len, int64_t sec, int32_t nanos, uint32_t addr_len,
                       uint32_t sig_len) {
  const int tl = time_body(nullptr, sec, nanos);
  if (tl < 0) return 0;
  uint64_t n = 0;
  if (height != 0) n += 1 + put_uvarint(nullptr, (uint64_t)height);
  if (txhash_len) n += 1 + put_uvarint(nullptr, txhash_len) + txhash_len;
  n += 34;
  if (tl > 0) n += 1 + put_uvarint(nullptr, (uint64_t)tl) + (uint64_t)tl;
  if (addr_len) n += 1 + put_uvarint(nullptr, addr_len) + addr_len;
  if (sig_len) n += 1 + put_uvarint(nullptr, sig_len) + sig_len;
  return (int)n;
}

// the TxVote bare body (= cdc.MarshalBinaryBare(vote), and of a CommitSig, which is a TxVote,
// types/tx_vote.go:154-159): Height 0x08 varint, TxHash 0x12, TxKey 0x1a 0x20 + 32 bytes,
// Timestamp 0x22, ValidatorAddress 0x2a, Signature 0x32; empty fields omitted.  Writes
// txvote_size(...) bytes at p (the caller checked the time: tl >= 0).
inline uint8_t* txvote_body(uint8_t* p, int64_t height, const uint8_t* txhash, uint32_t txhash_len, const uint8_t* txkey,
                            const uint8_t* tb, int tl, const uint8_t* addr, uint32_t addr_len, const uint8_t* sig,
                            uint32_t sig_len) {
  auto bytes_field = [&](uint8_t key, const uint8_t* b, uint32_t len) {
    if (!len) return;
    *p++ = key;
    p += put_uvarint(p, len);
    memcpy(p, b, len);
    p += len;
  };
  if (height != 0) { *p++ = 0x08; p += put_uvarint(p, (uint64_t)height); }
  bytes_field(0x12, txhash, txhash_len);
  *p++ = 0x1a; *p++ = 0x20;
  if (txkey) memcpy(p, txkey, 32); else memset(p, 0, 32);
  p += 32;
  bytes_field(0x22, tb, (uint32_t)tl);
  bytes_field(0x2a, addr, addr_len);
  bytes_field(0x32, sig, sig_len);
  return p;
}

// cdc.MarshalBinaryBare(&TxVoteMessage{Tx: vote}) (txvotepool/reactor.go:248, registered as
// "tendermint/txvotepool/TxVoteMessage" :273-276): 4 prefix bytes, field 1 (0x0a) + uvarint(len) +
// the TxVote bare body (fields as txvote_size).  out == nullptr: length only.  -1 on an amino time error.
inline int64_t txvote_msg(uint8_t* out, const uint8_t prefix[4], int64_t height, const uint8_t* txhash,
                          uint32_t txhash_len, const uint8_t* txkey, int64_t sec, int32_t nanos, const uint8_t* addr,
                          uint32_t addr_len, const uint8_t* sig, uint32_t sig_len) {
  uint8_t tb[24];
  const int tl = time_body(tb, sec, nanos);
  if (tl < 0) return -1;
  const uint64_t body = (uint64_t)txvote_size(height, txhash_len, sec, nanos, addr_len, sig_len);
  const uint64_t total = 5 + put_uvarint(nullptr, body) + body;
  if (!out) return (int64_t)total;
  memcpy(out, prefix, 4);
  out[4] = 0x0a;
  uint8_t* p = out + 5 + put_uvarint(out + 5, body);
  p = txvote_body(p, height, txhash, txhash_len, txkey, tb, tl, addr, addr_len, sig, sig_len);
  return (int64_t)(p - out);
}

// one accepted vote of a set (what TxVoteSet.votes holds) for the commit encodings
struct CommitVote {
  int64_t height, ts_sec;
  int32_t ts_nanos;
  const uint8_t* txkey;     // 32 bytes
  const uint8_t* addr;      // 20 bytes (the registry address the vote carried)
  const uint8_t* sig;       // 64 bytes
};

// cdc.MustMarshalBinaryBare(Commit{TxHash, Commits}) (types/vote_set.go:242-287; TxStore.SaveTx,
// tx/store.go:92-93): field 1 TxHash (0x0a, omitted when empty), field 2 (0x12) once per
// CommitSig, each length-prefixed with its TxVote body (the TxHash inside every CommitSig is the
// set's: the votes of a set all carry it).  Returns the length (out == nullptr: length only), -1
// when a vote's time is out of amino's range (MustMarshal panics).
inline int64_t commit_bytes(uint8_t* out, const uint8_t* txhash, uint32_t txhash_len, const CommitVote* v, uint32_t n) {
  uint64_t total = txhash_len ? 1 + put_uvarint(nullptr, txhash_len) + txhash_len : 0;
  for (uint32_t k = 0; k < n; ++k) {
    const int sz = txvote_size(v[k].height, txhash_len, v[k].ts_sec, v[k].ts_nanos, 20, 64);
    if (time_body(nullptr, v[k].ts_sec, v[k].ts_nanos) < 0) return -1;
    total += 1 + put_uvarint(nullptr, (uint64_t)sz) + (uint64_t)sz;
  }
  if (!out) return (int64_t)total;
  uint8_t* p = out;
  if (txhash_len) {
    *p++ = 0x0a;
    p += put_uvarint(p, txhash_len);
    memcpy(p, txhash, txhash_len);
    p += txhash_len;
  }
  for (uint32_t k = 0; k < n; ++k) {
    uint8_t tb[24];
    const int tl = time_body(tb, v[k].ts_sec, v[k].ts_nanos);
    const int sz = txvote_size(v[k].height, txhash_len, v[k].ts_sec, v[k].ts_nanos, 20, 64);
    *p++ = 0x12;
    p += put_uvarint(p, (uint64_t)sz);
    p = txvote_body(p, v[k].height, txhash, txhash_len, v[k].txkey, tb, tl, v[k].addr, 20, v[k].sig, 64);
  }
  return (int64_t)(p - out);
}

// cdc.MustMarshalBinaryBare(TxVoteSet) (tx/store.go:88-89): only the exported fields are
// encoded -- TxHash (0x0a, omitted when empty) and TxKey (0x12 0x20 + 32 bytes)
inline uint32_t txvoteset_bytes(uint8_t* out, const uint8_t* txhash, uint32_t txhash_len, const uint8_t txkey[32]) {
  const uint32_t total = (txhash_len ? 1 + put_uvarint(nullptr, txhash_len) + txhash_len : 0) + 34;
  if (!out) return total;
  uint8_t* p = out;
  if (txhash_len) {
    *p++ = 0x0a;
    p += put_uvarint(p, txhash_len);
    memcpy(p, txhash, txhash_len);
    p += txhash_len;
  }
  *p++ = 0x12; *p++ = 0x20;
  memcpy(p, txkey, 32);
  return total;
}

// calcTxKey / calcTxCommitKey (tx/store.go:111-117): fmt.Sprintf("H:%X", txHash) -- the
// upper-case hex of the TxHash string's bytes after a two-byte prefix
inline uint32_t store_key(uint8_t* out, char tag, const uint8_t* txhash, uint32_t txhash_len) {
  if (!out) return 2 + 2 * txhash_len;
  static const char hex[] = "0123456789ABCDEF";
  out[0] = (uint8_t)tag;
  out[1] = ':';
  for (uint32_t k = 0; k < txhash_len; ++k) {
    out[2 + 2 * k] = (uint8_t)hex[txhash[k] >> 4];
    out[3 + 2 * k] = (uint8_t)hex[txhash[k] & 15];
  }
  return 2 + 2 * txhash_len;
}

}  // namespace txv_host
