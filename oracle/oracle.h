/*
 * oracle.h — CPU restatement of go-txflow's TxVote admission path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X implementation under go-txflow_amd/.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product never links it.
 *
 * What it restates (reference = /root/reference, Fantom-foundation/go-txflow @2025-02-26):
 *   - types/tx_vote.go:83-89,177-192  TxVote.SignBytes / CanonicalTxVote  (amino, go-amino@25d5598ed22b, external)
 *   - types/tx_vote.go:110-119        TxVote.Verify
 *   - types/tx_vote.go:144-150        TxVote.Size (amino bare)
 *   - golang.org/x/crypto@c2843e01d9a2 ed25519.Verify (external)
 *   - types/vote_set.go:81-166        TxVoteSet.AddVote / addVote / addVerifiedVote
 *   - txflow/service.go:192-234       TxFlow.addVote routing by TxHash
 *   - txvotepool/reactor.go:170-190,273-291  Reactor.Receive / decodeMsg (TxVoteMessage amino wire codec)
 *
 * Parity pinning: the reference's Go code cannot be built here (no Go toolchain,
 * modules not vendored).  ed25519 results are pinned against
 * OpenSSL 3.0 (RFC 8032 deterministic) golden vectors in tests/golden/, SHA-2 against
 * hashlib, TxVote.Size against txvotepool/txvotepool_test.go:102 (Size()==114), and the
 * amino zero-time encoding against types/vote_test.go:62.  ed25519 decode rules for
 * non-canonical encodings follow Appendix A (x/crypto source is not present): those
 * verdicts are "parity unpinned" beyond OpenSSL agreement where the two libraries agree.
 */
#ifndef TXV_ORACLE_H
#define TXV_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- hashes ---- */
void orc_sha512(const uint8_t* msg, size_t len, uint8_t out[64]);
void orc_sha256(const uint8_t* msg, size_t len, uint8_t out[32]);

/* ---- ed25519 (x/crypto@c2843e01d9a2 semantics) ---- */
/* returns 1 accept / 0 reject.  sig_len != 64 rejects (tendermint VerifyBytes). */
int orc_ed25519_verify(const uint8_t pub[32], const uint8_t* msg, size_t msg_len,
                       const uint8_t* sig, size_t sig_len);
/* RFC 8032 key expansion from a 32-byte seed: pub = [a]B. */
void orc_ed25519_pubkey(const uint8_t seed[32], uint8_t pub[32]);
void orc_ed25519_sign(const uint8_t seed[32], const uint8_t* msg, size_t msg_len, uint8_t sig[64]);
/* point decode per ref10 FromBytes rules: 1 ok, 0 reject */
int orc_ed25519_decode_ok(const uint8_t pub[32]);
/* scalar helpers (exposed for tests) */
void orc_sc_reduce64(const uint8_t in[64], uint8_t out[32]);
int  orc_sc_minimal(const uint8_t s[32]);
/* crafted-point helpers for the adversarial generator:
 * [k]P where P is given by its 32-byte encoding (decode rules as verify; returns 0 if P invalid). */
int  orc_scalarmult(const uint8_t k[32], const uint8_t p_enc[32], uint8_t out[32]);
void orc_scalarmult_base(const uint8_t k[32], uint8_t out[32]);
/* canonical re-encoding of a decodable point (0 if not decodable) */
int  orc_point_canonical(const uint8_t p_enc[32], uint8_t out[32]);

/* ---- amino (go-amino@25d5598ed22b restatement) ---- */
/* SignBytes of CanonicalTxVote{Height, TxHash, TxKey=0, Timestamp, ChainID}, length-prefixed.
 * Returns byte count, or -1 when the timestamp is outside amino's range (SignBytes panics). */
int orc_signbytes(int64_t height, const uint8_t* txhash, size_t txhash_len,
                  int64_t ts_sec, int32_t ts_nanos,
                  const uint8_t* chain_id, size_t chain_len, uint8_t* out, size_t out_cap);
/* TxVote.Size(): amino MarshalBinaryBare(TxVote) length, 0 on error. */
int orc_txvote_size(int64_t height, size_t txhash_len, int64_t ts_sec, int32_t ts_nanos,
                    size_t addr_len, size_t sig_len);

/* ---- TxVote.Verify (types/tx_vote.go:110-119) ---- */
enum {
  ORC_ADDED = 0, ORC_DUPLICATE = 1, ORC_ERR_NIL = 2, ORC_ERR_EMPTY_ADDR = 3,
  ORC_ERR_UNKNOWN_VALIDATOR = 4, ORC_ERR_NONDETERMINISTIC = 5,
  ORC_ERR_INVALID_SIGNATURE = 6, ORC_ERR_INVALID_VALIDATOR_ADDRESS = 7
};

/* One TxVote in SoA-friendly flat form. */
typedef struct {
  int32_t  is_nil;
  int64_t  height;
  const uint8_t* txhash; uint32_t txhash_len;
  int64_t  ts_sec; int32_t ts_nanos;
  const uint8_t* addr; uint32_t addr_len;
  const uint8_t* sig;  uint32_t sig_len;
} orc_vote;

int orc_txvote_verify(const orc_vote* v, const uint8_t* chain_id, size_t chain_len,
                      const uint8_t pub[32]);

/* ---- sequential TxFlow.addVote -> TxVoteSet.AddVote restatement ---- */
typedef struct orc_flow orc_flow;
orc_flow* orc_flow_new(const uint8_t* pubs32, const int64_t* powers, uint32_t n_vals,
                       const uint8_t* chain_id, size_t chain_len);
void orc_flow_free(orc_flow*);
/* Process votes in order.  status[i] gets the ORC_* code; sum_after[i] the TxVoteSet
 * sum after the vote; fired[i] = 1 when the reference would run its commit side
 * effects for this vote (added && HasTwoThirdsMajority, txflow/service.go:216).
 * If verdicts != NULL it supplies precomputed ed25519 results (1/0) per vote and
 * the oracle does not verify; otherwise it verifies each vote that reaches step 4. */
void orc_flow_add_votes(orc_flow*, const orc_vote* votes, uint32_t n, const uint8_t* verdicts,
                        uint8_t* status, int64_t* sum_after, uint8_t* fired);
/* A batch in the txv_votes SoA layout (include/txvote.h): addr n x 20 and sig n x 64 hold
 * the first 20 / 64 bytes, addr_len / sig_len the true lengths; is_nil may be NULL. */
typedef struct {
  uint32_t n;
  const uint8_t* is_nil; const int64_t* height;
  const uint8_t* txhash; const uint32_t* txhash_off; const uint32_t* txhash_len;
  const int64_t* ts_sec; const int32_t* ts_nanos;
  const uint8_t* addr; const uint32_t* addr_len;
  const uint8_t* sig; const uint32_t* sig_len;
} orc_soa;
/* orc_flow_add_votes over an SoA batch; TxVote.Verify runs on `threads` threads first (for every
 * vote whose address is a validator's), then the sequential loop consumes those outcomes. */
void orc_flow_add_votes_soa(orc_flow*, const orc_soa* batch, int threads, uint8_t* status,
                            int64_t* sum_after, uint8_t* fired);
/* TxVote.Verify(chainID, pubKey) per vote of an SoA batch with caller-supplied keys pubs32[i]
 * (n x 32); nil votes -> ORC_ERR_NIL.  out[i] = ORC_ADDED (nil error) or the error code. */
void orc_txvote_verify_soa(const orc_soa* batch, const uint8_t* pubs32, const uint8_t* chain_id,
                           size_t chain_len, int threads, uint8_t* out);
/* Query a TxVoteSet: returns 0 if the tx has no set, else 1 and fills sum/maj23. */
int orc_flow_query(orc_flow*, const uint8_t* txhash, uint32_t txhash_len, int64_t* sum, int32_t* maj23);
uint32_t orc_flow_num_sets(orc_flow*);
/* TxVoteSet.GetVotes (types/vote_set.go:57-64) in validator index order: count of accepted votes;
 * val_out / sig_out (64 B each) receive up to cap of them */
uint32_t orc_flow_get_votes(orc_flow*, const uint8_t* txhash, uint32_t len, uint32_t* val_out, uint8_t* sig_out,
                            uint32_t cap);
/* count of ed25519 verifications performed (for baseline accounting) */
uint64_t orc_flow_num_verifies(orc_flow*);

/* ---- TxVotePool (txvotepool/txvotepool.go) restatement ----
 * cache_size 0xFFFFFFFF = nopTxCache.  orc_pool_check returns 0 ok, 1 ErrMempoolIsFull,
 * 2 ErrTxTooLarge, 3 ErrTxInCache, 4 WAL panic: with `wal` set, a vote whose TxVote.Size() is 0
 * (amino rejects its timestamp) panics in the WAL write after its cache push; without a WAL such
 * a vote is admitted with size 0 (types/tx_vote.go:144-150, txvotepool.go:192-261). */
typedef struct orc_pool orc_pool;
orc_pool* orc_pool_new(uint32_t size, uint32_t cache_size, uint64_t max_txs_bytes, uint32_t max_msg_bytes,
                       int64_t height, int wal);
void orc_pool_free(orc_pool*);
int orc_pool_check(orc_pool*, const orc_vote* v);
/* the same check for n votes given as (txVoteKey 32 B, TxVote.Size()) pairs */
void orc_pool_check_keys(orc_pool*, const uint8_t* keys32, const uint32_t* sizes, uint32_t n, uint8_t* out);
void orc_pool_check_soa(orc_pool*, const orc_soa* b, const uint8_t* sig_full, const uint64_t* sig_full_off,
                        uint8_t* out);
void orc_pool_update(orc_pool*, int64_t height, const orc_vote* votes, uint32_t n);
void orc_pool_update_keys(orc_pool*, int64_t height, const uint8_t* keys32, const uint32_t* sizes, uint32_t n);
void orc_pool_update_soa(orc_pool*, int64_t height, const orc_soa* b, const uint8_t* sig_full,
                         const uint64_t* sig_full_off);
uint64_t orc_pool_reap(orc_pool*, int64_t max, uint8_t* keys_out, uint32_t* sizes_out, uint64_t cap);
void orc_pool_flush(orc_pool*);
int64_t orc_pool_size(orc_pool*);
int64_t orc_pool_txs_bytes(orc_pool*);
uint64_t orc_pool_cache_keys(orc_pool*, uint8_t* keys_out, uint64_t cap);

/* ---- TxVoteMessage wire codec (txvotepool/reactor.go:170-190, 273-291; oracle/wire.c) ---- */
#define ORC_WIRE_OK 0          /* *TxVoteMessage decoded -> CheckTxWithInfo */
#define ORC_WIRE_TOO_LARGE 1   /* len > MaxMsgBytes: ErrTxTooLarge (decodeMsg) */
#define ORC_WIRE_ERR_DECODE 2  /* amino UnmarshalBinaryBare error */
#define ORC_WIRE_NIL 3         /* empty message: nil msg, "Unknown message type" */
typedef struct {
  int64_t height;
  uint32_t txhash_off, txhash_len;   /* offsets into the message bytes */
  uint8_t txkey[32];
  int64_t ts_sec;
  int32_t ts_nanos;
  uint32_t addr_off, addr_len, sig_off, sig_len;
} orc_wire_vote;
int orc_wire_decode(const uint8_t* bz, size_t len, uint32_t max_msg_bytes, orc_wire_vote* out);
/* cdc.MarshalBinaryBare(&TxVoteMessage{Tx: vote}); returns length, -1 on an amino time error or cap */
/* cdc.MarshalBinaryBare(TxVote) (= a CommitSig's bytes, types/tx_vote.go:154-159, used by
 * MakeCommit types/vote_set.go:242-259); out == 0: length only; -1 on an amino time error */
int orc_txvote_encode(int64_t height, const uint8_t* txhash, size_t txhash_len, const uint8_t* txkey,
                      int64_t ts_sec, int32_t ts_nanos, const uint8_t* addr, size_t addr_len,
                      const uint8_t* sig, size_t sig_len, uint8_t* out);
int orc_wire_encode(int64_t height, const uint8_t* txhash, size_t txhash_len, const uint8_t* txkey,
                    int64_t ts_sec, int32_t ts_nanos, const uint8_t* addr, size_t addr_len,
                    const uint8_t* sig, size_t sig_len, uint8_t* out, size_t cap);
void orc_wire_prefix(uint8_t disamb[3], uint8_t prefix[4]);
/* CPU baseline: n messages decoded on one thread (status_out [n], out [n]); returns seconds */
double orc_wire_decode_many(const uint8_t* wire, const uint64_t* off, const uint32_t* len, uint32_t n,
                            uint32_t max_msg_bytes, uint8_t* status_out, orc_wire_vote* out);

/* ---- CPU baseline: parallel verify with T threads (T = 1 mirrors checkMaj23Routine). ---- */
/* Verifies n (pub,msg,sig) triples; msgs in an arena with offsets/lengths. Returns seconds. */
double orc_verify_many(const uint8_t* pubs32, const uint32_t* val_idx,
                       const uint8_t* msg_arena, const uint32_t* msg_off, const uint16_t* msg_len,
                       const uint8_t* sigs64, uint32_t n, int threads, uint8_t* out_ok);

#ifdef __cplusplus
}
#endif
#endif
