// txv_flow.h — device state and argument blocks of the TxFlow.addVote path on the GPU
// (kernels_flow.hip): routing a batch of TxVotes to their TxVoteSets, the AddVote pre-checks
// and the stake tally (txflow/service.go:192-234, types/vote_set.go:81-166).
//
// Persistent device state of one TxFlow (HBM, survives batches until txv_reset_flow):
//   set table   SetEntry[tab_mask + 1]   TxHash -> dense TxVoteSet id, open addressing.  Ids are
//               handed out in first-seen arrival order, exactly as the sequential
//               `TxVoteSets[vote.TxHash]` creation would number them (service.go:200-209).
//   key slots   u8[max_txs][64]          TxHash bytes of set id s at s * 64 (TxHashes of up to 64
//               + overflow arena          bytes: every SHA-256 upper-hex TxHash); longer ones in
//                                         the overflow arena (key_arena_bytes)
//   per set id  set_entry (table slot), set_txkey [8] u32 (TxKey of the first vote,
//               service.go:201-207), set_sum i64, set_stamp (last batch that ADDED a vote)
//   cells       TallyCell [max_txs * n_vals], 16 B (one line touch per cell access):
//                 cand  (~stamp << 32 | arrival index) of the first verified vote of the (set,
//                       validator) cell in the batch with that stamp: one atomic min per verified
//                       vote, and a stale stamp reads as "none", so it is never cleared
//                 acc   0 or the accepted vote's arena row + 1 (the reference's `votes` map,
//                       vote_set.go:154), written once the batch's crossing step ran
//                 row   the arena row + 1 the running batch's ADDED vote of the cell took
//   arena       [max_accepted] rows, column-major (sig [16][rows] u32, height, ts_sec, ts_nanos,
//               val, seq, TxKey [8][rows]): every accepted vote in full, one row per ADDED vote,
//               rows taken by wave-aggregated atomics as the votes are resolved (the rows of a
//               wave are consecutive, so each column store is one coalesced line per wave; row
//               order carries no meaning -- the readers order by validator)
//   set_cross   [max_txs] arrival index at which the set's stake crossed 2/3 in the batch that
//               last touched it (TXV_NO_CROSS: none): the fired bit of each ADDED vote
//   set_digest  [max_txs][4] the first 16 bytes of SHA-256(TxHash) (whose byte 0 mod G is the
//               set's shard, txv_shard_of): written when the set is created, packed beside its
//               commit bit and sum, so a rank can name another rank's sets from the exchange alone
// The commit bitmap is derived from set_sum on demand (txv_commit_bitmap, the packed state).
//
// gfx950 has 8 XCDs with private L2s: the only hand-off INSIDE a launch is the set-table insert
// of the route kernel, done with write-through (sc1) stores, s_waitcnt vmcnt(0) and a relaxed
// flag store by the creating lane, and sc1 loads by the probing lanes (cdna_hip_programming.md,
// publish/consume recipe).  Every other producer -> consumer pair is separated by a launch.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#include "txv_hash.h"

#define TXV_NO_CROSS 0xFFFFFFFFu
#define TXV_NONE 0xFFFFFFFFu

// per-vote status codes (device copies of include/txvote.h)
#define TXV_S_ADDED 0u
#define TXV_S_DUPLICATE 1u
#define TXV_S_NIL 2u
#define TXV_S_EMPTY_ADDR 3u
#define TXV_S_UNKNOWN_VALIDATOR 4u
#define TXV_S_NONDETERMINISTIC 5u
#define TXV_S_INVALID_SIGNATURE 6u
#define TXV_S_SIGNBYTES 8u
#define TXV_S_PENDING 0xFFu
#define TXV_S_FIRED 0x80u

// FlowCounters.err bits: an infrastructure capacity was exceeded inside the batch (the
// context is poisoned until txv_reset_flow: TXV_ECAPACITY)
#define TXV_FERR_SETS 0x1u      // more TxVoteSets than max_txs
#define TXV_FERR_TABLE 0x2u     // set table full (probe bound)
#define TXV_FERR_KEYS 0x4u      // TxHash overflow key arena full
#define TXV_FERR_ARENA 0x8u     // accepted-vote arena full (max_accepted)
#define TXV_FERR_LOOKBACK 0x10u // the event compaction's look-back timed out (a broken invariant: device error)

struct TallyCell {              // 16 B, see the header comment
  uint64_t cand;
  uint32_t acc;
  uint32_t row;
};

// table entry states
#define TXV_SE_EMPTY 0u
#define TXV_SE_BUSY 1u          // being written by the lane that claimed it
#define TXV_SE_BATCH 2u         // created by the running batch: key bytes in the batch's TxHash arena
#define TXV_SE_KEPT 3u          // key bytes in the persistent key arena

struct SetEntry {               // 32 B; (state, len) and (first, id) are loaded as one 64-bit word each
  uint64_t h;                   // seeded 64-bit hash of the TxHash bytes
  uint32_t state;
  uint32_t len;                 // TxHash length
  uint64_t key_off;             // 1 + offset into the batch arena (BATCH) or the key store (KEPT); 0 = unset
  uint32_t first;               // BATCH: smallest arrival index of the key in the batch
  uint32_t id;                  // dense set id (assigned after the batch's routing step)
};
#define TXV_KEY_SLOT 64u        // key store bytes per set id

// one accepted vote (128 B): what TxVoteSet.votes holds, for MakeCommit / GetVotes
struct AccRow {
  uint32_t sig[16];             // the 64 signature bytes (an accepted vote has exactly 64)
  int64_t height;
  int64_t ts_sec;
  int32_t ts_nanos;
  uint32_t val;                 // validator index (its ValidatorAddress is the registry's)
  uint64_t seq;                 // sequence number of the vote since the last reset
  uint32_t txkey[8];
};

struct FlowCounters {           // device-resident, updated by the kernels
  uint32_t n_sets;              // TxVoteSets so far
  uint32_t arena_used;          // accepted-vote rows in use
  uint32_t err;                 // TXV_FERR_*
  uint32_t n_stamped;           // sets the running batch ADDED a vote to (zeroed by tally_min)
  uint32_t n_digested;          // sets [0, n_digested) have set_digest (computed by the pack's digest pass)
  uint32_t ev_ticket;           // event-compaction tiles taken by the running batch (zeroed by tally_min)
  uint64_t key_used;            // overflow key arena bytes in use
};

struct FlowSummary {            // written to mapped host memory by the last kernel of a batch
  uint32_t n_sets, n_events, arena_used, err;
  uint64_t key_used;
};

struct FlowEvent {              // txv_commit_event (include/txvote.h)
  uint32_t vote_index, tx_index;
  int64_t sum;
};

struct FlowState {
  SetEntry* tab;
  uint32_t tab_mask;
  uint32_t max_txs;
  uint8_t* keys;                // [max_txs][TXV_KEY_SLOT] key slots, then the overflow arena
  uint64_t keys_cap;            // overflow arena bytes
  uint32_t* set_entry;          // [max_txs]
  uint32_t* set_txkey;          // [max_txs][8]
  int64_t* set_sum;             // [max_txs]
  uint32_t* set_stamp;          // [max_txs]
  uint32_t* set_blk;            // [max_txs / 1024 + 2] scan blocks of the stamped-set compaction (large batches)
  uint32_t* set_cross;          // [max_txs]
  uint32_t* set_digest;         // [max_txs][4] SHA-256(TxHash bytes)[0:16]: the set's name in the exchange
  TallyCell* cell;              // [max_txs * n_vals]
  uint32_t* arena_sig;          // [16][max_accepted]
  int64_t* arena_height;        // [max_accepted]
  int64_t* arena_sec;
  int32_t* arena_nanos;
  uint32_t* arena_val;
  uint64_t* arena_seq;
  uint32_t* arena_txkey;        // [8][max_accepted]
  FlowCounters* ctr;
  uint32_t n_vals, max_accepted;
  int64_t quorum;
  const int64_t* power;         // [n_vals]
  const uint32_t* val_addr;     // [n_vals][5] registry addresses (SHA-256(pub)[:20])
  const uint32_t* addr_slots;   // [addr_mask + 1] validator index or TXV_NONE (AddrTable)
  uint32_t addr_mask;
  uint32_t pad0;
  uint64_t hash_seed;           // TxHash hash seed (random per context)
};

// one batch (raw columns as the caller passed them, uploaded; derived columns)
#define TXV_VCODE_EMPTY 0xFFFEu     // empty ValidatorAddress (vote_set.go:97-99)
#define TXV_VCODE_UNKNOWN 0xFFFFu   // GetByAddress found none (vote_set.go:102-106)
struct FlowBatch {
  uint32_t n, n_pad, msg_words, chain_len;
  uint64_t seq_base;            // sequence number of vote 0
  uint32_t stamp;               // this batch's stamp (>= 1, never reused by the context)
  uint32_t pad0;
  const int64_t* height;
  const int64_t* ts_sec;
  const int32_t* ts_nanos;
  const uint32_t* th_off;
  const uint32_t* th_len;
  const uint8_t* th;            // TxHash arena (>= 8 bytes of padding after the last key)
  const uint8_t* addr;          // [n][20]
  const uint32_t* addr_len;
  const uint8_t* sig_raw;       // [n][64]
  const uint32_t* sig_len;
  const uint8_t* nil;           // [n] or null
  const uint8_t* txkey;         // [n][32] or null (zero TxKey)
  const uint16_t* vcode;        // [n] validator index looked up on the host, TXV_VCODE_EMPTY /
                                // TXV_VCODE_UNKNOWN; or null: route_prep looks addr up itself
  // derived
  uint32_t* sig;                // [16][n_pad] column-major signature words (K1a / K1b / compares)
  uint32_t* msg_len;            // [n] SignBytes length (0: nil / amino error)
  uint32_t* val;                // [n] validator index
  uint8_t* flags;               // [n] TXV_FLAG_*
  uint8_t* pre;                 // [n] pre-check status or TXV_S_PENDING
  uint32_t* entry;              // [n] set-table slot (TXV_NONE for nil)
  uint32_t* set;                // [n] set id
  const uint8_t* ok;            // [n] verify verdicts (1 = valid)
  uint8_t* status;              // [n] tally status of pending votes
  uint8_t* ev_flag;             // [n] this vote's ADDED crossed 2/3 in the batch
  uint8_t* mark;                // [n] set by tally_min when a smaller arrival index took this vote's cell
  uint32_t* blk;                // scan scratch: [ceil(n / 1024) + 1]
  uint32_t* stamped;            // [n] ids of the sets this batch ADDED votes to (the crossing step's work list)
  uint64_t* ev_tiles;           // [ceil(n / 1024)] look-back words of the event compaction (tagged with the
                                // stamp, so never cleared)
  // outputs in mapped host memory
  uint8_t* status_host;         // [n]
  FlowEvent* ev_host;           // [n]
  FlowSummary* summary_host;
};

extern "C" {
// the whole AddVote chain of one batch except SignBytes and verify, on two streams:
// prep (pre-checks, validator lookup, signature transpose, SignBytes lengths: everything the
// verify kernels read, nothing keyed by the TxFlow) runs on the verify stream ...
hipError_t txv_flow_prep(const FlowState* fs, const FlowBatch* b, hipStream_t st);
// ... the TxFlow part on the flow stream, in batch order after the previous batch's tally:
// route (set-table find-or-insert of every TxHash) ...
hipError_t txv_flow_route(const FlowState* fs, const FlowBatch* b, hipStream_t st);
// ... new set ids (first-seen compaction) ...
hipError_t txv_flow_new_ids(const FlowState* fs, const FlowBatch* b, hipStream_t st);
// ... then, after K1a/K1b wrote b->ok and the new ids exist: tally, commit events, statuses
hipError_t txv_flow_tally(const FlowState* fs, const FlowBatch* b, uint32_t sets_bound, hipStream_t st);
// forget every TxVoteSet (keep_ids = 0) or empty them keeping their ids (keep_ids = 1)
hipError_t txv_flow_reset(const FlowState* fs, int keep_ids, hipStream_t st);
// cells of the first `cells` (set, validator) pairs: every candidate forgotten (cand = ~0), and
// with clear_acc the accepted votes too
hipError_t txv_flow_init_cells(const FlowState* fs, uint64_t cells, int clear_acc, hipStream_t st);
hipError_t txv_fill64(uint64_t* dst, uint64_t v, uint32_t n, hipStream_t st);
// txkey[i] = the 32 bytes the 64-char upper-hex TxHash of vote i spells (zero for nil votes)
hipError_t txv_txkey_from_hash(const uint8_t* th, const uint32_t* off, const uint8_t* nil, uint32_t n, uint8_t* txkey,
                               hipStream_t st);
// TxHash lookups for the readers: out_id[i] = set id or TXV_NONE
hipError_t txv_flow_lookup(const FlowState* fs, const uint8_t* keys, const uint32_t* off, const uint32_t* len,
                           uint32_t n, uint32_t* out_id, hipStream_t st);
// per set id: sum, TxKey, and the accepted vote of every validator (AccRow, val = TXV_NONE
// for none): out_rows[k * n_vals + v]
hipError_t txv_flow_gather(const FlowState* fs, const uint32_t* ids, uint32_t n, int64_t* out_sum,
                           uint32_t* out_txkey, AccRow* out_rows, hipStream_t st);
// key bytes of set ids (for SaveTx / MakeCommit): out_off/out_len into the key arena
hipError_t txv_flow_keys(const FlowState* fs, const uint32_t* ids, uint32_t n, uint64_t* out_off, uint32_t* out_len,
                         hipStream_t st);
// packed commit state of this shard: [n_sets u32][1 u32][bitmap words][sums i64][digests 16 B]
hipError_t txv_flow_pack(const FlowState* fs, uint32_t* dst, uint32_t bm_words, uint32_t n_cap, hipStream_t st);
// commit bitmap (bit s = set_sum[s] >= quorum) of the first bm_words * 32 set ids
hipError_t txv_flow_bitmap(const FlowState* fs, uint32_t* dst, uint32_t bm_words, hipStream_t st);
}
