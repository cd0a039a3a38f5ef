// txv_tally.h — argument block of the tally kernels (kernels_tally.hip).
//
// Device tally state (persistent across batches, HBM):
//   acc_slot[max_txs * n_vals]  u32  0 = no accepted vote, else arena row + 1
//   arena[max_accepted][16]     u32  accepted signature bytes (for dup/conflict compares)
//   set_sum[max_txs] i64, commit_bitmap[max_txs/32] u32
// Per batch (staged by the host with the votes, set-major):
//   toff[n_touched + 1]   u32  vote range of touched set t in tvote/tval
//   tvote[n_work], tval[n_work]  pending votes grouped by (set, validator), arrival order
//                              inside each group (stable counting sorts on the host)
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#define TXV_ADDED_DEV 0u
#define TXV_DUPLICATE_DEV 1u
#define TXV_ERR_NONDETERMINISTIC_DEV 5u
#define TXV_ERR_INVALID_SIGNATURE_DEV 6u
#define TXV_NO_CROSS 0xFFFFFFFFu

struct TallyArgs {
  uint32_t n, n_pad, n_vals, n_touched;
  int64_t quorum;
  uint32_t arena_base;          // arena rows [arena_base, arena_base + n) belong to this batch
  uint32_t pad0;
  const uint32_t* sig;          // [16][n_pad]
  const uint8_t* ok;            // [n] verify verdicts (1 = valid)
  const uint8_t* pre;           // [n] host pre-check: 0xFF pending, else the final error code
  uint8_t* status;              // [n] out: final code | fired bit (pre is never modified, so a
                                //      staged batch can be re-run)
  const uint32_t* touched;      // [n_touched] set ids present in the batch
  const uint32_t* toff;         // [n_touched + 1]
  const uint32_t* tvote;        // [n_work]
  const uint32_t* tval;         // [n_work]
  uint32_t* ent_vote;           // [n_work] scratch: ADDED votes of set t at toff[t]..
  int64_t* ent_power;           // [n_work]
  uint32_t* ent_val;            // [n_work]
  uint32_t* acc_slot;
  uint32_t* arena;
  const int64_t* power;         // [n_vals]
  int64_t* set_sum;
  uint32_t* commit_bitmap;
  int64_t* t_sum;               // [n_touched] outputs (mapped host memory)
  uint8_t* t_maj;
  uint32_t* t_cross;
  uint8_t* status_host;         // [n] final statuses, mapped host memory (written by K2b)
};

extern "C" hipError_t txv_launch_tally(const TallyArgs* args, hipStream_t st);
extern "C" hipError_t txv_launch_set_votes(const uint32_t* acc_row, uint32_t n_vals, const uint32_t* arena, uint32_t* rows,
                                           uint32_t* sigs, hipStream_t st);
