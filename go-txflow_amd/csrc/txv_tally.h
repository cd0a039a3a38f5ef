// txv_tally.h — argument block of the tally kernels (kernels_tally.hip).
//
// Device tally state (persistent across batches, HBM):
//   acc_slot[max_txs * n_vals]  u32  0 = no accepted vote, else arena index + 1
//   first_tag[max_txs * n_vals] u64  epoch-tagged smallest verified arrival index (atomicMin)
//   arena[max_accepted][16]     u32  accepted signature bytes (for dup/conflict compares)
//   set_sum[max_txs] i64, set_cross[max_txs] u32, commit_bitmap[max_txs/32] u32
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#define TXV_ADDED_DEV 0u
#define TXV_DUPLICATE_DEV 1u
#define TXV_ERR_NONDETERMINISTIC_DEV 5u
#define TXV_ERR_INVALID_SIGNATURE_DEV 6u
#define TXV_NO_CROSS 0xFFFFFFFFu
#define TXV_DEVERR_ARENA_FULL 1u

struct TallyArgs {
  uint32_t n, n_pad, n_vals, epoch_hi;
  int64_t quorum;
  const uint32_t* sig;          // [16][n_pad]
  const uint32_t* set;          // [n]
  const uint32_t* val;          // [n]
  const uint8_t* flags;         // [n]
  const uint8_t* ok;            // [n] verify verdicts
  const uint8_t* pre;           // [n] host pre-check: 0xFF pending, else the final error code
  uint8_t* status;              // [n] out: final code | fired bit (pre is never modified, so a
                                //      staged batch can be re-run)
  uint32_t* acc_slot;
  uint64_t* first_tag;
  uint32_t* arena;
  uint32_t* arena_count;
  uint32_t arena_cap, n_touched;
  uint32_t* error_flags;
  const int64_t* power;         // [n_vals]
  int64_t* set_sum;
  uint32_t* set_cross;
  uint32_t* commit_bitmap;
  const uint32_t* touched;      // [n_touched] set ids present in the batch
  int64_t* t_sum;               // [n_touched] outputs
  uint8_t* t_maj;
  uint32_t* t_cross;
};

extern "C" hipError_t txv_launch_tally(const TallyArgs* args, hipStream_t st);
