// txv_device.h — kernel argument blocks and launcher declarations shared by the
// HIP kernels and the host runtime.  Plain structs of device pointers and sizes.
//
// Batch layout in HBM (column-major SoA, stride n_pad = votes rounded up to 64 so a
// wave's lanes read consecutive words of the same field):
//   sig[16][n_pad]      u32  signature bytes 0..63 as little-endian words (R = 0..7, S = 8..15)
//   msg[msg_words][n_pad] u64 SignBytes as big-endian 64-bit words, zero beyond msg_len
//   msg_len[n], val[n] (validator index), flags[n] (TXV_FLAG_*), set[n] (tx-set id)
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#ifndef TXV_VERIFY_BLOCK
#define TXV_VERIFY_BLOCK 512   // 8 waves share one LDS copy of the B table; 2 blocks/CU
#endif

#define TXV_FLAG_PENDING 0x01u   // vote reaches the Verify step (pre-checks passed)
#define TXV_FLAG_SIG64   0x02u   // len(Signature) == 64
#define TXV_FLAG_BADMSG  0x04u   // SignBytes failed (amino time range): never verifies; the
                                 // tally still resolves it against an accepted vote first

struct VerifyArgs {
  uint32_t n, n_pad, msg_words, n_work;   // n_work: entries of order[] (pending votes)
  uint32_t* kbuf;              // [8][n_pad] challenge scalars k (K1a -> K1b)
  const uint32_t* sig;         // [16][n_pad]
  const uint64_t* msg;         // [msg_words][n_pad]
  const uint32_t* msg_len;     // [n]
  const uint32_t* val;         // [n]
  const uint8_t* flags;        // [n]
  const uint32_t* order;       // optional processing order (validator-grouped), may be null
  const uint32_t* pubs_le;     // [n_vals][8]
  const uint8_t* decode_ok;    // [n_vals]
  const uint32_t* atables;     // [slots][kTableWords] (validator v at slot tslot[v])
  const uint32_t* btable;      // [kTableWords]
  uint8_t* ok_out;             // [n]
  uint32_t* park;              // [waves][V-1][32][64] parked points of the multi-vote K1b
  uint32_t lane_votes;         // V: votes per lane sharing one inversion at W >= 8 (2, 4, 8);
                               // 1 = split: K1b stores R' per vote, K1c batch-inverts G per lane
  uint32_t* rpts;              // split mode: [TXV_RPTS_WORDS][n_pad] per work entry: X, Y, Z of R',
                               // then the exclusive prefix product of the lane's Z (K1b -> K1c)
  uint32_t* wctr;              // [8 * 16] chunk counters of the work-stealing K1b (one per XCD
                               // range, 64 B apart), zeroed before each launch
  uint32_t park_waves;         // waves the park buffer holds (V = 8 slots each): caps persistent grids
  uint32_t n_cus;              // CUs of the context's device
  uint32_t fused_k1a;          // TXV_K1B_FUSED: the work-stealing K1b computes the challenges itself (no K1a)
  const uint32_t* tslot;       // [n_vals] table slot of each validator in atables, or null (slot = index)
};

#define TXV_PARK_WORDS 33          // X, Y, prefix product, Z of one parked vote; its vote index + 1
#define TXV_MAX_LANE_VOTES 4
#define TXV_RPTS_WORDS 32

// TxVote.SignBytes on the device (kernels_signbytes.hip): fields in, msg words out
struct SignBytesArgs {
  uint32_t n, n_pad, msg_words, chain_len;
  const int64_t* height;       // [n]
  const int64_t* ts_sec;       // [n]
  const int32_t* ts_nanos;     // [n]
  const uint32_t* txhash_off;  // [n] into txhash
  const uint32_t* txhash_len;  // [n]
  const uint8_t* txhash;       // TxHash arena
  const uint8_t* chain;        // [chain_len]
  const uint32_t* msg_len;     // [n] SignBytes length, 0 = none (nil / amino error); or null:
  const uint8_t* nil;          // then every vote but the nil ones ([n] or null) is encoded
  uint64_t* msg;               // [msg_words][n_pad] out
};

struct SignArgs {
  uint32_t n, n_pad, msg_words, pad0;
  const uint64_t* msg;         // [msg_words][n_pad]
  const uint32_t* msg_len;     // [n]
  const uint32_t* val;         // [n] signer index
  const uint32_t* prefix;      // [n_signers][8]
  const uint32_t* araw;        // [n_signers][8] clamped secret scalar
  const uint32_t* pub;         // [n_signers][8]
  const uint32_t* btable;
  uint32_t* sig;               // [16][n_pad] output
};

// TxVoteMessage wire decode (kernels_wire.hip): statuses are include/txvote.h's TXV_WIRE_*
// (0 ok, 1 too large, 2 amino error, 3 empty/nil).  Output: one 160-byte record per message
// (TXV_WIRE_REC_WORDS u32, written as one contiguous stream), word layout:
//   0 status | 1-2 height | 3-4 ts_sec | 5 ts_nanos | 6 txhash_off | 7 txhash_len | 8 addr_len |
//   9 sig_off | 10 sig_len | 11-18 TxKey | 19-23 address (first 20 bytes) | 24-39 signature (first 64)
// offsets are absolute into `wire`; row bytes beyond a field's length are zero.
#define TXV_WIRE_REC_WORDS 40
#ifndef TXV_WIRE_BLOCK
#define TXV_WIRE_BLOCK 128         // messages per chunk (one block iteration)
#endif
struct WireArgs {
  uint32_t n, max_msg_bytes;
  uint32_t n_chunks, pad0;     // ceil(n / TXV_WIRE_BLOCK)
  const uint64_t* span;        // [n_chunks][2]: 16-aligned start and end of the chunk's message bytes
  uint32_t disamb, prefix;     // amino disambiguation (3 bytes) / prefix (4 bytes), little-endian packed
  const uint8_t* wire;         // messages, padded by >= 128 bytes
  const uint64_t* off;         // [n]
  const uint32_t* len;         // [n]
  uint32_t* rec;               // [n][TXV_WIRE_REC_WORDS]
};

// the raw TxVote columns of a flow slot, written on the device from decoded wire records
struct FlowCols {
  int64_t* height; int64_t* ts_sec; int32_t* ts_nanos;
  uint32_t* th_off; uint32_t* th_len;
  uint8_t* addr; uint32_t* addr_len;    // [n][20]
  uint8_t* sig; uint32_t* sig_len;      // [n][64]
  uint8_t* txkey;                       // [n][32]
};

extern "C" {
hipError_t txv_launch_decode_msgs(const WireArgs* args, uint32_t grid, hipStream_t st);
hipError_t txv_launch_rec_keys(const uint32_t* rec, const uint8_t* wire, uint32_t n, uint8_t* status, uint32_t* keys,
                               uint32_t* sizes, uint32_t* max_hl, hipStream_t st);
hipError_t txv_launch_rec_to_flow(const uint32_t* rec, const uint32_t* list, uint32_t n, const FlowCols* c,
                                  hipStream_t st);
hipError_t txv_launch_rec_to_flow_nil(const uint32_t* rec, const uint8_t* pool_status, uint32_t n, const FlowCols* c,
                                      uint8_t* nil, hipStream_t st);
// w = table window (4: LDS-staged B, 55 KB/point; 8: L2/MALL-resident, 396 KB/point)
hipError_t txv_launch_build_tables(int w, const uint32_t* pubs_le, uint32_t n_points, uint32_t* tables,
                                   uint8_t* decode_ok, uint32_t* addr_words, hipStream_t st);
// the same, point pt's tables written to slot out_slot[pt] of `tables` (decode_ok / addr_words by pt)
hipError_t txv_launch_build_tables_at(int w, const uint32_t* pubs_le, uint32_t n_points, const uint32_t* out_slot,
                                      uint32_t* tables, uint8_t* decode_ok, uint32_t* addr_words, hipStream_t st);
bool txv_verify_windows_supported(int wb, int wa);
hipError_t txv_launch_verify(int wb, int wa, const VerifyArgs* args, uint32_t grid, hipStream_t st);
// the two halves of txv_launch_verify: K1a (challenge), then K1b (+ K1c in split mode)
hipError_t txv_launch_challenge(const VerifyArgs* args, hipStream_t st);
hipError_t txv_launch_scalarmult(int wb, int wa, const VerifyArgs* args, uint32_t grid, hipStream_t st);
hipError_t txv_launch_keygen(const uint32_t* seeds_le, uint32_t n, const uint32_t* btable, uint32_t* scal,
                             uint32_t* araw, uint32_t* prefix, uint32_t* pub, hipStream_t st);
hipError_t txv_launch_sign(const SignArgs* args, hipStream_t st);
hipError_t txv_launch_valu_probe(int op, uint32_t* out, uint32_t blocks, int iters, hipStream_t st);
hipError_t txv_launch_signbytes(const SignBytesArgs* args, hipStream_t st);
bool txv_k1b_fusable(int wb, const VerifyArgs* args);   // the launch takes the work-stealing K1b
hipError_t txv_launch_nil_from_status(const uint8_t* st, uint32_t n, uint8_t* nil, uint32_t or_nil, hipStream_t s);
hipError_t txv_launch_sig_keys(const uint32_t* sig, const uint32_t* sig_len, uint32_t n, uint32_t* keys,
                                hipStream_t st);
hipError_t txv_launch_fe_selftest(const uint32_t* a, const uint32_t* b, uint32_t* out, uint32_t n, int op,
                                  hipStream_t st);
}
