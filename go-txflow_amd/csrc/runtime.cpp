// runtime.cpp — host runtime behind include/txvote.h (libtxvote.so).
//
// Responsibilities of the host side:
//   * validator registry: powers, quorum = Total*2/3 + 1 (types/vote_set.go:158) and the
//     address table (ValidatorSet.GetByAddress, ext, called at types/vote_set.go:102), uploaded
//   * the AddVote path (txv_submit_votes / txv_add_votes): copy the caller's raw TxVote columns
//     into pinned memory (or DMA them straight from caller memory registered with
//     txv_host_register) and queue the upload on the copy stream; every decision -- TxHash
//     routing to TxVoteSets (txflow/service.go:200-209), the AddVote pre-checks, SignBytes, the
//     verify, the tally -- is made by the kernel chain of run_slot on the compute stream
//     (kernels_flow.hip, kernels_signbytes.hip, kernels_verify.hip)
//   * the verify-only entry points (txv_verify_batch / txv_verify_bytes) and the signer pack
//     their SignBytes on the host (amino.hpp) into pinned column-major buffers
// Everything numeric about a vote's verdict runs on the GPU; there is no CPU verify path.
#include "../../include/txvote.h"
#include "txv_device.h"
#include "txv_flow.h"
#include "amino.hpp"
#include "host_pack.hpp"
#include "sha2.h"
#include "route.h"

#include <hip/hip_runtime.h>
#include <emmintrin.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cctype>
#include <cstdlib>
#include <sched.h>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <system_error>
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

void txv_sha256_bytes(const uint8_t* p, uint64_t n, uint8_t out[32]);   // SHA-256 on the host (below)

namespace {

// fixed-base table words per point for window W: ceil(256/W) positions x (2^(W-1)+1) entries x 32
// (one 128-byte half-Niels entry each, ge.h); W = 21 is the 12-position long-top layout
// (ed25519_dev.h Tab<21>: 11 x (2^20+1) + 2^21+9 entries)
inline size_t table_words(int w) {
  if (w == 21) return ((size_t)11 * ((1u << 20) + 1) + (1u << 21) + 9) * 32;
  return (size_t)((256 + w - 1) / w) * ((1u << (w - 1)) + 1) * 32;
}
constexpr uint32_t kTableWords4 = 64 * 9 * 32;
// 21 only on request (TXV_CFG_WINDOW): 1.70 GB of tables per validator, against the radix-2^26
// base table (select_window)
inline bool valid_window(int w) {
  return w == 4 || w == 8 || w == 10 || w == 12 || w == 14 || w == 16 || w == 18 || w == 20 || w == 21;
}
// TXV_K1A_ON_KEY_STREAM=1 runs K1a on the key stream, beside the previous batch's K1b (its 99
// VGPRs do not fit beside two K1b waves, so it mostly fills K1b's tail): measured 614-621 vs
// 608M votes/s (within box noise, profiles/r02/ab), while the two kernels' overlapping durations
// no longer add up to the verify time; off: K1a then K1b on the verify stream
#ifndef TXV_K1A_ON_KEY_STREAM
#define TXV_K1A_ON_KEY_STREAM 0
#endif
constexpr uint32_t kStagedSlots = 4;   // 0-3 staged (0-2 also the submit ring)
constexpr uint32_t kSubmitRing = 4;    // txv_submit_votes batches in flight
constexpr uint32_t kVcodeEmpty = TXV_VCODE_EMPTY, kVcodeUnknown = TXV_VCODE_UNKNOWN;   // txv_flow.h
// batches from which the pack threads look validators up (the link time the 18 bytes per vote
// save outweighs the host work there: C2's 1M-vote batches 593.4M vs 518.3M votes/s end to end,
// profiles/r04/hval1; C5's 64k-vote batches keep the device lookup)
constexpr uint32_t kHostValMin = 1u << 18;
constexpr uint32_t kSignerSlot = 4, kVerifySlot = 5, kIngestSlot = 6;   // signer, verify-only, wire ingest ring (6-8)
constexpr uint32_t kIngestRing = 3;
constexpr uint32_t kRouteSlot = kIngestSlot + kIngestRing;   // txv_route_admitted's columns
constexpr uint32_t kSlots = kRouteSlot + 1;

struct Slot {
  uint32_t cap = 0, n = 0, n_pad = 0, msg_words = 0, msg_cap_words = 0;
  bool staged = false, ran = false;
  // device: the verify kernels' columns (both paths)
  uint32_t* d_sig = nullptr; uint64_t* d_msg = nullptr; uint32_t* d_msg_len = nullptr;
  uint32_t* d_val = nullptr; uint32_t* d_set = nullptr; uint8_t* d_flags = nullptr;
  uint8_t* d_status = nullptr; uint8_t* d_ok = nullptr; uint8_t* d_pre = nullptr;
  uint32_t* d_kbuf = nullptr; uint32_t* d_rpts = nullptr; uint32_t* d_order = nullptr; uint32_t* h_order = nullptr;
  uint32_t n_work = 0;
  // pinned host (verify-only paths: host-packed columns)
  uint32_t* h_sig = nullptr; uint64_t* h_msg = nullptr; uint32_t* h_msg_len = nullptr;
  uint32_t* h_val = nullptr; uint32_t* h_set = nullptr; uint8_t* h_flags = nullptr; uint8_t* h_status = nullptr;
  std::vector<uint8_t> tmp_msg;   // SignBytes arena (verify-only paths)
  std::vector<size_t> tmp_off;
  // raw TxVote columns (the AddVote path uploads them as the caller passed them; the signer
  // uses height .. TxHash arena for its device SignBytes): pinned staging + device copies
  int64_t *h_fh = nullptr, *h_fs = nullptr, *d_fh = nullptr, *d_fs = nullptr;     // height, ts_sec
  int32_t *h_fn = nullptr, *d_fn = nullptr;                                        // ts_nanos
  uint32_t *h_fo = nullptr, *h_fl = nullptr, *d_fo = nullptr, *d_fl = nullptr;     // txhash off / len
  uint8_t *h_arena = nullptr, *d_arena_th = nullptr;                               // TxHash arena
  size_t arena_cap = 0;
  uint64_t arena_end = 0;          // the staged batch's TxHash arena extent
  uint32_t flow_cap = 0;           // capacity of the AddVote-only buffers below
  uint8_t *h_addr = nullptr, *d_addr = nullptr;            // [n][20]
  uint32_t *h_addr_len = nullptr, *d_addr_len = nullptr;
  uint8_t *h_sigraw = nullptr, *d_sigraw = nullptr;        // [n][64]
  uint32_t *h_sig_len = nullptr, *d_sig_len = nullptr;
  uint8_t *h_nil = nullptr, *d_nil = nullptr;
  uint8_t *h_txkey = nullptr, *d_txkey = nullptr;          // [n][32]
  uint16_t *h_vcode = nullptr, *d_vcode = nullptr;         // [n] validator index / kVcode* (host lookup)
  bool has_nil = false, has_txkey = false, host_val = false;
  // uniform columns (and a TxKey column spelled by the TxHashes) filled on the device at the next
  // run_slot, on the key stream, instead of on the copy stream at staging (stage_add)
  uint32_t fill_mask = 0;
  int64_t fill_h = 0, fill_s = 0;
  uint32_t fill_hl = 0, fill_al = 0, fill_sl = 0;
  bool fill_key = false;
  bool msg_on_device = false;      // the signer's SignBytes are built by txv_k_signbytes
  uint64_t seq_base = 0;
  uint32_t stamp = 0;              // batch stamp of the staged batch
  uint64_t run_seq = 0;            // txv_ctx::run_seq of the slot's last run (orders its summary)
  uint64_t counted = 0;            // votes of this slot's unfetched runs, included in txv_ctx::unfetched
  // AddVote derived columns and scan scratch
  uint32_t *d_entry = nullptr, *d_blk = nullptr;
  uint8_t* d_ev_flag = nullptr;
  uint8_t* d_mark = nullptr;
  uint32_t* d_stamped = nullptr;   // the batch's stamped set ids (tally_resolve -> tally_cross)
  uint64_t* d_ev_tiles = nullptr;  // look-back words of the event compaction (stamp-tagged: zeroed per tag cycle)
  uint32_t ev_tiles_n = 0;
  // results, written by the kernels straight into mapped host memory (m_* = device views)
  uint8_t* h_out = nullptr; uint8_t* m_out = nullptr;
  FlowEvent* h_ev = nullptr; FlowEvent* m_ev = nullptr;
  FlowSummary* h_sum = nullptr; FlowSummary* m_sum = nullptr;
  // copy stream: 3 upload done; key stream: 0 prep start, 8 prep + SignBytes done (K1a starts),
  // 1 K1a done; verify stream: 7 K1b start, 2 verify done; flow stream: 4 results in host memory
  // (+ commit sink), 5 tallied, 6 set keying done
  hipEvent_t ev[9] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  bool launched = false;           // a chain was enqueued on this slot (its ev[4] marks the end)
  uint32_t* sink = nullptr;        // txv_set_commit_sink: packed commit state after each batch of this slot
  uint32_t sink_cap = 0;
  uint64_t ticket = 0;    // txv_submit_votes ticket in flight on this slot (0 = none)
};

}  // namespace

// The last error message.  Threads holding c->mu (submit / wait, decode) and txv_sig_keys (its
// own pk_mu) may fail at the same time, so the string has a lock of its own; txv_last_error
// hands out a per-thread copy.
struct ErrMsg {
  std::mutex m;
  std::string s;
  ErrMsg& operator=(std::string v) {
    std::lock_guard<std::mutex> g(m);
    s = std::move(v);
    return *this;
  }
  const char* copy() {
    thread_local std::string t;
    std::lock_guard<std::mutex> g(m);
    t = s;
    return t.c_str();
  }
};

struct txv_ctx {
  txv_config cfg{};
  int device = 0;
  int n_cus = 256;
  hipStream_t stream = nullptr;        // flow: TxFlow keying + tally kernels, resets, readers (batch order)
  hipStream_t vstream = nullptr;       // verify: prep + K1a/K1b (batch k+1 verifies while batch k tallies)
  hipStream_t copy_stream = nullptr;   // batch uploads, so batch k+1's H2D overlaps batch k's kernels
  hipStream_t key_stream = nullptr;    // txv_sig_keys (pool ingest), wire decode, and each batch's prep + SignBytes
  hipEvent_t tally_ev = nullptr;        // TXV_K1B_AFTER_TALLY: the newest batch's tally end (flow stream)
  bool tally_ev_set = false;
  hipEvent_t vend_ev[4] = {};           // TXV_PREP_AFTER_K1B: the last batches' K1b ends (verify stream)
  uint64_t vend_n = 0;
  uint64_t next_ticket = 1;            // txv_submit_votes ring over slots 0 .. kSubmitRing - 1
  ErrMsg err;
  std::mutex mu;
  // validator registry
  uint32_t n_vals = 0;
  std::vector<uint8_t> pubs, addrs, decode_ok;
  std::vector<int64_t> powers;
  int64_t total = 0, quorum = 0;
  std::string chain;
  uint8_t* d_chain = nullptr; uint32_t d_chain_cap = 0;             // chain id for txv_k_signbytes
  uint8_t* d_chain_sign = nullptr; uint32_t d_chain_sign_cap = 0;   // txv_sign_votes' chain id
  std::unordered_map<std::string, uint32_t> addr_index;
  txv_host::AddrTable addr_tab;    // same map, lock-free reads for the parallel pack
  uint32_t* d_pubs = nullptr; uint8_t* d_decode_ok = nullptr; uint32_t* d_atables = nullptr;
  uint32_t* d_addr = nullptr; int64_t* d_power = nullptr;
  uint32_t* d_btable = nullptr;    // B table for the verify window tab_w
  uint32_t* d_btable4 = nullptr;   // radix-16 B table (keygen / sign)
  uint32_t* d_btable8 = nullptr;   // B table for window btable_w (>= 8)
  int btable_w = 0;
  int cfg_w = 0;                   // requested window, 0 = auto (largest that fits the budget)
  int tab_w = 0;                   // window of the current validator tables
  int cfg_bw = 0;                  // requested base-point window, 0 = auto
  int b_w = 0;                     // base-point window of the verify kernel (>= tab_w)
  uint32_t* d_btable_wide = nullptr;   // base-point table for b_w > tab_w (gigabytes at b_w >= 22)
  int btable_wide_w = 0;
  uint32_t lane_votes = 4;         // K1b votes per lane (one shared inversion)
  bool lane_auto = true;           // no configured V: 8 for batches that still give >= 1.5 waves/SIMD
  uint32_t* d_park = nullptr;      // K1b parked points: [wave][V][33][64]
  uint32_t* d_wctr = nullptr;      // chunk counters of the work-stealing K1b
  // the validator tables as a pool of per-key slots: a new validator set builds (K0) only the
  // keys no slot holds; validator v's tables are at slot vslot[v] (d_vslot, VerifyArgs.tslot)
  uint32_t tab_slots = 0;              // slots allocated in d_atables
  int pool_w = 0;                      // window of the pool's tables
  std::vector<std::string> slot_key;   // key each slot holds ("" = empty)
  std::vector<uint8_t> slot_ok;        // its decode flag
  std::vector<uint8_t> slot_addr;      // [slot][20] its address
  std::vector<uint64_t> slot_gen;      // last validator set that used the slot (eviction order)
  uint64_t set_gen = 0;
  std::vector<uint32_t> vslot;         // validator index -> slot
  uint32_t* d_vslot = nullptr;
  uint32_t tables_built = 0;           // keys K0 built in the last txv_set_validators
  size_t park_words = 0;
  // scratch registry for caller-supplied keys (txv_verify_batch with pubs32)
  uint32_t tmp_cap = 0;
  int tmp_w = 0;
  uint32_t* d_tmp_pubs = nullptr; uint8_t* d_tmp_ok = nullptr; uint32_t* d_tmp_tables = nullptr; uint32_t* d_tmp_addr = nullptr;
  std::unique_ptr<txv_host::WorkerPool> pool;   // host pack threads
  bool profile_host = false;                    // TXV_PROFILE_HOST
  bool uniform_cols = true;                     // uniform columns filled on the device (TXV_UNIFORM_COLS=0: off)
  bool derive_txkey = true;                     // TxKey decoded from TxHash on the device when it spells it (TXV_DERIVE_TXKEY=0: off)
  int host_val = -1;                            // validator lookup on the host pack threads: 1 always, 0 never
                                                // (TXV_HOST_VAL), -1 for batches of >= kHostValMin votes
  uint64_t staged_bytes = 0;                    // host bytes the last staged batch moved over PCIe
  // TxFlow state on the device (txv_flow.h): set table, key arena, per-set arrays, cells,
  // accepted-vote arena, counters
  SetEntry* d_tab = nullptr; uint32_t tab_mask = 0;
  uint8_t* d_keys = nullptr; uint64_t keys_cap = 0;
  uint32_t *d_set_entry = nullptr, *d_set_txkey = nullptr, *d_set_stamp = nullptr, *d_set_cross = nullptr, *d_bitmap = nullptr;
  uint32_t* d_set_blk = nullptr;   // scan blocks over the set ids (the stamped-set compaction of large batches)
  uint32_t* d_set_digest = nullptr;   // [max_txs][4] SHA-256(TxHash)[0:16]
  int64_t* d_set_sum = nullptr;
  TallyCell* d_cells = nullptr;
  uint32_t *d_arena_sig = nullptr, *d_arena_nanos = nullptr, *d_arena_val = nullptr, *d_arena_txkey = nullptr;
  int64_t *d_arena_height = nullptr, *d_arena_sec = nullptr;
  uint64_t* d_arena_seq = nullptr;
  uint32_t stamp = 0;               // last batch stamp handed out (never reused by the context)
  FlowCounters* d_ctr = nullptr;
  uint32_t* d_addr_slots = nullptr; uint32_t addr_mask = 0;
  uint32_t max_accepted = 0;        // accepted-vote rows (AccRow) of the arena
  uint64_t hash_seed = 0;           // TxHash hash seed (random per context)
  uint64_t seq_next = 0;            // sequence number of the next submitted vote
  uint32_t n_sets_host = 0;         // TxVoteSets as of the newest run whose results were fetched
  uint64_t run_seq = 0;             // runs handed out (run_slot), in flow-stream order
  uint64_t sets_seq = 0;            // run_seq n_sets_host belongs to (older summaries are not applied)
  uint64_t unfetched = 0;           // votes of batches run but not fetched yet (each may add sets)
  uint32_t poisoned = 0;            // TXV_FERR_* seen: every AddVote call fails until txv_reset_flow
  // caller memory registered with txv_host_register (DMA'd without a staging copy)
  std::vector<std::pair<uintptr_t, uint64_t>> registered;
  std::mutex reg_mu;               // `registered` is changed under mu and reg_mu: read under either (the
                                   // pool's uploads check it under reg_mu, off the context's lock)
  // reader scratch (lookups / gathers)
  uint8_t* d_q = nullptr; uint64_t q_cap = 0;
  // signer slots (load generator)
  uint32_t n_signers = 0;
  uint32_t *d_sk_scal = nullptr, *d_sk_araw = nullptr, *d_sk_prefix = nullptr, *d_sk_pub = nullptr;
  Slot slots[kSlots];
  // txv_route_admitted scratch (kernels_route.hip): per-vote shard, per-wave counts / bytes, per
  // shard longest TxHash and totals, the metas in mapped memory; route_mu serialises route calls
  std::mutex route_mu;
  uint32_t route_n_cap = 0, route_w_cap = 0;
  uint8_t* d_rshard = nullptr;
  uint32_t *d_rw = nullptr, *d_rmax = nullptr;
  uint64_t* d_rtot = nullptr;
  txv_route_meta *h_rmeta = nullptr, *m_rmeta = nullptr;
  hipEvent_t route_ev = nullptr;
  // txv_sig_keys scratch: signatures [n][16] u32, lengths, keys [n][8] u32
  uint32_t pk_cap = 0;
  std::mutex pk_mu;                  // txv_sig_keys' buffers (not c->mu: CheckTx's keys run beside txv_submit_votes)
  uint32_t *d_pk_sig = nullptr, *d_pk_len = nullptr, *d_pk_keys = nullptr;
  hipEvent_t pk_ev = nullptr;        // the keys' read-back on the key stream has landed
  uint32_t *h_pk_sig = nullptr, *h_pk_len = nullptr, *h_pk_keys = nullptr;
  // txv_decode_* (TxVoteMessage wire decode): staged messages, packed outputs (one D2H copy)
  uint32_t wd_n = 0, wd_cap = 0;
  uint64_t wd_bytes = 0, wd_bytes_cap = 0;
  bool wd_ran = false;
  uint8_t *d_wd_wire = nullptr, *h_wd_wire = nullptr;
  uint64_t *d_wd_off = nullptr, *h_wd_off = nullptr;
  uint32_t *d_wd_len = nullptr, *h_wd_len = nullptr;
  uint8_t *d_wd_out = nullptr, *h_wd_out = nullptr;
  uint64_t *d_wd_span = nullptr, *h_wd_span = nullptr;   // [chunks][2] byte span of each 128-message chunk
  hipEvent_t wd_ev[2] = {nullptr, nullptr};
  // txv_ingest_decode / _admit / _wait (wire bytes -> pool -> TxFlow, device-resident): a ring of
  // three batches (slots kIngestSlot + 0..2), each with its own offsets, decode records (they stay
  // in HBM until the admitted votes' columns are built from them), per-message status / pool key /
  // TxVote.Size, the longest TxHash and the admitted messages' indices
  struct Ingest {
    uint32_t cap = 0;
    uint64_t *d_off = nullptr, *h_off = nullptr;
    uint32_t *d_len = nullptr, *h_len = nullptr;
    uint8_t* d_rec = nullptr;
    uint64_t *d_span = nullptr, *h_span = nullptr;
    uint8_t *d_status = nullptr, *h_status = nullptr;
    uint32_t *d_keys = nullptr, *h_keys = nullptr, *d_sizes = nullptr, *h_sizes = nullptr;
    uint32_t *d_list = nullptr, *h_list = nullptr, *d_max = nullptr, *h_max = nullptr;
    uint8_t* d_pstat = nullptr;    // the pool's device statuses of the batch (the early TxFlow chain's nil column)
    hipEvent_t kev = nullptr;      // statuses (and, for a host-path admission, keys and sizes) are back in pinned memory
    hipEvent_t uev = nullptr;      // the batch's uploads have landed (the decode kernels' stream waits for it)
    uint64_t ticket = 0;           // the batch in this slot (0 = free); guarded by mu
    int phase = 0;                 // 0 free, 1 decoded (keys in flight), 3 CheckTx submitted to the device
                                   // (pool_ticket), 2 admitted (TxFlow chain enqueued)
    uint64_t pool_ticket = 0;      // phase 3: the pool's ticket (txv_pool_check_wait) of its decisions
    txv_pool* pool = nullptr;      // the pool the batch is checked against
    uint32_t n = 0, n_adm = 0;     // messages of the batch; votes the pool admitted (h_list)
    uint32_t max_len = 0;          // the longest message: bounds every TxHash (SignBytes column words)
    bool early = false;            // TxFlow chain enqueued over all n messages behind the device CheckTx
    uint64_t wire_bytes = 0;       // bounds the decoded votes' summed TxVote.Size()
    int flow_err = 0;              // the admitted votes' AddVote chain could not be enqueued
    std::string flow_msg;
  } ing[kIngestRing];
  std::mutex sub_mu;               // txv_submit_votes / txv_submit_checked one at a time (the latter stages,
                                   // takes the pool's lock, then runs: no other submit in between)
  std::mutex ing_dec_mu;           // decodes one at a time (they hand out the tickets)
  std::mutex ing_adm_mu;           // admissions one at a time, in ticket order: pool order = TxFlow order
  std::mutex ing_fin_mu;           // the admissions' second halves (ingest_admit_finish), in ticket order
  uint64_t ing_next = 1;           // next ticket to decode; guarded by mu
  uint64_t ing_admit_next = 1;     // next ticket to admit (submit half); guarded by mu
};

// TXV_PROFILE_SLOW=1 (debugging aid): every HIP call made through HIP_TRY that takes longer than
// 1 ms on the host is reported on stderr with its start on the monotonic clock
inline bool txv_profile_slow() {
  static const bool on = getenv("TXV_PROFILE_SLOW") && atoi(getenv("TXV_PROFILE_SLOW")) == 1;
  return on;
}
inline void txv_slow_report(const char* what, std::chrono::steady_clock::time_point t0) {
  const auto t1 = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  if (ms > 1.0)
    fprintf(stderr, "[txv slow] @%.4f %.3fms %s\n", std::chrono::duration<double>(t0.time_since_epoch()).count(), ms, what);
}

#define HIP_TRY(ctx, x)                                                                    \
  do {                                                                                     \
    const bool sl_ = txv_profile_slow();                                                   \
    const auto t0_ = sl_ ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{}; \
    hipError_t e_ = (x);                                                                   \
    if (sl_) txv_slow_report(#x, t0_);                                                     \
    if (e_ != hipSuccess) {                                                                \
      (ctx)->err = std::string(#x) + ": " + hipGetErrorString(e_);                       \
      return TXV_EDEVICE;                                                                  \
    }                                                                                      \
  } while (0)

namespace {

// TXV_PROFILE_HOST=1: per-phase wall times of the host pack on stderr
struct HostTimer {
  bool on;
  std::chrono::steady_clock::time_point t;
  std::string line;
  explicit HostTimer(bool o) : on(o), t(std::chrono::steady_clock::now()) {
    if (on) {   // the start on the monotonic clock (Python's time.perf_counter), for traces
      char b[48];
      snprintf(b, sizeof b, " @%.4f", std::chrono::duration<double>(t.time_since_epoch()).count());
      line = b;
    }
  }
  void mark(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    char b[64];
    snprintf(b, sizeof b, " %s=%.3fms", what, std::chrono::duration<double, std::milli>(now - t).count());
    line += b;
    t = now;
  }
  ~HostTimer() { if (on && line.find('=') != std::string::npos) fprintf(stderr, "[txv host]%s\n", line.c_str()); }
};

template <typename T>
int dalloc(txv_ctx* c, T** p, size_t count) {
  if (*p) { (void)hipFree(*p); *p = nullptr; }
  if (!count) return TXV_OK;
  HIP_TRY(c, hipMalloc((void**)p, count * sizeof(T)));
  return TXV_OK;
}
template <typename T>
int halloc(txv_ctx* c, T** p, size_t count, unsigned flags = hipHostMallocDefault) {
  if (*p) { (void)hipHostFree(*p); *p = nullptr; }
  if (!count) return TXV_OK;
  HIP_TRY(c, hipHostMalloc((void**)p, count * sizeof(T), flags));
  return TXV_OK;
}
// host buffer the kernels write into directly over PCIe (results: no D2H copy to schedule)
template <typename T>
int halloc_mapped(txv_ctx* c, T** p, T** dev, size_t count) {
  int r = halloc(c, p, count, hipHostMallocMapped);
  if (r) return r;
  *dev = nullptr;
  if (*p) HIP_TRY(c, hipHostGetDevicePointer((void**)dev, *p, 0));
  return TXV_OK;
}
template <typename T> void dfree(T*& p) { if (p) { (void)hipFree(p); p = nullptr; } }
template <typename T> void hfree(T*& p) { if (p) { (void)hipHostFree(p); p = nullptr; } }

inline uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
inline uint64_t be64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return v;
}

int ensure_slot(txv_ctx* c, Slot& s, uint32_t n, uint32_t msg_words) {
  const uint32_t need = std::max<uint32_t>(n, 64);
  if (s.cap < need || s.msg_cap_words < msg_words) {
    const uint32_t cap = std::max(need, s.cap);
    const uint32_t mw = std::max(msg_words, s.msg_cap_words);
    const size_t npad = (cap + 63) / 64 * 64;
    int r;
    if ((r = dalloc(c, &s.d_sig, 16 * npad)) || (r = dalloc(c, &s.d_msg, (size_t)mw * npad)) ||
        (r = dalloc(c, &s.d_msg_len, npad)) || (r = dalloc(c, &s.d_val, npad)) || (r = dalloc(c, &s.d_set, npad)) ||
        (r = dalloc(c, &s.d_flags, npad)) || (r = dalloc(c, &s.d_status, npad)) || (r = dalloc(c, &s.d_ok, npad)) ||
        (r = dalloc(c, &s.d_pre, npad)) || (r = dalloc(c, &s.d_kbuf, 8 * npad)) ||
        ((c->lane_votes == 1 || c->lane_auto) && (r = dalloc(c, &s.d_rpts, (size_t)TXV_RPTS_WORDS * npad))) ||
        (r = dalloc(c, &s.d_order, npad)) || (r = halloc(c, &s.h_order, npad)) ||
        (r = halloc(c, &s.h_sig, 16 * npad)) || (r = halloc(c, &s.h_msg, (size_t)mw * npad)) ||
        (r = halloc(c, &s.h_msg_len, npad)) || (r = halloc(c, &s.h_val, npad)) || (r = halloc(c, &s.h_set, npad)) ||
        (r = halloc(c, &s.h_flags, npad)) || (r = halloc(c, &s.h_status, npad)) ||
        (r = halloc_mapped(c, &s.h_out, &s.m_out, npad)) ||
        (r = halloc(c, &s.h_fh, npad)) || (r = halloc(c, &s.h_fs, npad)) || (r = halloc(c, &s.h_fn, npad)) ||
        (r = halloc(c, &s.h_fo, npad)) || (r = halloc(c, &s.h_fl, npad)) || (r = dalloc(c, &s.d_fh, npad)) ||
        (r = dalloc(c, &s.d_fs, npad)) || (r = dalloc(c, &s.d_fn, npad)) || (r = dalloc(c, &s.d_fo, npad)) ||
        (r = dalloc(c, &s.d_fl, npad)))
      return r;
    s.cap = cap;
    s.msg_cap_words = mw;
  }
  if (!s.ev[0])
    for (auto& e : s.ev) HIP_TRY(c, hipEventCreate(&e));
  return TXV_OK;
}

// the AddVote path's raw columns, derived columns and mapped outputs for n votes
int ensure_flow_slot(txv_ctx* c, Slot& s, uint32_t n) {
  const uint32_t need = std::max<uint32_t>(n, 64);
  if (s.flow_cap >= need) return TXV_OK;
  const uint32_t cap = std::max(need, s.flow_cap);
  const size_t npad = (cap + 63) / 64 * 64;
  const size_t nblk = (npad + 1023) / 1024 + 1;
  int r;
  if ((r = halloc(c, &s.h_addr, 20 * npad)) || (r = dalloc(c, &s.d_addr, 20 * npad)) ||
      (r = halloc(c, &s.h_addr_len, npad)) || (r = dalloc(c, &s.d_addr_len, npad)) ||
      (r = halloc(c, &s.h_sigraw, 64 * npad)) || (r = dalloc(c, &s.d_sigraw, 64 * npad)) ||
      (r = halloc(c, &s.h_sig_len, npad)) || (r = dalloc(c, &s.d_sig_len, npad)) ||
      (r = halloc(c, &s.h_nil, npad)) || (r = dalloc(c, &s.d_nil, npad)) ||
      (r = halloc(c, &s.h_txkey, 32 * npad)) || (r = dalloc(c, &s.d_txkey, 32 * npad)) ||
      (r = halloc(c, &s.h_vcode, npad)) || (r = dalloc(c, &s.d_vcode, npad)) ||
      (r = dalloc(c, &s.d_entry, npad)) || (r = dalloc(c, &s.d_blk, nblk)) ||
      (r = dalloc(c, &s.d_ev_flag, npad)) || (r = dalloc(c, &s.d_mark, npad)) || (r = dalloc(c, &s.d_stamped, npad)) || (r = halloc_mapped(c, &s.h_ev, &s.m_ev, npad)) ||
      (r = halloc_mapped(c, &s.h_sum, &s.m_sum, 1)) || (r = dalloc(c, &s.d_ev_tiles, nblk)))
    return r;
  HIP_TRY(c, hipMemset(s.d_ev_tiles, 0, nblk * sizeof(uint64_t)));   // epoch 0: no stamp matches
  s.ev_tiles_n = (uint32_t)nblk;
  s.flow_cap = cap;
  return TXV_OK;
}

FlowState flow_state(const txv_ctx* c) {
  FlowState f{};
  f.tab = c->d_tab; f.tab_mask = c->tab_mask; f.max_txs = c->cfg.max_txs;
  f.keys = c->d_keys; f.keys_cap = c->keys_cap;
  f.set_entry = c->d_set_entry; f.set_txkey = c->d_set_txkey; f.set_sum = c->d_set_sum; f.set_stamp = c->d_set_stamp; f.set_digest = c->d_set_digest;
  f.set_blk = c->d_set_blk;
  f.cell = c->d_cells; f.set_cross = c->d_set_cross;
  f.arena_sig = c->d_arena_sig; f.arena_height = c->d_arena_height; f.arena_sec = c->d_arena_sec;
  f.arena_nanos = reinterpret_cast<int32_t*>(c->d_arena_nanos); f.arena_val = c->d_arena_val;
  f.arena_seq = c->d_arena_seq; f.arena_txkey = c->d_arena_txkey;
  f.ctr = c->d_ctr; f.n_vals = c->n_vals; f.max_accepted = c->max_accepted; f.quorum = c->quorum;
  f.power = c->d_power; f.val_addr = c->d_addr; f.addr_slots = c->d_addr_slots; f.addr_mask = c->addr_mask;
  f.hash_seed = c->hash_seed;
  return f;
}

// device TxFlow state sized for the registry: cells are max_txs x
// n_vals, the accepted-vote arena holds max_accepted rows (default: one per cell, capped at
// 2^26 rows = 8 GiB), the set table has >= 2 (max_txs + max_batch) slots
int alloc_tally(txv_ctx* c) {
  const uint64_t nv = std::max<uint32_t>(c->n_vals, 1);
  const uint64_t cells = (uint64_t)c->cfg.max_txs * nv;
  c->max_accepted = c->cfg.max_accepted ? c->cfg.max_accepted : (uint32_t)std::min<uint64_t>(cells, 1u << 26);
  uint64_t tab = 1024;
  while (tab < 2 * ((uint64_t)c->cfg.max_txs + c->cfg.max_batch)) tab *= 2;
  c->tab_mask = (uint32_t)(tab - 1);
  // key store: a 64-byte slot per set id, then the overflow arena for longer TxHashes
  c->keys_cap = c->cfg.key_arena_bytes ? c->cfg.key_arena_bytes : std::max<uint64_t>((uint64_t)c->cfg.max_txs * 16, 1u << 20);
  int r;
  const size_t M = c->max_accepted;
  if ((r = dalloc(c, &c->d_cells, cells)) || (r = dalloc(c, &c->d_set_cross, c->cfg.max_txs)) ||
      (r = dalloc(c, &c->d_arena_sig, 16 * M)) || (r = dalloc(c, &c->d_arena_height, M)) ||
      (r = dalloc(c, &c->d_arena_sec, M)) || (r = dalloc(c, &c->d_arena_nanos, M)) || (r = dalloc(c, &c->d_arena_val, M)) ||
      (r = dalloc(c, &c->d_arena_seq, M)) || (r = dalloc(c, &c->d_arena_txkey, 8 * M)) ||
      (r = dalloc(c, &c->d_set_sum, c->cfg.max_txs)) ||
      (r = dalloc(c, &c->d_set_stamp, c->cfg.max_txs)) || (r = dalloc(c, &c->d_set_blk, (size_t)c->cfg.max_txs / 1024 + 2)) || (r = dalloc(c, &c->d_set_entry, c->cfg.max_txs)) ||
      (r = dalloc(c, &c->d_set_digest, (size_t)c->cfg.max_txs * 4)) ||
      (r = dalloc(c, &c->d_set_txkey, (size_t)c->cfg.max_txs * 8)) ||
      (r = dalloc(c, &c->d_bitmap, (c->cfg.max_txs + 31) / 32)) || (r = dalloc(c, &c->d_tab, tab)) ||
      (r = dalloc(c, &c->d_keys, (uint64_t)c->cfg.max_txs * TXV_KEY_SLOT + c->keys_cap)) || (r = dalloc(c, &c->d_ctr, 1)))
    return r;
  {
    const FlowState fs = flow_state(c);
    HIP_TRY(c, txv_flow_init_cells(&fs, cells, 1, c->stream));   // no candidate, no accepted vote
  }
  HIP_TRY(c, hipMemsetAsync(c->d_set_sum, 0, (size_t)c->cfg.max_txs * 8, c->stream));
  HIP_TRY(c, hipMemsetAsync(c->d_set_stamp, 0, (size_t)c->cfg.max_txs * 4, c->stream));
  HIP_TRY(c, hipMemsetAsync(c->d_tab, 0, tab * sizeof(SetEntry), c->stream));
  c->stamp = 0;
  HIP_TRY(c, hipMemsetAsync(c->d_ctr, 0, sizeof(FlowCounters), c->stream));
  c->seq_next = 0;
  c->n_sets_host = 0;
  c->sets_seq = c->run_seq;   // summaries of earlier runs describe the old state
  c->poisoned = 0;
  return TXV_OK;
}

// empty every TxVoteSet (keep_ids) or forget them (txv_reset_flow), on the compute stream
// after every batch already submitted
int reset_tally(txv_ctx* c, bool keep_ids = false) {
  if (c->poisoned && !keep_ids) {   // a capacity overflow left partial state: clear everything
    const uint64_t cells = (uint64_t)c->cfg.max_txs * std::max<uint32_t>(c->n_vals, 1);
    {
      const FlowState fs = flow_state(c);
      HIP_TRY(c, txv_flow_init_cells(&fs, cells, 1, c->stream));
    }
    HIP_TRY(c, hipMemsetAsync(c->d_set_sum, 0, (size_t)c->cfg.max_txs * 8, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->d_tab, 0, ((size_t)c->tab_mask + 1) * sizeof(SetEntry), c->stream));
    HIP_TRY(c, hipMemsetAsync(c->d_ctr, 0, sizeof(FlowCounters), c->stream));
    c->poisoned = 0;
  } else {
    const FlowState fs = flow_state(c);
    HIP_TRY(c, txv_flow_reset(&fs, keep_ids ? 1 : 0, c->stream));
    if (keep_ids) c->poisoned &= ~TXV_FERR_ARENA;
  }
  c->seq_next = 0;
  if (!keep_ids) {
    c->n_sets_host = 0;
    c->sets_seq = c->run_seq;   // a summary of a run enqueued before the reset is stale
  }
  return TXV_OK;
}

// SignBytes for every vote into s.tmp_msg (arena; offsets in s.tmp_off); returns max len
uint32_t encode_all(txv_ctx* c, Slot& s, const txv_votes* v, const char* chain, uint32_t chain_len,
                    std::vector<int>& lens) {
  s.tmp_msg.clear();
  s.tmp_msg.reserve((size_t)v->n * (160 + chain_len));
  s.tmp_off.resize(v->n);
  lens.resize(v->n);
  uint32_t mx = 0;
  for (uint32_t i = 0; i < v->n; ++i) {
    s.tmp_off[i] = s.tmp_msg.size();
    if (v->is_nil && v->is_nil[i]) { lens[i] = -2; continue; }
    const uint32_t need = 32 + 10 + 10 + v->txhash_len[i] + 24 + chain_len + 16;
    const size_t at = s.tmp_msg.size();
    s.tmp_msg.resize(at + need);
    const int L = txv_host::sign_bytes(s.tmp_msg.data() + at, need, v->height[i], v->txhash + v->txhash_off[i],
                                       v->txhash_len[i], v->ts_sec[i], v->ts_nanos[i], (const uint8_t*)chain,
                                       chain_len);
    s.tmp_msg.resize(at + (L > 0 ? (size_t)L : 0));
    lens[i] = L;
    if (L > 0 && (uint32_t)L > mx) mx = (uint32_t)L;
  }
  (void)c;
  return mx;
}

// column-major transposes into the slot's pinned buffers
void pack_columns(Slot& s, const txv_votes* v, const std::vector<int>& lens) {
  const uint32_t n = v->n, np = s.n_pad, mw = s.msg_words;
  s.msg_on_device = false;
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t* sg = v->sig + (size_t)i * 64;
    const uint32_t sl = v->sig_len[i] > 64 ? 64 : v->sig_len[i];
    uint8_t tmp[64];
    memset(tmp, 0, 64);
    memcpy(tmp, sg, sl);
    for (int j = 0; j < 16; ++j) s.h_sig[(size_t)j * np + i] = le32(tmp + 4 * j);
    const int L = lens[i];
    s.h_msg_len[i] = L > 0 ? (uint32_t)L : 0;
    const uint8_t* m = s.tmp_msg.data() + s.tmp_off[i];
    for (uint32_t w = 0; w < mw; ++w) {
      uint8_t b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (L > 0) {
        const int off = (int)(8 * w);
        const int take = std::min(8, L - off);
        if (take > 0) memcpy(b, m + off, (size_t)take);
      }
      s.h_msg[(size_t)w * np + i] = be64(b);
    }
  }
  for (uint32_t i = n; i < np; ++i) {
    for (int j = 0; j < 16; ++j) s.h_sig[(size_t)j * np + i] = 0;
    for (uint32_t w = 0; w < mw; ++w) s.h_msg[(size_t)w * np + i] = 0;
    s.h_msg_len[i] = 0; s.h_val[i] = 0; s.h_set[i] = 0; s.h_flags[i] = 0; s.h_status[i] = TXV_ERR_NIL;
  }
}

int upload_slot(txv_ctx* c, Slot& s) {
  const size_t np = s.n_pad;
  HIP_TRY(c, hipMemcpyAsync(s.d_sig, s.h_sig, 16 * np * 4, hipMemcpyHostToDevice, c->copy_stream));
  if (!s.msg_on_device)
    HIP_TRY(c, hipMemcpyAsync(s.d_msg, s.h_msg, (size_t)s.msg_words * np * 8, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_msg_len, s.h_msg_len, np * 4, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_val, s.h_val, np * 4, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_set, s.h_set, np * 4, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_flags, s.h_flags, np, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_pre, s.h_status, np, hipMemcpyHostToDevice, c->copy_stream));
  if (s.n_work)
    HIP_TRY(c, hipMemcpyAsync(s.d_order, s.h_order, (size_t)s.n_work * 4, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipEventRecord(s.ev[3], c->copy_stream));   // kernels on c->stream wait for it
  return TXV_OK;
}

// Counting sort of the pending votes by validator (keys = validator or caller-key index <
// n_keys), the verify-only paths' K1b work list with the small tables (verify_args).
void build_order(txv_ctx* c, Slot& s, uint32_t n_keys) {
  s.n_work = txv_host::counting_sort(*c->pool, s.n, std::max<uint32_t>(n_keys, 1),
      [&](uint32_t i) { return (s.h_flags[i] & TXV_FLAG_PENDING) ? s.h_val[i] : UINT32_MAX; },
      [&](uint32_t p, uint32_t i) { s.h_order[p] = i; });
}

uint32_t verify_grid(txv_ctx* c, uint32_t n) {
  const uint32_t blocks = (n + TXV_VERIFY_BLOCK - 1) / TXV_VERIFY_BLOCK;
  const uint32_t cap = (uint32_t)c->n_cus * 2;   // 2 x 512-thread workgroups per CU (LDS: 2 x 55 KB B table)
  return std::max<uint32_t>(1, std::min(blocks, cap));
}

// K1b's work list.  With the small tables (w <= 12: at most 4.3 MB per validator) it is the
// validator-sorted pending list, so the lanes of a wave mostly share one validator's A table
// (L2-resident gathers).  With wider tables a validator's table is tens to hundreds of MB and
// every gather misses L2 whatever the order, while the validator order scatters the vote-column
// reads (sig, kbuf: 24 words per vote at a stride of ~n_vals votes) over 24 distinct lines per
// vote (measured at w = 20: 59 L2 line misses per vote, 36 of them table lines); there K1b walks
// the votes in arrival order (order = null, n_work = n; K1a marks non-pending votes ok = 0).
VerifyArgs verify_args(txv_ctx* c, Slot& s, const uint32_t* pubs, const uint8_t* dok, const uint32_t* tabs, int w,
                       const uint32_t* tslot) {
  VerifyArgs a{};
  a.n = s.n; a.n_pad = s.n_pad; a.msg_words = s.msg_words;
  a.sig = s.d_sig; a.msg = s.d_msg; a.msg_len = s.d_msg_len; a.val = s.d_val; a.flags = s.d_flags;
  const bool by_val = w <= 12;
  a.n_work = by_val || !s.n_work ? s.n_work : s.n; a.kbuf = s.d_kbuf;
  a.order = by_val ? s.d_order : nullptr; a.pubs_le = pubs; a.decode_ok = dok; a.atables = tabs; a.btable = c->d_btable;
  a.ok_out = s.d_ok;
  a.tslot = tslot;
  a.park = c->d_park;
  a.park_waves = (uint32_t)(c->park_words / ((size_t)8 * TXV_PARK_WORDS * 64));
  a.n_cus = (uint32_t)c->n_cus;
  a.wctr = c->d_wctr;
  a.rpts = s.d_rpts;
  a.lane_votes = c->lane_votes;
  return a;
}

// K1b votes per lane for a launch with base window wb.  V = 8 halves the inversions per vote
// but also the waves; with the divstep inverse it wins once the batch still fills >= 1.5 waves
// per SIMD (C2, 1M votes: 517 vs 503-512M votes/s, profiles/r01/inv_var, profiles/r01/park);
// smaller batches run one vote per lane (split mode: the points kernel + K1c's batched
// inversion), which gives them the most waves (C5's 65k votes: 0.52 ms vs 0.60 at V = 4,
// profiles/r02/small_batch).  V = 8 kernels exist for the radix-2^24 / 2^26 base
// tables only, so a configured V = 8 runs V = 4 on any other base table (e.g. when no wide
// table could be allocated, or for caller-key tables).
uint32_t launch_lane_votes(const txv_ctx* c, int wb, uint32_t n_work) {
  const bool wide = wb == 24 || wb == 26;
  if (c->lane_auto) return wide && n_work >= (3u << 18) ? 8u : 1u;
  if (!wide) return c->lane_votes == 8 ? 4u : c->lane_votes;
  return c->lane_votes;
}

// scratch for the parked results per K1b lane (V slots: the last one with TXV_PARK_LAST) (the grid never exceeds verify_grid's cap)
int ensure_park(txv_ctx* c) {
  if (c->lane_votes == 1) return TXV_OK;   // split mode parks nothing
  const size_t words = (size_t)(c->lane_auto ? 8u : c->lane_votes) * TXV_PARK_WORDS * (size_t)c->n_cus * 2 * TXV_VERIFY_BLOCK;
  int r;
  if (!c->d_wctr && (r = dalloc(c, &c->d_wctr, 8 * 16))) return r;
  if (words <= c->park_words) return TXV_OK;
  if ((r = dalloc(c, &c->d_park, words))) return r;
  c->park_words = words;
  return TXV_OK;
}

// Device SignBytes for slot s: stage the raw fields + the TxHash arena prefix
// [0, arena_end) into pinned buffers (parallel), upload them on the copy stream and build the
// column-major message words there with txv_k_signbytes.  s.h_msg_len must be set already.
int encode_signbytes_device(txv_ctx* c, Slot& s, const txv_votes* v, const uint8_t* d_chain, uint32_t chain_len,
                            uint64_t arena_end) {
  const uint32_t n = s.n, np = s.n_pad;
  if (arena_end + 16 > s.arena_cap) {   // + 16 zero bytes: txv_k_signbytes reads 8 bytes at a time
    int r;
    const size_t cap = std::max<size_t>((size_t)arena_end + 16, s.arena_cap * 2);
    if ((r = halloc(c, &s.h_arena, cap)) || (r = dalloc(c, &s.d_arena_th, cap))) return r;
    s.arena_cap = cap;
  }
  c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
    memcpy(s.h_fh + lo, v->height + lo, (size_t)(hi - lo) * 8);
    memcpy(s.h_fs + lo, v->ts_sec + lo, (size_t)(hi - lo) * 8);
    memcpy(s.h_fn + lo, v->ts_nanos + lo, (size_t)(hi - lo) * 4);
    memcpy(s.h_fo + lo, v->txhash_off + lo, (size_t)(hi - lo) * 4);
    memcpy(s.h_fl + lo, v->txhash_len + lo, (size_t)(hi - lo) * 4);
  }, 16384);
  if (arena_end) memcpy(s.h_arena, v->txhash, (size_t)arena_end);
  memset(s.h_arena + arena_end, 0, 16);
  HIP_TRY(c, hipMemcpyAsync(s.d_fh, s.h_fh, (size_t)n * 8, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_fs, s.h_fs, (size_t)n * 8, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_fn, s.h_fn, (size_t)n * 4, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_fo, s.h_fo, (size_t)n * 4, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_fl, s.h_fl, (size_t)n * 4, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_arena_th, s.h_arena, (size_t)arena_end + 16, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_msg_len, s.h_msg_len, (size_t)np * 4, hipMemcpyHostToDevice, c->copy_stream));
  SignBytesArgs a{};
  a.n = n; a.n_pad = np; a.msg_words = s.msg_words; a.chain_len = chain_len;
  a.height = s.d_fh; a.ts_sec = s.d_fs; a.ts_nanos = s.d_fn; a.txhash_off = s.d_fo; a.txhash_len = s.d_fl;
  a.txhash = s.d_arena_th; a.chain = d_chain; a.msg_len = s.d_msg_len; a.msg = s.d_msg;
  HIP_TRY(c, txv_launch_signbytes(&a, c->copy_stream));
  s.msg_on_device = true;
  return TXV_OK;
}

// txv_set_validators / txv_sign_votes chain ids on the device
int upload_chain(txv_ctx* c, const char* chain, uint32_t len, uint8_t** d, uint32_t* cap) {
  if (len + 16 > *cap) {   // 16 bytes of zero padding: the SignBytes kernel reads 8 bytes at a time
    int r;
    if ((r = dalloc(c, d, (size_t)len + 16))) return r;
    *cap = len + 16;
  }
  HIP_TRY(c, hipMemsetAsync(*d, 0, *cap, c->copy_stream));
  if (len) HIP_TRY(c, hipMemcpyAsync(*d, chain, len, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipStreamSynchronize(c->copy_stream));
  return TXV_OK;
}

// Bound on the SignBytes length of any vote whose TxHash has at most max_hl bytes (the verify
// kernels' message-column count): length prefix + Height (9) + TxHash field + TxKey (34) +
// Timestamp field (<= 19) + ChainID field
uint32_t signbytes_bound(uint32_t max_hl, uint32_t chain_len) {
  const uint64_t body = 9 + (1 + txv_host::put_uvarint(nullptr, max_hl) + (uint64_t)max_hl) + 34 + 19 +
                        (chain_len ? 1 + txv_host::put_uvarint(nullptr, chain_len) + chain_len : 0);
  return (uint32_t)(txv_host::put_uvarint(nullptr, body) + body);
}

bool is_registered(const txv_ctx* c, const void* p, uint64_t bytes) {
  // TXV_IGNORE_REGISTERED=1 (experiment): every upload through the library's own pinned staging
  static const bool ignore = getenv("TXV_IGNORE_REGISTERED") && atoi(getenv("TXV_IGNORE_REGISTERED")) == 1;
  if (ignore) return false;
  const uintptr_t a = (uintptr_t)p;
  for (const auto& r : c->registered)
    if (a >= r.first && a + bytes <= r.first + r.second) return true;
  return false;
}

// AddVote staging: the caller's raw columns go to the device as they are (txv_flow.h
// FlowBatch); the only host pass reads TxHash offsets / lengths (arena extent, message-column
// bound).  Registered columns are DMA'd straight from caller memory; the others are copied into
// the slot's pinned buffers chunk by chunk on the pack threads, each chunk's DMA queued as soon
// as it is copied, so copies and PCIe transfers overlap.
// TxKey = SHA-256(tx), TxHash = its upper-hex digest (types/tx_vote.go:38-45): true when the key
// is the 32 bytes the 64 characters at hex spell.  SSE2 (x86-64 baseline): nibbles interleaved,
// to ASCII, compared 16 characters at a time (7.6 ns per vote on one core vs 30-55 for a
// table-driven encode + memcmp: this runs over every vote of a staged batch)
inline bool txkey_spelled(const uint8_t* key, const uint8_t* hex) {
  const __m128i m = _mm_set1_epi8(0x0F), nine = _mm_set1_epi8(9), zero = _mm_set1_epi8('0'), seven = _mm_set1_epi8(7);
  int ok = 0xFFFF;
  for (int h = 0; h < 2; ++h) {
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(key + 16 * h));
    const __m128i hi = _mm_and_si128(_mm_srli_epi16(v, 4), m), lo = _mm_and_si128(v, m);
    const __m128i a = _mm_unpacklo_epi8(hi, lo), b = _mm_unpackhi_epi8(hi, lo);
    const __m128i ca = _mm_add_epi8(_mm_add_epi8(a, zero), _mm_and_si128(_mm_cmpgt_epi8(a, nine), seven));
    const __m128i cb = _mm_add_epi8(_mm_add_epi8(b, zero), _mm_and_si128(_mm_cmpgt_epi8(b, nine), seven));
    ok &= _mm_movemask_epi8(_mm_cmpeq_epi8(ca, _mm_loadu_si128(reinterpret_cast<const __m128i*>(hex + 32 * h))));
    ok &= _mm_movemask_epi8(_mm_cmpeq_epi8(cb, _mm_loadu_si128(reinterpret_cast<const __m128i*>(hex + 32 * h + 16))));
  }
  return ok == 0xFFFF;
}

// the staged batch's pending fills (Slot::fill_*) on stream st, behind its uploads
int slot_fills(txv_ctx* c, Slot& s, hipStream_t st) {
  const uint32_t n = s.n;
  enum { kUH, kUS, kUHL, kUAL, kUSL };
  if (n && s.fill_mask) {
    if (s.fill_mask >> kUH & 1) HIP_TRY(c, txv_fill64(reinterpret_cast<uint64_t*>(s.d_fh), (uint64_t)s.fill_h, n, st));
    if (s.fill_mask >> kUS & 1) HIP_TRY(c, txv_fill64(reinterpret_cast<uint64_t*>(s.d_fs), (uint64_t)s.fill_s, n, st));
    if (s.fill_mask >> kUHL & 1) HIP_TRY(c, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(s.d_fl), (int)s.fill_hl, n, st));
    if (s.fill_mask >> kUAL & 1) HIP_TRY(c, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(s.d_addr_len), (int)s.fill_al, n, st));
    if (s.fill_mask >> kUSL & 1) HIP_TRY(c, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(s.d_sig_len), (int)s.fill_sl, n, st));
  }
  if (n && s.fill_key)
    HIP_TRY(c, txv_txkey_from_hash(s.d_arena_th, s.d_fo, s.has_nil ? s.d_nil : nullptr, n, s.d_txkey, st));
  s.fill_mask = 0;
  s.fill_key = false;
  return TXV_OK;
}

// route = true: the columns of a batch txv_route_admitted packs for the ranks (no TxFlow run: no
// validator set needed, no sequence numbers taken, every address column uploaded)
int stage_add(txv_ctx* c, uint32_t slot, const txv_votes* v, bool route = false) {
  if (!route && !c->n_vals) { c->err = "no validator set"; return TXV_ESTATE; }
  if (v->n > c->cfg.max_batch) { c->err = "batch exceeds max_batch"; return TXV_ECAPACITY; }
  if (!route && c->poisoned) { c->err = "a TxFlow capacity was exceeded: txv_reset_flow first"; return TXV_ECAPACITY; }
  Slot& s = c->slots[slot];
  const uint32_t n = v->n;
  const uint32_t chain_len = (uint32_t)c->chain.size();
  HostTimer ht(c->profile_host);
  std::atomic<uint64_t> arena_end{0};
  std::atomic<uint32_t> max_hl{0};
  // columns whose every element equals the first are not uploaded but filled on the device
  // (height, seconds and the three length columns: 28 of a vote's 152 bytes when uniform)
  enum { kUH, kUS, kUHL, kUAL, kUSL, kU };
  std::atomic<uint32_t> varying{0};
  const bool check_uniform = n > 0 && c->uniform_cols && v->height && v->ts_sec && v->txhash_len && v->addr_len &&
                             v->sig_len;
  // the TxKey column is decoded from the TxHash arena on the device when every non-nil vote's
  // key is what its TxHash spells (32 of a vote's bytes)
  const bool check_key = n > 0 && c->derive_txkey && v->txkey && v->txhash && v->txhash_off && v->txhash_len;
  std::atomic<bool> key_differs{false};
  c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
    uint64_t ae = 0;
    uint32_t mh = 0, var = 0;
    for (uint32_t i = lo; i < hi; ++i) {
      if (v->is_nil && v->is_nil[i]) continue;
      ae = std::max<uint64_t>(ae, (uint64_t)v->txhash_off[i] + v->txhash_len[i]);
      mh = std::max(mh, v->txhash_len[i]);
    }
    if (check_uniform) {
      for (uint32_t i = lo; i < hi; ++i) {
        var |= (uint32_t)(v->height[i] != v->height[0]) << kUH | (uint32_t)(v->ts_sec[i] != v->ts_sec[0]) << kUS |
               (uint32_t)(v->txhash_len[i] != v->txhash_len[0]) << kUHL |
               (uint32_t)(v->addr_len[i] != v->addr_len[0]) << kUAL | (uint32_t)(v->sig_len[i] != v->sig_len[0]) << kUSL;
      }
      if (var) varying.fetch_or(var);
    }
    if (check_key && !key_differs.load(std::memory_order_relaxed)) {
      for (uint32_t i = lo; i < hi; ++i) {
        if (v->is_nil && v->is_nil[i]) continue;
        if (v->txhash_len[i] != 64 || !txkey_spelled(v->txkey + (size_t)i * 32, v->txhash + v->txhash_off[i])) {
          key_differs.store(true, std::memory_order_relaxed);
          break;
        }
      }
    }
    uint64_t ca = arena_end.load();
    while (ae > ca && !arena_end.compare_exchange_weak(ca, ae)) {}
    uint32_t cm = max_hl.load();
    while (mh > cm && !max_hl.compare_exchange_weak(cm, mh)) {}
  }, 4096);   // a 64k batch (C5) over 16 workers: this scan sits between CheckTx and the chain
  const uint32_t uniform = check_uniform ? ~varying.load() & ((1u << kU) - 1u) : 0u;
  const uint64_t ae = arena_end.load();
  if (ae >= (1ull << 32)) { c->err = "TxHash arena >= 4 GiB"; return TXV_EINVAL; }
  const uint32_t mw = (signbytes_bound(max_hl.load(), chain_len) + 7) / 8;
  int r;
  if ((r = ensure_slot(c, s, n, mw)) || (r = ensure_flow_slot(c, s, n))) return r;
  if (ae + 16 > s.arena_cap) {
    const size_t cap = std::max<size_t>((size_t)ae + 16, s.arena_cap * 2);
    if ((r = halloc(c, &s.h_arena, cap)) || (r = dalloc(c, &s.d_arena_th, cap))) return r;
    s.arena_cap = cap;
  }
  s.n = n; s.n_pad = (n + 63) / 64 * 64; s.msg_words = mw;
  s.has_nil = v->is_nil != nullptr;
  s.has_txkey = v->txkey != nullptr;
  s.arena_end = ae;
  if (!route) {
    s.seq_base = c->seq_next;
    c->seq_next += n;
  }
  ht.mark("scan");
  struct Col { const uint8_t* src; uint8_t* pin; uint8_t* dev; size_t elem; bool reg; };
  Col cols[11];
  int nc = 0;
  auto add = [&](const void* src, void* pin, void* dev, size_t elem) {
    if (!src) return;
    cols[nc++] = Col{(const uint8_t*)src, (uint8_t*)pin, (uint8_t*)dev, elem, is_registered(c, src, (uint64_t)n * elem)};
  };
  add((uniform >> kUH & 1) ? nullptr : v->height, s.h_fh, s.d_fh, 8);
  add((uniform >> kUS & 1) ? nullptr : v->ts_sec, s.h_fs, s.d_fs, 8);
  add(v->ts_nanos, s.h_fn, s.d_fn, 4);
  add(v->txhash_off, s.h_fo, s.d_fo, 4);
  add((uniform >> kUHL & 1) ? nullptr : v->txhash_len, s.h_fl, s.d_fl, 4);
  // ValidatorSet.GetByAddress on the pack threads (the device's table, host_pack.hpp AddrTable):
  // a 2-byte code per vote crosses PCIe instead of the 20-byte address and its length
  const bool host_val = !route && (c->host_val == 1 || (c->host_val < 0 && n >= kHostValMin)) && v->addr &&
                        v->addr_len && c->n_vals < kVcodeEmpty;
  s.host_val = host_val;
  if (!host_val) {
    add(v->addr, s.h_addr, s.d_addr, 20);
    add((uniform >> kUAL & 1) ? nullptr : v->addr_len, s.h_addr_len, s.d_addr_len, 4);
  }
  add(v->sig, s.h_sigraw, s.d_sigraw, 64);
  add((uniform >> kUSL & 1) ? nullptr : v->sig_len, s.h_sig_len, s.d_sig_len, 4);
  add(v->is_nil, s.h_nil, s.d_nil, 1);
  const bool derive_key = check_key && !key_differs.load();
  add(derive_key ? nullptr : v->txkey, s.h_txkey, s.d_txkey, 32);
  if (s.launched) HIP_TRY(c, hipStreamWaitEvent(c->copy_stream, s.ev[4], 0));   // its last chain has ended
  // the fills: a TxFlow batch's at its run_slot on the key stream (the copy stream keeps to DMA), a
  // route batch's here (its columns are read by the route kernels, not a chain)
  s.fill_mask = uniform & ~(host_val ? (1u << kUAL) : 0u);
  s.fill_h = n ? v->height[0] : 0; s.fill_s = n ? v->ts_sec[0] : 0;
  s.fill_hl = n ? v->txhash_len[0] : 0; s.fill_al = n ? v->addr_len[0] : 0; s.fill_sl = n ? v->sig_len[0] : 0;
  if (route && (r = slot_fills(c, s, c->copy_stream))) return r;
  for (int k = 0; k < nc; ++k)
    if (cols[k].reg && n) HIP_TRY(c, hipMemcpyAsync(cols[k].dev, cols[k].src, (size_t)n * cols[k].elem, hipMemcpyHostToDevice, c->copy_stream));
  // TxHash arena (+ 16 zero bytes: the device reads keys 8 bytes at a time)
  const bool arena_reg = is_registered(c, v->txhash, ae);
  if (arena_reg) {
    if (ae) HIP_TRY(c, hipMemcpyAsync(s.d_arena_th, v->txhash, (size_t)ae, hipMemcpyHostToDevice, c->copy_stream));
    HIP_TRY(c, hipMemsetAsync(s.d_arena_th + ae, 0, 16, c->copy_stream));
  }
  const uint32_t chunk = std::max<uint32_t>(65536, (n + 7) / 8);
  const uint64_t achunk = std::max<uint64_t>(1u << 20, (ae + 7) / 8);
  const uint32_t n_chunks = std::max<uint32_t>((n + chunk - 1) / chunk, arena_reg ? 0u : (uint32_t)((ae + achunk - 1) / achunk));
  for (uint32_t k = 0; k < n_chunks; ++k) {
    const uint32_t lo = std::min<uint64_t>((uint64_t)k * chunk, n), hi = std::min<uint64_t>((uint64_t)(k + 1) * chunk, n);
    const uint64_t alo = arena_reg ? 0 : std::min<uint64_t>(k * achunk, ae), ahi = arena_reg ? 0 : std::min<uint64_t>((k + 1) * achunk, ae);
    c->pool->parallel_for(hi - lo + (uint32_t)((ahi - alo + 4095) / 4096), [&](uint32_t a, uint32_t b) {
      // items [0, hi - lo) are votes of this chunk, the rest 4 KiB pages of its arena slice
      const uint32_t nv = hi - lo;
      if (a < nv) {
        const uint32_t va = lo + a, vb = lo + std::min(b, nv);
        for (int q = 0; q < nc; ++q)
          if (!cols[q].reg) memcpy(cols[q].pin + (size_t)va * cols[q].elem, cols[q].src + (size_t)va * cols[q].elem, (size_t)(vb - va) * cols[q].elem);
        if (host_val)
          for (uint32_t i = va; i < vb; ++i) {   // vote_set.go:97-106: empty address, then GetByAddress
            const uint32_t al = v->addr_len[i];
            uint32_t code = kVcodeUnknown;
            if (al == 0) code = kVcodeEmpty;
            else if (al == 20) code = std::min<uint32_t>(c->addr_tab.find(v->addr + (size_t)i * 20), kVcodeUnknown);
            s.h_vcode[i] = (uint16_t)code;
          }
      }
      if (b > nv) {
        const uint64_t pa = alo + (uint64_t)(std::max(a, nv) - nv) * 4096, pb = std::min<uint64_t>(alo + (uint64_t)(b - nv) * 4096, ahi);
        if (pb > pa) memcpy(s.h_arena + pa, v->txhash + pa, pb - pa);
      }
    }, 4096);
    for (int q = 0; q < nc; ++q)
      if (!cols[q].reg && hi > lo)
        HIP_TRY(c, hipMemcpyAsync(cols[q].dev + (size_t)lo * cols[q].elem, cols[q].pin + (size_t)lo * cols[q].elem,
                                  (size_t)(hi - lo) * cols[q].elem, hipMemcpyHostToDevice, c->copy_stream));
    if (host_val && hi > lo)
      HIP_TRY(c, hipMemcpyAsync(s.d_vcode + lo, s.h_vcode + lo, (size_t)(hi - lo) * 2, hipMemcpyHostToDevice, c->copy_stream));
    if (ahi > alo)
      HIP_TRY(c, hipMemcpyAsync(s.d_arena_th + alo, s.h_arena + alo, ahi - alo, hipMemcpyHostToDevice, c->copy_stream));
  }
  if (!arena_reg) {
    memset(s.h_arena + ae, 0, 16);
    HIP_TRY(c, hipMemcpyAsync(s.d_arena_th + ae, s.h_arena + ae, 16, hipMemcpyHostToDevice, c->copy_stream));
  }
  s.fill_key = derive_key;
  if (route && (r = slot_fills(c, s, c->copy_stream))) return r;
  {
    uint64_t up = ae + 16 + (host_val ? (uint64_t)n * 2 : 0);
    for (int k = 0; k < nc; ++k) up += (uint64_t)n * cols[k].elem;
    c->staged_bytes = up;
  }
  HIP_TRY(c, hipEventRecord(s.ev[3], c->copy_stream));   // run_slot's kernels wait for this
  ht.mark("upload");
  s.staged = true; s.ran = false;
  return TXV_OK;
}

FlowBatch flow_batch(const txv_ctx* c, const Slot& s) {
  FlowBatch b{};
  b.n = s.n; b.n_pad = s.n_pad; b.msg_words = s.msg_words; b.chain_len = (uint32_t)c->chain.size();
  b.seq_base = s.seq_base;
  b.stamp = s.stamp;
  b.height = s.d_fh; b.ts_sec = s.d_fs; b.ts_nanos = s.d_fn; b.th_off = s.d_fo; b.th_len = s.d_fl; b.th = s.d_arena_th;
  b.addr = s.d_addr; b.addr_len = s.d_addr_len; b.sig_raw = s.d_sigraw; b.sig_len = s.d_sig_len;
  b.nil = s.has_nil ? s.d_nil : nullptr; b.txkey = s.has_txkey ? s.d_txkey : nullptr;
  b.vcode = s.host_val ? s.d_vcode : nullptr;
  b.sig = s.d_sig; b.msg_len = s.d_msg_len; b.val = s.d_val; b.flags = s.d_flags; b.pre = s.d_pre;
  b.entry = s.d_entry; b.set = s.d_set; b.ok = s.d_ok; b.status = s.d_status;
  b.ev_flag = s.d_ev_flag; b.mark = s.d_mark; b.blk = s.d_blk; b.stamped = s.d_stamped; b.ev_tiles = s.d_ev_tiles;
  b.status_host = s.m_out; b.ev_host = s.m_ev; b.summary_host = s.m_sum;
  return b;
}

// device times of a slot's last run (its events have completed): prep (+ SignBytes), verify,
// tally after verify, and the whole chain from the prep's start
int slot_kernel_ms(txv_ctx* c, Slot& s, float* ms) {
  // prep + SignBytes; K1a + K1b (each on its own stream: their durations added)
  float k1a = 0.f, k1b = 0.f;
  if (TXV_K1A_ON_KEY_STREAM) {
    HIP_TRY(c, hipEventElapsedTime(&ms[0], s.ev[0], s.ev[8]));
    HIP_TRY(c, hipEventElapsedTime(&k1a, s.ev[8], s.ev[1]));
  } else {
    HIP_TRY(c, hipEventElapsedTime(&ms[0], s.ev[0], s.ev[1]));
  }
  HIP_TRY(c, hipEventElapsedTime(&k1b, s.ev[7], s.ev[2]));
  ms[1] = k1a + k1b;
  HIP_TRY(c, hipEventElapsedTime(&ms[2], s.ev[2], s.ev[5]));
  HIP_TRY(c, hipEventElapsedTime(&ms[3], s.ev[0], s.ev[5]));
  return TXV_OK;
}

// the whole AddVote chain of a staged batch: prep + SignBytes -> K1a/K1b verify (verify
// stream), set keying -> new ids -> tally -> results into mapped host memory (flow stream)
int run_slot(txv_ctx* c, uint32_t slot, float* ms) {
  Slot& s = c->slots[slot];
  if (!s.staged) { c->err = "slot not staged"; return TXV_ESTATE; }
  if (c->poisoned) { c->err = "a TxFlow capacity was exceeded: txv_reset_flow first"; return TXV_ECAPACITY; }
  int r;
  if ((r = ensure_park(c))) return r;
  if (c->stamp == 0xFFFFFFFEu) {   // stamps are about to wrap: forget every candidate first
    const FlowState fs0 = flow_state(c);
    HIP_TRY(c, txv_flow_init_cells(&fs0, (uint64_t)c->cfg.max_txs * std::max<uint32_t>(c->n_vals, 1), 0, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->d_set_stamp, 0, (size_t)c->cfg.max_txs * 4, c->stream));
    c->stamp = 0;
  }
  s.stamp = ++c->stamp;            // every run of a batch gets a stamp of its own
  // The event compaction's look-back words carry the stamp's low 30 bits and are never cleared
  // between runs.  A new tag cycle -- the first run after alloc_tally or the wrap above reset the
  // stamp, or every 2^30 runs -- could meet a word an earlier cycle left with the same tag (ADVICE
  // r5): every slot's words are zeroed first, on the flow stream behind the runs before.
  if ((s.stamp & 0x3FFFFFFFu) == 1u)
    for (Slot& o : c->slots)
      if (o.d_ev_tiles) HIP_TRY(c, hipMemsetAsync(o.d_ev_tiles, 0, (size_t)o.ev_tiles_n * sizeof(uint64_t), c->stream));
  s.run_seq = ++c->run_seq;
  const FlowState fs = flow_state(c);
  const FlowBatch fb = flow_batch(c, s);
  // Three compute queues, so that batch k+1 verifies while batch k tallies and nothing but
  // K1a/K1b sits on the verify stream:
  //   key stream   (after the uploads on the copy stream) prep (pre-checks, validator lookup,
  //                signature transpose) and SignBytes: they read only the uploaded columns and
  //                run beside the previous batch's K1b; the copy stream stays pure DMA, so batch
  //                k+2's upload never queues behind them
  //   vstream      K1a/K1b: reads nothing the TxFlow owns, so it never waits for an earlier
  //                batch's tally
  //   flow stream  set keying + new set ids, then -- after this batch's verify -- the tally:
  //                every TxFlow access stays in batch order on this one stream
  // (GPU_MAX_HW_QUEUES = 4: flow, copy, key and verify streams each get a hardware queue; a
  // further stream would share, i.e. serialise with, one of them)
  // the slot's previous chain (its tally reads the derived columns prep rewrites) has ended
  hipStream_t ps = c->key_stream;
  HIP_TRY(c, hipStreamWaitEvent(ps, s.ev[3], 0));
  if (s.launched) HIP_TRY(c, hipStreamWaitEvent(ps, s.ev[4], 0));
  if (s.fill_mask || s.fill_key) {   // the staging's fills (first run of a staging only)
    if ((r = slot_fills(c, s, ps))) return r;
    HIP_TRY(c, hipEventRecord(s.ev[3], ps));
  }
  HIP_TRY(c, hipStreamWaitEvent(c->stream, s.ev[3], 0));
  // TXV_PREP_AFTER_K1B=1 (experiment): this batch's prep + SignBytes wait for the K1b two batches
  // back, so they run beside the next K1a instead of beside a K1b
  static const bool prep_after = getenv("TXV_PREP_AFTER_K1B") && atoi(getenv("TXV_PREP_AFTER_K1B")) == 1;
  if (prep_after && c->vend_n >= 2) HIP_TRY(c, hipStreamWaitEvent(ps, c->vend_ev[(c->vend_n - 2) % 4], 0));
  HIP_TRY(c, hipEventRecord(s.ev[0], ps));
  SignBytesArgs sa{};
  sa.n = s.n; sa.n_pad = s.n_pad; sa.msg_words = s.msg_words; sa.chain_len = fb.chain_len;
  sa.height = s.d_fh; sa.ts_sec = s.d_fs; sa.ts_nanos = s.d_fn; sa.txhash_off = s.d_fo; sa.txhash_len = s.d_fl;
  sa.txhash = s.d_arena_th; sa.chain = c->d_chain; sa.msg_len = nullptr; sa.nil = s.has_nil ? s.d_nil : nullptr;
  sa.msg = s.d_msg;
  VerifyArgs va = verify_args(c, s, c->d_pubs, c->d_decode_ok, c->d_atables, c->tab_w, c->d_vslot);
  va.order = nullptr;          // arrival order; K1a marks the non-pending votes
  va.n_work = s.n;
  va.lane_votes = launch_lane_votes(c, c->b_w, va.n_work);
  if (!txv_verify_windows_supported(c->b_w, c->tab_w)) { c->err = "verify windows"; return TXV_EDEVICE; }
  // TXV_K1B_FUSED=1 (experiment): the work-stealing K1b computes each chunk's challenges itself
  static const bool fuse = getenv("TXV_K1B_FUSED") && atoi(getenv("TXV_K1B_FUSED")) == 1;
  va.fused_k1a = fuse && txv_k1b_fusable(c->b_w, &va) ? 1u : 0u;
  HIP_TRY(c, txv_flow_prep(&fs, &fb, ps));
  HIP_TRY(c, txv_launch_signbytes(&sa, ps));
  if (TXV_K1A_ON_KEY_STREAM && !va.fused_k1a) {
    HIP_TRY(c, hipEventRecord(s.ev[8], ps));
    HIP_TRY(c, txv_launch_challenge(&va, ps));
  }
  HIP_TRY(c, hipEventRecord(s.ev[1], ps));
  HIP_TRY(c, hipStreamWaitEvent(c->vstream, s.ev[1], 0));
  HIP_TRY(c, hipEventRecord(s.ev[7], c->vstream));
  // TXV_K1B_AFTER_TALLY=1 (experiment): K1b waits for the previous batch's tally, which then runs
  // beside this batch's K1a instead of beside its K1b
  static const bool after_tally = getenv("TXV_K1B_AFTER_TALLY") && atoi(getenv("TXV_K1B_AFTER_TALLY")) == 1;
  if (!TXV_K1A_ON_KEY_STREAM || va.fused_k1a) {
    if (!va.fused_k1a) HIP_TRY(c, txv_launch_challenge(&va, c->vstream));
    if (after_tally && c->tally_ev_set) HIP_TRY(c, hipStreamWaitEvent(c->vstream, c->tally_ev, 0));
    HIP_TRY(c, hipEventRecord(s.ev[8], c->vstream));   // K1a | K1b split (txv_slot_verify_ms)
  }
  HIP_TRY(c, txv_launch_scalarmult(c->b_w, c->tab_w, &va, verify_grid(c, s.n), c->vstream));
  HIP_TRY(c, hipEventRecord(s.ev[2], c->vstream));
  if (prep_after) {
    hipEvent_t& ve = c->vend_ev[c->vend_n % 4];
    if (!ve) HIP_TRY(c, hipEventCreateWithFlags(&ve, hipEventDisableTiming));
    HIP_TRY(c, hipEventRecord(ve, c->vstream));
    ++c->vend_n;
  }
  HIP_TRY(c, txv_flow_route(&fs, &fb, c->stream));
  HIP_TRY(c, txv_flow_new_ids(&fs, &fb, c->stream));
  HIP_TRY(c, hipEventRecord(s.ev[6], c->stream));
  // set ids in use after this batch: at most those known at the newest fetched run + one per
  // vote of every run not fetched yet (a bound for the touched-set scan).  A slot run again
  // before it was fetched keeps its earlier run's votes counted too: that run's sets only show
  // in a later summary.
  c->unfetched += s.n;
  s.counted += s.n;
  const uint32_t sets_bound = (uint32_t)std::min<uint64_t>((uint64_t)c->n_sets_host + c->unfetched, c->cfg.max_txs);
  HIP_TRY(c, hipStreamWaitEvent(c->stream, s.ev[2], 0));
  HIP_TRY(c, txv_flow_tally(&fs, &fb, sets_bound, c->stream));
  HIP_TRY(c, hipEventRecord(s.ev[5], c->stream));
  if (after_tally) {
    if (!c->tally_ev) HIP_TRY(c, hipEventCreateWithFlags(&c->tally_ev, hipEventDisableTiming));
    HIP_TRY(c, hipEventRecord(c->tally_ev, c->stream));
    c->tally_ev_set = true;
  }
  if (s.sink) HIP_TRY(c, txv_flow_pack(&fs, s.sink, (s.sink_cap + 31) / 32, s.sink_cap, c->stream));
  HIP_TRY(c, hipEventRecord(s.ev[4], c->stream));
  s.ran = true;
  s.launched = true;
  if (ms) {
    HIP_TRY(c, hipEventSynchronize(s.ev[4]));
    if ((r = slot_kernel_ms(c, s, ms))) return r;
  }
  return TXV_OK;
}

int fetch_slot(txv_ctx* c, uint32_t slot, uint8_t* status_out, txv_commit_event* ev, uint32_t ev_cap, uint32_t* n_ev) {
  Slot& s = c->slots[slot];
  if (!s.ran) { c->err = "slot not run"; return TXV_ESTATE; }
  HostTimer ht(c->profile_host);
  HIP_TRY(c, hipEventSynchronize(s.ev[4]));
  ht.mark("fetch_sync");
  FlowSummary sm;
  memcpy(&sm, (const void*)s.h_sum, sizeof sm);   // written over PCIe by the last kernel
  // only a summary newer than the one applied last moves the set count (slots may be fetched out
  // of run order, e.g. staged slots beside the submit ring); an older one is covered by it
  if (s.run_seq > c->sets_seq) {
    c->n_sets_host = sm.n_sets;
    c->sets_seq = s.run_seq;
  }
  c->unfetched -= s.counted;
  s.counted = 0;
  if (sm.err & TXV_FERR_LOOKBACK) {   // a broken invariant, not a capacity: the event ranks are not trusted
    c->poisoned |= sm.err;
    c->err = "TxFlow event compaction: look-back timed out (device error; txv_reset_flow to recover)";
    return TXV_EDEVICE;
  }
  if (sm.err) {
    c->poisoned |= sm.err;
    c->err = std::string("TxFlow capacity exceeded:") + ((sm.err & TXV_FERR_SETS) ? " max_txs" : "") +
             ((sm.err & TXV_FERR_TABLE) ? " set-table" : "") + ((sm.err & TXV_FERR_KEYS) ? " key_arena_bytes" : "") +
             ((sm.err & TXV_FERR_ARENA) ? " max_accepted" : "") + " (txv_reset_flow to recover)";
    return TXV_ECAPACITY;
  }
  if (status_out && s.n) memcpy(status_out, s.h_out, s.n);
  ht.mark("fetch_copy");
  static_assert(sizeof(FlowEvent) == sizeof(txv_commit_event), "event layout");
  const uint32_t ne = sm.n_events;
  if (ev && ne) memcpy(ev, s.h_ev, (size_t)std::min(ne, ev_cap) * sizeof(FlowEvent));
  if (n_ev) *n_ev = ne;
  return TXV_OK;
}

// base-point table for window w (w = 4 lives in d_btable4, built at init for keygen/sign)
int build_base_table(txv_ctx* c, int w) {
  uint32_t* d_b = nullptr;
  int r;
  if ((r = dalloc(c, &d_b, 8))) return r;
  const uint32_t bw[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                          0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  HIP_TRY(c, hipMemcpyAsync(d_b, bw, 32, hipMemcpyHostToDevice, c->stream));
  if (w == 4) {
    if ((r = dalloc(c, &c->d_btable4, kTableWords4))) return r;
    HIP_TRY(c, txv_launch_build_tables(4, d_b, 1, c->d_btable4, nullptr, nullptr, c->stream));
  } else if (c->btable_w != w) {
    if ((r = dalloc(c, &c->d_btable8, table_words(w)))) return r;
    HIP_TRY(c, txv_launch_build_tables(w, d_b, 1, c->d_btable8, nullptr, nullptr, c->stream));
    c->btable_w = w;
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  dfree(d_b);
  return TXV_OK;
}

// Largest window whose per-validator tables for n keys fit the table budget (more table
// memory = fewer point additions per vote: 2 * ceil(256 / W)).
int choose_window(const txv_ctx* c, uint32_t n) {
  if (c->cfg_w) return c->cfg_w;
  const uint64_t budget = (uint64_t)c->cfg.table_budget_mb << 20;
  for (int w : {20, 18, 16, 14, 12, 10, 8})
    if ((w <= 16 || c->lane_votes >= 4 || c->lane_votes == 1) && (uint64_t)std::max<uint32_t>(n, 1) * table_words(w) * 4 <= budget) return w;
  return 4;
}

// The wide base-point tables (11.8 GB at b_w = 24, 43 GB at 26) are the same constants for every
// context: one per (device, window) per process, shared by reference count, built by the first
// context that asks (under the registry lock, so a second one waits for the build).
struct SharedBaseTable { int device, w, refs; uint32_t* ptr; };
std::mutex g_base_mu;
std::vector<SharedBaseTable> g_base_tabs;

// a reference to the (device, w) table, built if absent; nullptr when it cannot be allocated
uint32_t* acquire_base_table(txv_ctx* c, int w, int* err) {
  std::lock_guard<std::mutex> g(g_base_mu);
  *err = TXV_OK;
  for (auto& t : g_base_tabs)
    if (t.device == c->device && t.w == w) { ++t.refs; return t.ptr; }
  uint32_t* p = nullptr;
  if (hipMalloc((void**)&p, table_words(w) * 4) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
  uint32_t* d_b = nullptr;
  auto fail = [&](hipError_t e) {
    c->err = std::string("base table build: ") + hipGetErrorString(e);
    (void)hipFree(p);
    if (d_b) (void)hipFree(d_b);
    *err = TXV_EDEVICE;
    return nullptr;
  };
  hipError_t e;
  if ((e = hipMalloc((void**)&d_b, 32)) != hipSuccess) return fail(e);
  const uint32_t bwords[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                              0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  if ((e = hipMemcpyAsync(d_b, bwords, 32, hipMemcpyHostToDevice, c->stream)) != hipSuccess) return fail(e);
  if ((e = txv_launch_build_tables(w, d_b, 1, p, nullptr, nullptr, c->stream)) != hipSuccess) return fail(e);
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return fail(e);
  (void)hipFree(d_b);
  g_base_tabs.push_back(SharedBaseTable{c->device, w, 1, p});
  return p;
}

void release_base_table(int device, uint32_t*& p) {
  if (!p) return;
  std::lock_guard<std::mutex> g(g_base_mu);
  for (size_t i = 0; i < g_base_tabs.size(); ++i)
    if (g_base_tabs[i].device == device && g_base_tabs[i].ptr == p) {
      if (--g_base_tabs[i].refs == 0) {
        (void)hipFree(p);
        g_base_tabs.erase(g_base_tabs.begin() + (long)i);
      }
      break;
    }
  p = nullptr;
}

// make tab_w = w current: its B table exists; then the verify kernel's base-point window
// b_w: the requested one if the kernels support (b_w, w), else by default the 11.8 GB radix-2^24
// table over radix-2^12..2^20 validator tables (11 instead of 16..22 additions for [s]B).  The
// 43 GB radix-2^26 table (10 positions) is selectable (TXV_CFG_SET_B_WINDOW(26)) but not the
// default: one addition of 23 saved buys +0.7-1.9 % (round 3) / +1.4 % (672.6 vs 662-664M
// votes/s on one box, profiles/r04/ab1), and with it as the default the GPU test suite -- several
// contexts alive, with throw-away key tables -- ran out of HBM (profiles/r04/v2_oom_gpu_tests.log).
// Wide tables are shared by every context of the process (acquire_base_table).  A wide table that
// cannot be allocated falls back to radix-2^24, then to b_w = w.  d_btable = table of b_w.
int select_window(txv_ctx* c, int w) {
  int r;
  // radix-2^18 / 2^20 validator tables only run against the wide base tables
  if (w != 4 && w <= 16 && (r = build_base_table(c, w))) return r;
  c->tab_w = w;
  c->d_btable = w == 4 ? c->d_btable4 : c->d_btable8;
  c->b_w = w;
  int bw = c->cfg_bw ? c->cfg_bw : (w == 21 ? 26 : w >= 12 ? 24 : w);
  if ((c->lane_votes < 4 && c->lane_votes != 1) || !txv_verify_windows_supported(bw, w)) bw = w;
  while (bw != w && c->btable_wide_w != bw) {
    release_base_table(c->device, c->d_btable_wide);
    c->btable_wide_w = 0;
    int e = TXV_OK;
    uint32_t* t = acquire_base_table(c, bw, &e);
    if (e) return e;
    if (!t) {
      bw = (bw == 26 && txv_verify_windows_supported(24, w)) ? 24 : w;   // no room: a narrower table
      continue;
    }
    c->d_btable_wide = t;
    c->btable_wide_w = bw;
  }
  if (bw != w) {
    c->b_w = bw;
    c->d_btable = c->d_btable_wide;
  }
  if (!txv_verify_windows_supported(c->b_w, w)) { c->err = "no verify kernel for this table window"; return TXV_ENOMEM; }
  return TXV_OK;
}

// Key registry a verify-only call runs against: the validator registry, or a throw-away set
// built from caller-supplied keys.
struct KeySet {
  const uint32_t* pubs;
  const uint8_t* ok;
  const uint32_t* tables;
  int w;
  const uint32_t* slot;   // table slot per key, null = key order
};

KeySet registry_keys(const txv_ctx* c) { return KeySet{c->d_pubs, c->d_decode_ok, c->d_atables, c->tab_w, c->d_vslot}; }

// Caller-supplied keys (txv_verify_batch with pubs32, txv_verify_bytes): de-duplicated into
// throw-away tables -- the registry's window when they fit the table budget (its B table
// already exists), else the 55 KB radix-16 tables; without a registry the window is chosen
// for these keys alone.  kidx[i] = key slot of item i; key_addr (optional) receives
// SHA-256(key)[:20] per slot, computed on the device by K0.
int prepare_keys(txv_ctx* c, const uint8_t* pubs32, uint32_t n, std::vector<uint32_t>& kidx,
                 std::vector<uint8_t>* key_addr, KeySet& ks) {
  std::unordered_map<std::string, uint32_t> uniq;
  std::vector<uint8_t> ukeys;
  kidx.resize(n);
  for (uint32_t i = 0; i < n; ++i) {
    std::string k((const char*)pubs32 + (size_t)i * 32, 32);
    auto it = uniq.find(k);
    if (it == uniq.end()) {
      it = uniq.emplace(k, (uint32_t)uniq.size()).first;
      ukeys.insert(ukeys.end(), k.begin(), k.end());
    }
    kidx[i] = it->second;
  }
  const uint32_t nu = (uint32_t)uniq.size();
  int r, w_keys;
  if (c->tab_w) {
    w_keys = (uint64_t)nu * table_words(c->tab_w) * 4 <= ((uint64_t)c->cfg.table_budget_mb << 20) ? c->tab_w : 4;
  } else {
    w_keys = std::min(choose_window(c, nu), 16);   // windows > 16 need the registry's wide B table
    if (w_keys != 4 && (r = build_base_table(c, w_keys))) return r;
  }
  if (nu > c->tmp_cap || w_keys != c->tmp_w) {
    if ((r = dalloc(c, &c->d_tmp_pubs, (size_t)nu * 8)) || (r = dalloc(c, &c->d_tmp_ok, nu)) ||
        (r = dalloc(c, &c->d_tmp_tables, (size_t)nu * table_words(w_keys))) || (r = dalloc(c, &c->d_tmp_addr, (size_t)nu * 5)))
      return r;
    c->tmp_cap = nu;
    c->tmp_w = w_keys;
  }
  if (nu) {
    HIP_TRY(c, hipMemcpyAsync(c->d_tmp_pubs, ukeys.data(), (size_t)nu * 32, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, txv_launch_build_tables(w_keys, c->d_tmp_pubs, nu, c->d_tmp_tables, c->d_tmp_ok, c->d_tmp_addr, c->stream));
  }
  if (key_addr) {
    key_addr->resize((size_t)nu * 20);
    if (nu) HIP_TRY(c, hipMemcpyAsync(key_addr->data(), c->d_tmp_addr, (size_t)nu * 20, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  ks = KeySet{c->d_tmp_pubs, c->d_tmp_ok, c->d_tmp_tables, w_keys, nullptr};
  return TXV_OK;
}

// Upload slot s and run K1 (verify only) against key set ks; ok[i] = 1 when vote i verified.
int run_verify(txv_ctx* c, Slot& s, const KeySet& ks, std::vector<uint8_t>& ok) {
  int r;
  if ((r = upload_slot(c, s)) || (r = ensure_park(c))) return r;
  HIP_TRY(c, hipStreamWaitEvent(c->vstream, s.ev[3], 0));
  VerifyArgs va = verify_args(c, s, ks.pubs, ks.ok, ks.tables, ks.w, ks.slot);
  const bool reg_w = ks.w == c->tab_w;
  const int w_base = reg_w ? c->b_w : ks.w;
  va.btable = reg_w ? c->d_btable : (ks.w == 4 ? c->d_btable4 : c->d_btable8);
  va.lane_votes = launch_lane_votes(c, w_base, va.n_work);
  HIP_TRY(c, txv_launch_verify(w_base, ks.w, &va, verify_grid(c, s.n), c->vstream));
  ok.resize(s.n);
  if (s.n) HIP_TRY(c, hipMemcpyAsync(ok.data(), s.d_ok, s.n, hipMemcpyDeviceToHost, c->vstream));
  HIP_TRY(c, hipStreamSynchronize(c->vstream));
  return TXV_OK;
}

// txv_submit_votes ring: ticket t runs in slot (t - 1) % kSubmitRing; a slot is reused only
// after its ticket was waited for (its pinned and device buffers are free again).  Three slots:
// batch k+2's host pass and staging run while batch k+1 uploads and batch k computes, so the
// host pass does not leave the link idle between uploads (two slots: 428.5M votes/s end to end,
// the host pass between a wait and the next upload)
int submit_votes(txv_ctx* c, const txv_votes* v, uint64_t* ticket) {
  const uint64_t t = c->next_ticket;
  const uint32_t slot = (uint32_t)((t - 1) % kSubmitRing);
  Slot& s = c->slots[slot];
  if (s.ticket) { c->err = "four batches already in flight: wait for the oldest one first"; return TXV_ESTATE; }
  int r;
  if ((r = stage_add(c, slot, v))) return r;
  if ((r = run_slot(c, slot, nullptr))) return r;
  s.ticket = t;
  c->next_ticket = t + 1;
  *ticket = t;
  return TXV_OK;
}

int wait_votes(txv_ctx* c, uint64_t ticket, uint8_t* status_out, txv_commit_event* ev, uint32_t ev_cap,
               uint32_t* n_ev) {
  if (!ticket) return TXV_EINVAL;
  const uint32_t slot = (uint32_t)((ticket - 1) % kSubmitRing);
  Slot& s = c->slots[slot];
  if (s.ticket != ticket) { c->err = "unknown or already waited ticket"; return TXV_ESTATE; }
  for (uint32_t o = 0; o < kSubmitRing; ++o)   // the other ring slots
    if (o != slot && c->slots[o].ticket && c->slots[o].ticket < ticket) {
      c->err = "tickets must be waited in submission order";
      return TXV_ESTATE;
    }
  s.ticket = 0;
  return fetch_slot(c, slot, status_out, ev, ev_cap, n_ev);
}

// The context's four streams.  Experiment knobs (environment, read once per context):
// TXV_VSTREAM_PRIO=1 creates the verify stream at the device's highest priority; TXV_FLOW_CUS=N
// restricts the flow and key streams to N CUs spread over the XCDs (hipExtStreamCreateWithCUMask),
// so their latency-bound kernels stay off the CUs K1b runs on.
hipError_t create_streams(txv_ctx* c) {
  hipError_t e;
  const char* fc = getenv("TXV_FLOW_CUS");
  const int flow_cus = fc ? atoi(fc) : 0;
  int ncu = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->device) == hipSuccess) ncu = prop.multiProcessorCount;
  if (flow_cus > 0 && flow_cus < ncu) {
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    const int stride = ncu / flow_cus;
    for (int i = 0, k = 0; i < ncu && k < flow_cus; i += stride, ++k) mask[i / 32] |= 1u << (i % 32);
    if ((e = hipExtStreamCreateWithCUMask(&c->stream, (uint32_t)mask.size(), mask.data())) != hipSuccess) return e;
    if ((e = hipExtStreamCreateWithCUMask(&c->key_stream, (uint32_t)mask.size(), mask.data())) != hipSuccess) return e;
  } else {
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return e;
    if ((e = hipStreamCreateWithFlags(&c->key_stream, hipStreamNonBlocking)) != hipSuccess) return e;
  }
  if ((e = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking)) != hipSuccess) return e;
  // TXV_VERIFY_CUS_OFF=N: the verify stream leaves N CUs (spread over the XCDs) to the flow and
  // key streams' kernels, which otherwise find no VGPRs beside a 3-wave/SIMD K1b
  const char* vo = getenv("TXV_VERIFY_CUS_OFF");
  const int off_cus = vo ? atoi(vo) : 0;
  if (off_cus > 0 && off_cus < ncu) {
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int i = 0; i < ncu; ++i) mask[i / 32] |= 1u << (i % 32);
    const int stride = ncu / off_cus;
    for (int i = 0, k = 0; i < ncu && k < off_cus; i += stride, ++k) mask[i / 32] &= ~(1u << (i % 32));
    return hipExtStreamCreateWithCUMask(&c->vstream, (uint32_t)mask.size(), mask.data());
  }
  const char* vp = getenv("TXV_VSTREAM_PRIO");
  if (vp && atoi(vp) > 0) {
    int lo = 0, hi = 0;
    if ((e = hipDeviceGetStreamPriorityRange(&lo, &hi)) != hipSuccess) return e;
    return hipStreamCreateWithPriority(&c->vstream, hipStreamNonBlocking, hi);
  }
  return hipStreamCreateWithFlags(&c->vstream, hipStreamNonBlocking);
}

}  // namespace

// ==================================================================== C ABI
extern "C" {

int txv_init(const txv_config* cfg, txv_ctx** out) {
  if (!out) return TXV_EINVAL;
  *out = nullptr;
  txv_ctx* c = new (std::nothrow) txv_ctx();
  if (!c) return TXV_ENOMEM;
  if (cfg) c->cfg = *cfg;
  else { c->cfg.device = -1; }
  if (!c->cfg.max_batch) c->cfg.max_batch = 1u << 20;
  if (!c->cfg.max_txs) c->cfg.max_txs = 1u << 20;
  if (!c->cfg.max_validators) c->cfg.max_validators = 1024;
  if (c->cfg.max_batch > (8u << 20)) { delete c; return TXV_EINVAL; }   // the device scans cover 8M votes
  c->hash_seed = ((uint64_t)std::random_device{}() << 32 | std::random_device{}()) ^ 0x7478666c6f77ULL;
  if (!c->cfg.max_msg_bytes) c->cfg.max_msg_bytes = 256;
  if (!c->cfg.table_budget_mb) c->cfg.table_budget_mb = 112u << 10;   // 112 GiB of the 288 GB HBM
  c->cfg_w = (c->cfg.flags & TXV_CFG_TABLE_W4) ? 4 : 0;
  if (TXV_CFG_WINDOW(c->cfg.flags)) c->cfg_w = (int)TXV_CFG_WINDOW(c->cfg.flags);
  if (c->cfg_w && !valid_window(c->cfg_w)) { delete c; return TXV_EINVAL; }
  if (TXV_CFG_LANE_VOTES(c->cfg.flags)) { c->lane_votes = TXV_CFG_LANE_VOTES(c->cfg.flags); c->lane_auto = false; }
  if (c->lane_votes != 1 && c->lane_votes != 2 && c->lane_votes != 4 && c->lane_votes != 8) { delete c; return TXV_EINVAL; }
  c->cfg_bw = (int)TXV_CFG_B_WINDOW(c->cfg.flags);
  if (c->cfg_bw && c->cfg_bw != 4 && !valid_window(c->cfg_bw) && c->cfg_bw != 20 && c->cfg_bw != 22 && c->cfg_bw != 24 &&
      c->cfg_bw != 26) {
    delete c;
    return TXV_EINVAL;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    delete c;
    return TXV_EDEVICE;
  }
  int dev = c->cfg.device;
  if (dev < 0) { if (hipGetDevice(&dev) != hipSuccess) dev = 0; }
  if (dev >= ndev) { delete c; return TXV_EINVAL; }
  c->device = dev;
  if (hipSetDevice(dev) != hipSuccess || create_streams(c) != hipSuccess) {
    delete c;
    return TXV_EDEVICE;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess) c->n_cus = prop.multiProcessorCount;
  if (build_base_table(c, 4) != TXV_OK) { txv_destroy(c); return TXV_EDEVICE; }
  {
    // host pack threads: TXV_HOST_THREADS, else min(16, hardware threads)
    unsigned nt = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    if (const char* e = getenv("TXV_HOST_THREADS")) nt = (unsigned)std::max(1, std::min(256, atoi(e)));
    c->pool.reset(new txv_host::WorkerPool(nt));
    c->profile_host = getenv("TXV_PROFILE_HOST") != nullptr;
    c->uniform_cols = !(getenv("TXV_UNIFORM_COLS") && atoi(getenv("TXV_UNIFORM_COLS")) == 0);
    c->derive_txkey = !(getenv("TXV_DERIVE_TXKEY") && atoi(getenv("TXV_DERIVE_TXKEY")) == 0);
    c->host_val = getenv("TXV_HOST_VAL") ? (atoi(getenv("TXV_HOST_VAL")) != 0) : -1;
  }
  *out = c;
  return TXV_OK;
}

void txv_destroy(txv_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
  if (c->key_stream) (void)hipStreamSynchronize(c->key_stream);
  if (c->vstream) (void)hipStreamSynchronize(c->vstream);
  for (auto& s : c->slots) {
    dfree(s.d_sig); dfree(s.d_msg); dfree(s.d_msg_len); dfree(s.d_val); dfree(s.d_set); dfree(s.d_flags);
    dfree(s.d_status); dfree(s.d_ok); dfree(s.d_pre); dfree(s.d_kbuf); dfree(s.d_rpts); dfree(s.d_order); hfree(s.h_order);
    hfree(s.h_sig); hfree(s.h_msg); hfree(s.h_msg_len); hfree(s.h_val); hfree(s.h_set); hfree(s.h_flags);
    hfree(s.h_status); hfree(s.h_out);
    hfree(s.h_addr); dfree(s.d_addr); hfree(s.h_addr_len); dfree(s.d_addr_len); hfree(s.h_sigraw); dfree(s.d_sigraw);
    hfree(s.h_sig_len); dfree(s.d_sig_len); hfree(s.h_nil); dfree(s.d_nil); hfree(s.h_txkey); dfree(s.d_txkey); hfree(s.h_vcode); dfree(s.d_vcode);
    dfree(s.d_entry); dfree(s.d_blk); dfree(s.d_ev_flag); dfree(s.d_mark); dfree(s.d_stamped); dfree(s.d_ev_tiles); hfree(s.h_ev); hfree(s.h_sum);
    hfree(s.h_fh); hfree(s.h_fs); hfree(s.h_fn); hfree(s.h_fo); hfree(s.h_fl); hfree(s.h_arena);
    dfree(s.d_fh); dfree(s.d_fs); dfree(s.d_fn); dfree(s.d_fo); dfree(s.d_fl); dfree(s.d_arena_th);
    for (auto& e : s.ev) if (e) (void)hipEventDestroy(e);
  }
  dfree(c->d_pubs); dfree(c->d_decode_ok); dfree(c->d_atables); dfree(c->d_vslot); dfree(c->d_addr); dfree(c->d_power);
  dfree(c->d_btable4); dfree(c->d_btable8); dfree(c->d_park); dfree(c->d_wctr); release_base_table(c->device, c->d_btable_wide); c->d_btable = nullptr; dfree(c->d_tmp_pubs); dfree(c->d_tmp_ok); dfree(c->d_tmp_tables); dfree(c->d_tmp_addr);
  dfree(c->d_cells); dfree(c->d_set_cross); dfree(c->d_set_sum);
  dfree(c->d_arena_sig); dfree(c->d_arena_height); dfree(c->d_arena_sec); dfree(c->d_arena_nanos); dfree(c->d_arena_val);
  dfree(c->d_arena_seq); dfree(c->d_arena_txkey); dfree(c->d_set_stamp); dfree(c->d_set_blk); dfree(c->d_set_digest); dfree(c->d_bitmap);
  dfree(c->d_set_entry); dfree(c->d_set_txkey); dfree(c->d_tab); dfree(c->d_keys); dfree(c->d_ctr);
  dfree(c->d_addr_slots); dfree(c->d_q);
  dfree(c->d_rshard); dfree(c->d_rw); dfree(c->d_rmax); dfree(c->d_rtot); hfree(c->h_rmeta);
  if (c->route_ev) (void)hipEventDestroy(c->route_ev);
  for (const auto& rg : c->registered) (void)hipHostUnregister((void*)rg.first);
  dfree(c->d_sk_scal); dfree(c->d_sk_araw); dfree(c->d_sk_prefix); dfree(c->d_sk_pub);
  dfree(c->d_chain); dfree(c->d_chain_sign);
  dfree(c->d_pk_sig); dfree(c->d_pk_len); dfree(c->d_pk_keys); hfree(c->h_pk_sig); hfree(c->h_pk_len); hfree(c->h_pk_keys);
  dfree(c->d_wd_wire); hfree(c->h_wd_wire); dfree(c->d_wd_off); hfree(c->h_wd_off); dfree(c->d_wd_len); hfree(c->h_wd_len);
  dfree(c->d_wd_out); hfree(c->h_wd_out); dfree(c->d_wd_span); hfree(c->h_wd_span);
  for (auto& e : c->wd_ev) if (e) (void)hipEventDestroy(e);
  for (auto& g : c->ing) {
    dfree(g.d_off); hfree(g.h_off); dfree(g.d_len); hfree(g.h_len); dfree(g.d_rec); dfree(g.d_span); hfree(g.h_span);
    dfree(g.d_status); hfree(g.h_status); dfree(g.d_keys); hfree(g.h_keys); dfree(g.d_sizes); hfree(g.h_sizes);
    dfree(g.d_list); hfree(g.h_list); dfree(g.d_max); hfree(g.h_max); dfree(g.d_pstat);
    if (g.kev) (void)hipEventDestroy(g.kev);
    if (g.uev) (void)hipEventDestroy(g.uev);
  }
  if (c->pk_ev) (void)hipEventDestroy(c->pk_ev);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->key_stream) (void)hipStreamDestroy(c->key_stream);
  if (c->vstream) (void)hipStreamDestroy(c->vstream);
  delete c;
}

const char* txv_last_error(txv_ctx* c) { return c ? c->err.copy() : "null context"; }

int txv_device_name(txv_ctx* c, char* buf, uint32_t cap) {
  if (!c || !buf || !cap) return TXV_EINVAL;
  hipDeviceProp_t p;
  HIP_TRY(c, hipGetDeviceProperties(&p, c->device));
  snprintf(buf, cap, "%s (%s, %d CUs)", p.name, p.gcnArchName, p.multiProcessorCount);
  return TXV_OK;
}

// The validator tables of a new set (txv_set_validators; the reference builds each tx's VoteSet
// from the current state's validators, txflow/service.go:200-207, and that set changes with the
// chain).  Keys some slot of the pool already holds keep their tables, in any order; the others
// take empty slots, then the slots of departed keys least recently in a set, and only they run
// K0 (0.89 s for 100 keys at radix 2^20, 872 MB each).  A set larger than the pool grows it
// (the kept tables copied device to device, an eighth spare; a full rebuild if HBM cannot hold
// both pools), a new window empties it.  Then the per-validator arrays: keys, decode flags,
// addresses (from the slots), vslot.
int assign_tables(txv_ctx* c, const uint8_t* pubs32, uint32_t n, int w) {
  // K0 rewrites slots an enqueued verify may still read
  for (hipStream_t st : {c->copy_stream, c->key_stream, c->vstream, c->stream}) HIP_TRY(c, hipStreamSynchronize(st));
  c->tables_built = 0;
  ++c->set_gen;
  const size_t words = table_words(w);
  int r;
  auto reset_pool = [&](uint32_t slots) -> int {
    c->tab_slots = 0;
    if ((r = dalloc(c, &c->d_atables, (size_t)slots * words))) return r;
    c->tab_slots = slots;
    c->slot_key.assign(slots, std::string());
    c->slot_ok.assign(slots, 0);
    c->slot_addr.assign((size_t)slots * 20, 0);
    c->slot_gen.assign(slots, 0);
    return TXV_OK;
  };
  if (c->pool_w != w) {
    c->pool_w = w;
    if ((r = reset_pool(0))) return r;
  }
  c->vslot.assign(n, UINT32_MAX);
  std::vector<char> taken(c->tab_slots, 0);
  {
    std::unordered_map<std::string, uint32_t> held;
    for (uint32_t sl = 0; sl < c->tab_slots; ++sl)
      if (!c->slot_key[sl].empty()) held.emplace(c->slot_key[sl], sl);
    for (uint32_t i = 0; i < n; ++i) {
      auto it = held.find(std::string((const char*)pubs32 + (size_t)i * 32, 32));
      if (it != held.end() && !taken[it->second]) { c->vslot[i] = it->second; taken[it->second] = 1; }
    }
  }
  if (n > c->tab_slots) {
    const uint64_t budget_slots = ((uint64_t)c->cfg.table_budget_mb << 20) / (words * 4);
    const uint32_t cap = c->tab_slots ? (uint32_t)std::max<uint64_t>(n, std::min<uint64_t>(budget_slots, n + std::max(1u, n / 8))) : n;
    uint32_t* np = nullptr;
    uint32_t kept = 0;
    for (char t : taken) kept += t != 0;
    if (kept && hipMalloc((void**)&np, (size_t)cap * words * 4) == hipSuccess) {
      // the kept tables to slots 0..kept-1 of the larger pool
      std::vector<uint32_t> moved(c->tab_slots, UINT32_MAX);
      std::vector<std::string> key(cap);
      std::vector<uint8_t> ok(cap, 0), addr((size_t)cap * 20, 0);
      uint32_t j = 0;
      for (uint32_t sl = 0; sl < c->tab_slots; ++sl) {
        if (!taken[sl]) continue;
        const hipError_t e = hipMemcpyAsync(np + (size_t)j * words, c->d_atables + (size_t)sl * words, words * 4,
                                            hipMemcpyDeviceToDevice, c->stream);
        if (e != hipSuccess) {
          (void)hipStreamSynchronize(c->stream);
          (void)hipFree(np);
          c->err = std::string("table pool copy: ") + hipGetErrorString(e);
          return TXV_EDEVICE;
        }
        key[j] = c->slot_key[sl];
        ok[j] = c->slot_ok[sl];
        memcpy(&addr[(size_t)j * 20], &c->slot_addr[(size_t)sl * 20], 20);
        moved[sl] = j++;
      }
      if (const hipError_t e = hipStreamSynchronize(c->stream); e != hipSuccess) {
        (void)hipFree(np);
        c->err = std::string("table pool copy: ") + hipGetErrorString(e);
        return TXV_EDEVICE;
      }
      (void)hipFree(c->d_atables);
      c->d_atables = np;
      c->tab_slots = cap;
      c->slot_key.swap(key);
      c->slot_ok.swap(ok);
      c->slot_addr.swap(addr);
      c->slot_gen.assign(cap, 0);
      for (auto& v : c->vslot) if (v != UINT32_MAX) v = moved[v];
      taken.assign(cap, 0);
      for (uint32_t k = 0; k < kept; ++k) taken[k] = 1;
    } else {
      (void)hipGetLastError();
      if ((r = reset_pool(0)) || (r = reset_pool(cap))) return r;   // free the old pool first
      c->vslot.assign(n, UINT32_MAX);
      taken.assign(cap, 0);
    }
  }
  // slots for the keys without one: empty slots first, then the least recently used
  std::vector<uint32_t> miss, free_sl;
  for (uint32_t i = 0; i < n; ++i) if (c->vslot[i] == UINT32_MAX) miss.push_back(i);
  for (uint32_t sl = 0; sl < c->tab_slots; ++sl) if (!taken[sl]) free_sl.push_back(sl);
  std::stable_sort(free_sl.begin(), free_sl.end(), [&](uint32_t a, uint32_t b) {
    const bool ea = c->slot_key[a].empty(), eb = c->slot_key[b].empty();
    return ea != eb ? ea : c->slot_gen[a] < c->slot_gen[b];
  });
  const uint32_t m = (uint32_t)miss.size();
  if (m > free_sl.size()) { c->err = "table pool"; return TXV_EDEVICE; }   // n <= tab_slots by construction
  if (m) {
    std::vector<uint8_t> mk((size_t)m * 32);
    std::vector<uint32_t> ms(m);
    for (uint32_t j = 0; j < m; ++j) {
      const uint32_t i = miss[j], sl = free_sl[j];
      memcpy(&mk[(size_t)j * 32], pubs32 + (size_t)i * 32, 32);
      ms[j] = sl;
      c->vslot[i] = sl;
      c->slot_key[sl] = std::string((const char*)pubs32 + (size_t)i * 32, 32);
    }
    uint32_t *d_k = nullptr, *d_s = nullptr, *d_a = nullptr;
    uint8_t* d_o = nullptr;
    auto fin = [&](int rr) { dfree(d_k); dfree(d_s); dfree(d_a); dfree(d_o); return rr; };
    if ((r = dalloc(c, &d_k, (size_t)m * 8)) || (r = dalloc(c, &d_s, m)) || (r = dalloc(c, &d_a, (size_t)m * 5)) ||
        (r = dalloc(c, &d_o, m)))
      return fin(r);
    std::vector<uint8_t> ok(m), addr((size_t)m * 20);
    hipError_t e;
    if ((e = hipMemcpyAsync(d_k, mk.data(), mk.size(), hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(d_s, ms.data(), (size_t)m * 4, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = txv_launch_build_tables_at(w, d_k, m, d_s, c->d_atables, d_o, d_a, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(ok.data(), d_o, m, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(addr.data(), d_a, (size_t)m * 20, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess) {
      for (uint32_t j = 0; j < m; ++j) c->slot_key[ms[j]].clear();   // their tables are not trustworthy
      c->err = std::string("K0: ") + hipGetErrorString(e);
      return fin(TXV_EDEVICE);
    }
    for (uint32_t j = 0; j < m; ++j) {
      c->slot_ok[ms[j]] = ok[j];
      memcpy(&c->slot_addr[(size_t)ms[j] * 20], &addr[(size_t)j * 20], 20);
    }
    c->tables_built = m;
    fin(TXV_OK);
  }
  for (uint32_t i = 0; i < n; ++i) c->slot_gen[c->vslot[i]] = c->set_gen;
  // per-validator arrays, in the set's order
  c->addrs.resize((size_t)n * 20);
  c->decode_ok.resize(n);
  for (uint32_t i = 0; i < n; ++i) {
    memcpy(&c->addrs[(size_t)i * 20], &c->slot_addr[(size_t)c->vslot[i] * 20], 20);
    c->decode_ok[i] = c->slot_ok[c->vslot[i]];
  }
  if ((r = dalloc(c, &c->d_pubs, (size_t)n * 8)) || (r = dalloc(c, &c->d_decode_ok, n)) ||
      (r = dalloc(c, &c->d_addr, (size_t)n * 5)) || (r = dalloc(c, &c->d_vslot, n)))
    return r;
  if (n) {
    HIP_TRY(c, hipMemcpyAsync(c->d_pubs, pubs32, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->d_decode_ok, c->decode_ok.data(), n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->d_addr, c->addrs.data(), (size_t)n * 20, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->d_vslot, c->vslot.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return TXV_OK;
}

int txv_set_validators(txv_ctx* c, const uint8_t* pubs32, const int64_t* powers, uint32_t n, const char* chain_id,
                       uint32_t chain_len) {
  if (!c || (!pubs32 && n) || (!powers && n)) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (n > c->cfg.max_validators) { c->err = "validator set exceeds max_validators"; return TXV_ECAPACITY; }
  c->n_vals = n;
  c->pubs.assign(pubs32, pubs32 + (size_t)n * 32);
  c->powers.assign(powers, powers + n);
  c->total = 0;
  for (uint32_t i = 0; i < n; ++i) c->total += powers[i];
  c->quorum = c->total * 2 / 3 + 1;
  c->chain.assign(chain_id ? chain_id : "", chain_id ? chain_len : 0);
  {
    int rr = upload_chain(c, c->chain.data(), (uint32_t)c->chain.size(), &c->d_chain, &c->d_chain_cap);
    if (rr) return rr;
  }
  int r;
  const int w = choose_window(c, n);
  if ((r = select_window(c, w)) || (r = assign_tables(c, pubs32, n, w))) return r;
  if ((r = dalloc(c, &c->d_power, n))) return r;
  if (n) HIP_TRY(c, hipMemcpyAsync(c->d_power, powers, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->addr_index.clear();
  for (uint32_t i = 0; i < n; ++i) c->addr_index.emplace(std::string((const char*)c->addrs.data() + 20 * i, 20), i);
  c->addr_tab.build(c->addrs.data(), n);
  // the same open-addressing table on the device (the AddVote path's validator lookup)
  c->addr_mask = (uint32_t)c->addr_tab.mask();
  if ((r = dalloc(c, &c->d_addr_slots, c->addr_tab.slots().size()))) return r;
  HIP_TRY(c, hipMemcpyAsync(c->d_addr_slots, c->addr_tab.slots().data(), c->addr_tab.slots().size() * 4,
                            hipMemcpyHostToDevice, c->stream));
  if ((r = alloc_tally(c))) return r;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return TXV_OK;
}

int txv_get_validator_info(txv_ctx* c, uint8_t* addr20_out, uint8_t* decode_ok_out, uint32_t cap) {
  if (!c) return TXV_EINVAL;
  const uint32_t n = std::min(cap, c->n_vals);
  if (addr20_out) memcpy(addr20_out, c->addrs.data(), (size_t)n * 20);
  if (decode_ok_out) memcpy(decode_ok_out, c->decode_ok.data(), n);
  return (int)c->n_vals;
}

int txv_verify_batch(txv_ctx* c, const txv_votes* v, const uint8_t* pubs32, uint8_t* status_out) {
  if (!c || !v || !status_out) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (v->n > c->cfg.max_batch) { c->err = "batch exceeds max_batch"; return TXV_ECAPACITY; }
  if (!pubs32 && !c->n_vals) { c->err = "no validator set"; return TXV_ESTATE; }
  Slot& s = c->slots[kVerifySlot];
  std::vector<int> lens;
  const uint32_t mx = encode_all(c, s, v, c->chain.data(), (uint32_t)c->chain.size(), lens);
  const uint32_t mw = std::max<uint32_t>(1, (mx + 7) / 8);
  int r = ensure_slot(c, s, v->n, mw);
  if (r) return r;
  s.n = v->n; s.n_pad = (v->n + 63) / 64 * 64; s.msg_words = mw;
  KeySet ks = registry_keys(c);
  uint32_t n_keys = c->n_vals;
  if (pubs32) {
    std::vector<uint32_t> kidx;
    std::vector<uint8_t> key_addr;
    if ((r = prepare_keys(c, pubs32, v->n, kidx, &key_addr, ks))) return r;
    n_keys = (uint32_t)(key_addr.size() / 20);
    for (uint32_t i = 0; i < v->n; ++i) {
      s.h_flags[i] = 0; s.h_set[i] = 0; s.h_val[i] = kidx[i];
      if (v->is_nil && v->is_nil[i]) { s.h_status[i] = TXV_ERR_NIL; continue; }
      const bool addr_ok = v->addr_len[i] == 20 && !memcmp(key_addr.data() + (size_t)kidx[i] * 20, v->addr + (size_t)i * 20, 20);
      if (!addr_ok) { s.h_status[i] = TXV_ERR_INVALID_VALIDATOR_ADDRESS; continue; }
      if (lens[i] < 0) { s.h_status[i] = TXV_ERR_SIGNBYTES; continue; }
      s.h_status[i] = 0xFF;
      s.h_flags[i] = TXV_FLAG_PENDING | (v->sig_len[i] == 64 ? TXV_FLAG_SIG64 : 0);
    }
  } else {
    for (uint32_t i = 0; i < v->n; ++i) {
      s.h_flags[i] = 0; s.h_set[i] = 0; s.h_val[i] = 0;
      if (v->is_nil && v->is_nil[i]) { s.h_status[i] = TXV_ERR_NIL; continue; }
      uint32_t vi = UINT32_MAX;
      if (v->addr_len[i] == 20) {
        auto a = c->addr_index.find(std::string((const char*)v->addr + (size_t)i * 20, 20));
        if (a != c->addr_index.end()) vi = a->second;
      }
      if (vi == UINT32_MAX) { s.h_status[i] = v->addr_len[i] ? TXV_ERR_UNKNOWN_VALIDATOR : TXV_ERR_EMPTY_ADDR; continue; }
      s.h_val[i] = vi;
      if (lens[i] < 0) { s.h_status[i] = TXV_ERR_SIGNBYTES; continue; }
      s.h_status[i] = 0xFF;
      s.h_flags[i] = TXV_FLAG_PENDING | (v->sig_len[i] == 64 ? TXV_FLAG_SIG64 : 0);
    }
  }
  build_order(c, s, n_keys);
  pack_columns(s, v, lens);
  std::vector<uint8_t> ok;
  if ((r = run_verify(c, s, ks, ok))) return r;
  for (uint32_t i = 0; i < v->n; ++i) {
    if (s.h_status[i] == 0xFF) status_out[i] = ok[i] == 1 ? TXV_ADDED : TXV_ERR_INVALID_SIGNATURE;
    else status_out[i] = s.h_status[i];
  }
  return TXV_OK;
}

int txv_verify_bytes(txv_ctx* c, const uint8_t* pubs32, const uint8_t* msgs, const uint32_t* msg_off,
                     const uint32_t* msg_len, const uint8_t* sigs64, const uint32_t* sig_len, uint32_t n,
                     uint8_t* ok_out) {
  if (!c || (n && (!pubs32 || !msg_off || !msg_len || !sigs64 || !sig_len || !ok_out))) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (n > c->cfg.max_batch) { c->err = "batch exceeds max_batch"; return TXV_ECAPACITY; }
  if (!n) return TXV_OK;
  Slot& s = c->slots[kVerifySlot];
  // the messages go to the device as they are (SHA-512 input R || A || msg)
  std::vector<int> lens(n);
  s.tmp_msg.clear();
  s.tmp_off.resize(n);
  uint32_t mx = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (msg_len[i] > TXV_MAX_RAW_MSG || (msg_len[i] && !msgs)) { c->err = "bad message length"; return TXV_EINVAL; }
    s.tmp_off[i] = s.tmp_msg.size();
    s.tmp_msg.insert(s.tmp_msg.end(), msgs + (msg_len[i] ? msg_off[i] : 0), msgs + (msg_len[i] ? msg_off[i] + msg_len[i] : 0));
    lens[i] = (int)msg_len[i];
    mx = std::max(mx, msg_len[i]);
  }
  const uint32_t mw = std::max<uint32_t>(1, (mx + 7) / 8);
  int r = ensure_slot(c, s, n, mw);
  if (r) return r;
  s.n = n; s.n_pad = (n + 63) / 64 * 64; s.msg_words = mw;
  std::vector<uint32_t> kidx;
  KeySet ks;
  if ((r = prepare_keys(c, pubs32, n, kidx, nullptr, ks))) return r;
  for (uint32_t i = 0; i < n; ++i) {
    s.h_set[i] = 0; s.h_val[i] = kidx[i]; s.h_status[i] = 0xFF;
    s.h_flags[i] = TXV_FLAG_PENDING | (sig_len[i] == 64 ? TXV_FLAG_SIG64 : 0);
  }
  build_order(c, s, kidx.empty() ? 1u : *std::max_element(kidx.begin(), kidx.end()) + 1);
  txv_votes view{};
  view.n = n; view.sig = sigs64; view.sig_len = sig_len;
  pack_columns(s, &view, lens);
  std::vector<uint8_t> ok;
  if ((r = run_verify(c, s, ks, ok))) return r;
  for (uint32_t i = 0; i < n; ++i) ok_out[i] = ok[i] == 1 ? 1 : 0;
  return TXV_OK;
}

int txv_add_votes(txv_ctx* c, const txv_votes* v, uint8_t* status_out, txv_commit_event* ev, uint32_t ev_cap,
                  uint32_t* n_ev) {
  if (!c || !v) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  uint64_t t;
  int r = submit_votes(c, v, &t);
  if (r) return r;
  return wait_votes(c, t, status_out, ev, ev_cap, n_ev);
}

int txv_submit_votes(txv_ctx* c, const txv_votes* v, uint64_t* ticket) {
  if (!c || !v || !ticket) return TXV_EINVAL;
  std::lock_guard<std::mutex> so(c->sub_mu);
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  return submit_votes(c, v, ticket);
}

int txv_wait_votes(txv_ctx* c, uint64_t ticket, uint8_t* status_out, txv_commit_event* ev, uint32_t ev_cap,
                   uint32_t* n_ev) {
  if (!c) return TXV_EINVAL;
  // wait for the batch's kernels without holding the context lock, so other threads' calls
  // (pool ingest keys, decode) proceed meanwhile; the slot cannot be reused before this ticket
  // is waited (submit refuses a slot whose ticket is set)
  hipEvent_t done = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(c, hipSetDevice(c->device));
    if (ticket) {
      const Slot& s = c->slots[(ticket - 1) % kSubmitRing];
      if (s.ticket == ticket && s.ran) done = s.ev[4];
    }
  }
  if (done) {
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipEventSynchronize(done));
  }
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  return wait_votes(c, ticket, status_out, ev, ev_cap, n_ev);
}

}  // extern "C"

namespace {

// Readers: set ids of n TxHashes (arena + off / len), looked up on the compute stream, i.e.
// after every batch submitted so far.  Scratch layout in d_q: keys (16 B padded) | off | len | ids.
int lookup_sets(txv_ctx* c, const uint8_t* arena, const uint32_t* off, const uint32_t* len, uint32_t n,
                std::vector<uint32_t>& ids) {
  ids.assign(n, TXV_NONE);
  if (!n || !c->d_tab) return TXV_OK;
  uint64_t kb = 0;
  for (uint32_t q = 0; q < n; ++q) kb += len[q];
  const uint64_t kpad = (kb + 16 + 15) / 16 * 16;
  const uint64_t need = kpad + 12ull * n;
  int r;
  if (need > c->q_cap) {
    if ((r = dalloc(c, &c->d_q, need))) return r;
    c->q_cap = need;
  }
  std::vector<uint8_t> hk(kpad, 0);
  std::vector<uint32_t> ho(n), hl(n);
  uint64_t at = 0;
  for (uint32_t q = 0; q < n; ++q) {
    if (len[q]) memcpy(hk.data() + at, arena + off[q], len[q]);
    ho[q] = (uint32_t)at;
    hl[q] = len[q];
    at += len[q];
  }
  uint32_t* d_off = reinterpret_cast<uint32_t*>(c->d_q + kpad);
  uint32_t* d_len = d_off + n;
  uint32_t* d_ids = d_len + n;
  HIP_TRY(c, hipMemcpyAsync(c->d_q, hk.data(), kpad, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(d_off, ho.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(d_len, hl.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
  const FlowState fs = flow_state(c);
  HIP_TRY(c, txv_flow_lookup(&fs, c->d_q, d_off, d_len, n, d_ids, c->stream));
  HIP_TRY(c, hipMemcpyAsync(ids.data(), d_ids, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return TXV_OK;
}

// sums, TxKeys and (optionally) every validator's accepted vote of n set ids
int read_sets(txv_ctx* c, const std::vector<uint32_t>& ids, std::vector<int64_t>* sums, std::vector<uint8_t>* txkeys,
              std::vector<AccRow>* rows) {
  const uint32_t n = (uint32_t)ids.size();
  if (!n || !c->n_vals) return TXV_OK;
  const size_t nv = c->n_vals;
  uint32_t* d_ids = nullptr; int64_t* d_sum = nullptr; uint32_t* d_tk = nullptr; AccRow* d_rows = nullptr;
  int r;
  if ((r = dalloc(c, &d_ids, n)) || (r = dalloc(c, &d_sum, n)) || (r = dalloc(c, &d_tk, (size_t)n * 8)) ||
      (rows && (r = dalloc(c, &d_rows, (size_t)n * nv)))) {
    dfree(d_ids); dfree(d_sum); dfree(d_tk); dfree(d_rows);
    return r;
  }
  const FlowState fs = flow_state(c);
  hipError_t e = hipMemcpyAsync(d_ids, ids.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = txv_flow_gather(&fs, d_ids, n, d_sum, d_tk, d_rows, c->stream);
  if (sums) sums->resize(n);
  if (txkeys) txkeys->resize((size_t)n * 32);
  if (rows) rows->resize((size_t)n * nv);
  if (e == hipSuccess && sums) e = hipMemcpyAsync(sums->data(), d_sum, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && txkeys) e = hipMemcpyAsync(txkeys->data(), d_tk, (size_t)n * 32, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && rows)
    e = hipMemcpyAsync(rows->data(), d_rows, (size_t)n * nv * sizeof(AccRow), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(d_ids); dfree(d_sum); dfree(d_tk); dfree(d_rows);
  HIP_TRY(c, e);
  return TXV_OK;
}

// the accepted votes of one set in validator order, as the commit encodings need them
int set_commit_votes(txv_ctx* c, uint32_t id, std::vector<AccRow>& rows, std::vector<txv_host::CommitVote>& out,
                     uint8_t txkey[32], int64_t* sum) {
  std::vector<int64_t> sums;
  std::vector<uint8_t> tks;
  int r = read_sets(c, std::vector<uint32_t>{id}, &sums, &tks, &rows);
  if (r) return r;
  memcpy(txkey, tks.data(), 32);
  *sum = sums[0];
  out.clear();
  for (const AccRow& a : rows) {
    if (a.val == TXV_NONE) continue;
    out.push_back(txv_host::CommitVote{a.height, a.ts_sec, a.ts_nanos, reinterpret_cast<const uint8_t*>(a.txkey),
                                       c->addrs.data() + (size_t)a.val * 20, reinterpret_cast<const uint8_t*>(a.sig)});
  }
  return TXV_OK;
}

}  // namespace

extern "C" {

int txv_query_txs(txv_ctx* c, const uint8_t* txhash, const uint32_t* off, const uint32_t* len, uint32_t n,
                  uint8_t* exists_out, int64_t* sum_out, uint8_t* maj23_out, uint8_t* txkey_out) {
  if (!c || (n && (!off || !len || (!txhash && n)))) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  std::vector<uint32_t> ids;
  int r = lookup_sets(c, txhash, off, len, n, ids);
  if (r) return r;
  std::vector<int64_t> sums;
  std::vector<uint8_t> tks;
  if ((r = read_sets(c, ids, &sums, txkey_out ? &tks : nullptr, nullptr))) return r;
  for (uint32_t q = 0; q < n; ++q) {
    const bool ex = ids[q] != TXV_NONE;
    if (exists_out) exists_out[q] = ex ? 1 : 0;
    const int64_t sm = ex && !sums.empty() ? sums[q] : 0;
    if (sum_out) sum_out[q] = sm;
    if (maj23_out) maj23_out[q] = ex && sm >= c->quorum ? 1 : 0;   // maj23 is sticky and sum only grows
    if (txkey_out) {
      if (ex && !tks.empty()) memcpy(txkey_out + (size_t)q * 32, tks.data() + (size_t)q * 32, 32);
      else memset(txkey_out + (size_t)q * 32, 0, 32);
    }
  }
  return TXV_OK;
}

int txv_query_tx(txv_ctx* c, const uint8_t* txhash, uint32_t len, int64_t* sum, uint8_t* maj23) {
  if (!c || (!txhash && len)) return TXV_EINVAL;
  const uint32_t off = 0;
  uint8_t ex = 0;
  int64_t sm = 0;
  uint8_t mj = 0;
  const uint8_t dummy = 0;
  int r = txv_query_txs(c, txhash ? txhash : &dummy, &off, &len, 1, &ex, &sm, &mj, nullptr);
  if (r) return r;
  if (!ex) return 0;
  if (sum) *sum = sm;
  if (maj23) *maj23 = mj;
  return 1;
}

int txv_get_votes(txv_ctx* c, const uint8_t* txhash, uint32_t len, uint32_t* val_out, uint64_t* seq_out,
                  uint8_t* sig_out, uint32_t cap, uint32_t* n_out) {
  if (!c || (!txhash && len) || !n_out) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  *n_out = 0;
  const uint32_t off = 0;
  const uint8_t dummy = 0;
  std::vector<uint32_t> ids;
  int r = lookup_sets(c, txhash ? txhash : &dummy, &off, &len, 1, ids);
  if (r) return r;
  if (ids[0] == TXV_NONE || !c->n_vals) return TXV_OK;
  std::vector<AccRow> rows;
  if ((r = read_sets(c, ids, nullptr, nullptr, &rows))) return r;
  uint32_t k = 0;
  for (const AccRow& a : rows) {
    if (a.val == TXV_NONE) continue;
    if (k < cap) {
      if (val_out) val_out[k] = a.val;
      if (seq_out) seq_out[k] = a.seq;
      if (sig_out) memcpy(sig_out + (size_t)k * 64, a.sig, 64);
    }
    ++k;
  }
  *n_out = k;
  return TXV_OK;
}

int txv_make_commit(txv_ctx* c, const uint8_t* txhash, uint32_t len, uint8_t* out, uint64_t cap, uint64_t* len_out) {
  if (!c || (!txhash && len) || !len_out) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  const uint32_t off = 0;
  const uint8_t dummy = 0;
  std::vector<uint32_t> ids;
  int r = lookup_sets(c, txhash ? txhash : &dummy, &off, &len, 1, ids);
  if (r) return r;
  if (ids[0] == TXV_NONE) { c->err = "no TxVoteSet for this TxHash"; return TXV_ESTATE; }
  std::vector<AccRow> rows;
  std::vector<txv_host::CommitVote> votes;
  uint8_t tk[32];
  int64_t sum;
  if ((r = set_commit_votes(c, ids[0], rows, votes, tk, &sum))) return r;
  if (sum < c->quorum) { c->err = "MakeCommit without +2/3 (the reference panics)"; return TXV_ESTATE; }
  const int64_t L = txv_host::commit_bytes(nullptr, txhash, len, votes.data(), (uint32_t)votes.size());
  if (L < 0) { c->err = "amino time error in a commit vote"; return TXV_EINVAL; }
  *len_out = (uint64_t)L;
  if ((uint64_t)L > cap || !out) return TXV_ECAPACITY;
  txv_host::commit_bytes(out, txhash, len, votes.data(), (uint32_t)votes.size());
  return TXV_OK;
}

int txv_save_tx_bytes(txv_ctx* c, const uint8_t* txhash, uint32_t len, uint8_t* out, uint64_t cap, uint64_t lens_out[4]) {
  if (!c || (!txhash && len) || !lens_out) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  const uint32_t off = 0;
  const uint8_t dummy = 0;
  std::vector<uint32_t> ids;
  int r = lookup_sets(c, txhash ? txhash : &dummy, &off, &len, 1, ids);
  if (r) return r;
  if (ids[0] == TXV_NONE) { c->err = "no TxVoteSet for this TxHash"; return TXV_ESTATE; }
  std::vector<AccRow> rows;
  std::vector<txv_host::CommitVote> votes;
  uint8_t tk[32];
  int64_t sum;
  if ((r = set_commit_votes(c, ids[0], rows, votes, tk, &sum))) return r;
  if (sum < c->quorum) { c->err = "SaveTx -> MakeCommit without +2/3 (the reference panics)"; return TXV_ESTATE; }
  const int64_t cl = txv_host::commit_bytes(nullptr, txhash, len, votes.data(), (uint32_t)votes.size());
  if (cl < 0) { c->err = "amino time error in a commit vote"; return TXV_EINVAL; }
  lens_out[0] = txv_host::store_key(nullptr, 'H', txhash, len);
  lens_out[1] = txv_host::txvoteset_bytes(nullptr, txhash, len, tk);
  lens_out[2] = txv_host::store_key(nullptr, 'C', txhash, len);
  lens_out[3] = (uint64_t)cl;
  const uint64_t total = lens_out[0] + lens_out[1] + lens_out[2] + lens_out[3];
  if (total > cap || !out) return TXV_ECAPACITY;
  uint8_t* p = out;
  p += txv_host::store_key(p, 'H', txhash, len);
  p += txv_host::txvoteset_bytes(p, txhash, len, tk);
  p += txv_host::store_key(p, 'C', txhash, len);
  txv_host::commit_bytes(p, txhash, len, votes.data(), (uint32_t)votes.size());
  return TXV_OK;
}

uint32_t txv_num_tx_sets(txv_ctx* c) { return c ? c->n_sets_host : 0; }
int64_t txv_total_power(txv_ctx* c) { return c ? c->total : 0; }

int txv_signbytes(int64_t height, const uint8_t* txhash, uint32_t txhash_len, int64_t ts_sec, int32_t ts_nanos,
                  const char* chain_id, uint32_t chain_len, uint8_t* out, uint32_t cap) {
  if (!out) return TXV_EINVAL;
  return txv_host::sign_bytes(out, cap, height, txhash, txhash_len, ts_sec, ts_nanos, (const uint8_t*)chain_id,
                              chain_len);
}

int txv_txvote_size(int64_t height, uint32_t txhash_len, int64_t ts_sec, int32_t ts_nanos, uint32_t addr_len,
                    uint32_t sig_len) {
  return txv_host::txvote_size(height, txhash_len, ts_sec, ts_nanos, addr_len, sig_len);
}

int txv_keygen(txv_ctx* c, const uint8_t* seeds32, uint32_t n, uint8_t* pubs_out) {
  if (!c || (!seeds32 && n)) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  uint32_t* d_seeds = nullptr;
  int r;
  if ((r = dalloc(c, &d_seeds, (size_t)n * 8)) || (r = dalloc(c, &c->d_sk_scal, (size_t)n * 8)) ||
      (r = dalloc(c, &c->d_sk_araw, (size_t)n * 8)) || (r = dalloc(c, &c->d_sk_prefix, (size_t)n * 8)) ||
      (r = dalloc(c, &c->d_sk_pub, (size_t)n * 8)))
    return r;
  if (n) {
    HIP_TRY(c, hipMemcpyAsync(d_seeds, seeds32, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, txv_launch_keygen(d_seeds, n, c->d_btable4,c->d_sk_scal, c->d_sk_araw, c->d_sk_prefix, c->d_sk_pub,
                                 c->stream));
    if (pubs_out) HIP_TRY(c, hipMemcpyAsync(pubs_out, c->d_sk_pub, (size_t)n * 32, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  dfree(d_seeds);
  c->n_signers = n;
  return TXV_OK;
}

int txv_sign_votes(txv_ctx* c, const txv_votes* v, const uint32_t* signer, const char* chain_id, uint32_t chain_len,
                   uint8_t* sig_out) {
  if (!c || !v || !signer || !sig_out) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  for (uint32_t i = 0; i < v->n; ++i)
    if (signer[i] >= c->n_signers) { c->err = "signer index out of range"; return TXV_EINVAL; }
  Slot& s = c->slots[kSignerSlot];
  // SignBytes are built on the device (txv_k_signbytes), the same encoder the AddVote path uses
  std::vector<int> lens(v->n);
  uint32_t mx = 0;
  uint64_t ae = 0;
  for (uint32_t i = 0; i < v->n; ++i) {
    if (v->is_nil && v->is_nil[i]) { lens[i] = -2; continue; }
    lens[i] = txv_host::sign_bytes_len(v->height[i], v->txhash_len[i], v->ts_sec[i], v->ts_nanos[i], chain_len);
    if (lens[i] > 0) mx = std::max(mx, (uint32_t)lens[i]);
    ae = std::max<uint64_t>(ae, (uint64_t)v->txhash_off[i] + v->txhash_len[i]);
  }
  const uint32_t mw = std::max<uint32_t>(1, (mx + 7) / 8);
  int r = ensure_slot(c, s, v->n, mw);
  if (r) return r;
  s.n = v->n; s.n_pad = (v->n + 63) / 64 * 64; s.msg_words = mw; s.n_work = 0;
  for (uint32_t i = 0; i < s.n_pad; ++i) {
    const bool in = i < v->n;
    s.h_val[i] = in ? signer[i] : 0; s.h_flags[i] = 0; s.h_set[i] = 0; s.h_status[i] = 0;
    s.h_msg_len[i] = in && lens[i] > 0 ? (uint32_t)lens[i] : 0;
    for (int j = 0; j < 16; ++j) s.h_sig[(size_t)j * s.n_pad + i] = 0;
  }
  if ((r = upload_chain(c, chain_id, chain_len, &c->d_chain_sign, &c->d_chain_sign_cap)) ||
      (r = encode_signbytes_device(c, s, v, c->d_chain_sign, chain_len, ae)) || (r = upload_slot(c, s)))
    return r;
  HIP_TRY(c, hipStreamWaitEvent(c->stream, s.ev[3], 0));
  SignArgs a{};
  a.n = s.n; a.n_pad = s.n_pad; a.msg_words = s.msg_words; a.msg = s.d_msg; a.msg_len = s.d_msg_len; a.val = s.d_val;
  a.prefix = c->d_sk_prefix; a.araw = c->d_sk_araw; a.pub = c->d_sk_pub; a.btable = c->d_btable4; a.sig = s.d_sig;
  HIP_TRY(c, txv_launch_sign(&a, c->stream));
  HIP_TRY(c, hipMemcpyAsync(s.h_sig, s.d_sig, (size_t)16 * s.n_pad * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  for (uint32_t i = 0; i < v->n; ++i)
    for (int j = 0; j < 16; ++j) {
      const uint32_t w = s.h_sig[(size_t)j * s.n_pad + i];
      uint8_t* o = sig_out + (size_t)i * 64 + 4 * j;
      o[0] = (uint8_t)w; o[1] = (uint8_t)(w >> 8); o[2] = (uint8_t)(w >> 16); o[3] = (uint8_t)(w >> 24);
    }
  return TXV_OK;
}

int txv_stage(txv_ctx* c, uint32_t slot, const txv_votes* v) {
  if (!c || !v || slot >= kStagedSlots) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->slots[slot].ticket) { c->err = "slot holds a txv_submit_votes batch in flight"; return TXV_ESTATE; }
  int r = stage_add(c, slot, v);
  if (r) return r;
  HIP_TRY(c, hipStreamSynchronize(c->copy_stream));   // resident before any timed run
  return TXV_OK;
}

int txv_run_staged(txv_ctx* c, uint32_t slot, float* ms) {
  if (!c || slot >= kStagedSlots) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->slots[slot].ticket) { c->err = "slot holds a txv_submit_votes batch in flight"; return TXV_ESTATE; }
  return run_slot(c, slot, ms);
}

int txv_fetch_staged(txv_ctx* c, uint32_t slot, uint8_t* status_out, txv_commit_event* ev, uint32_t ev_cap,
                     uint32_t* n_ev) {
  if (!c || slot >= kStagedSlots) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  return fetch_slot(c, slot, status_out, ev, ev_cap, n_ev);
}

int txv_set_commit_sink(txv_ctx* c, uint32_t slot, void* dst_dev, uint32_t n_sets_cap) {
  if (!c || slot >= kStagedSlots || (dst_dev && !n_sets_cap)) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  Slot& s = c->slots[slot];
  if (s.ticket) { c->err = "slot holds a txv_submit_votes batch in flight"; return TXV_ESTATE; }
  if (s.launched) HIP_TRY(c, hipEventSynchronize(s.ev[4]));   // no pack into the old sink still pending
  s.sink = static_cast<uint32_t*>(dst_dev);
  s.sink_cap = dst_dev ? n_sets_cap : 0;
  return TXV_OK;
}

int txv_slot_kernel_ms(txv_ctx* c, uint32_t slot, float* ms4) {
  if (!c || !ms4 || slot >= kStagedSlots) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  Slot& s = c->slots[slot];
  if (!s.launched) { c->err = "slot never ran"; return TXV_ESTATE; }
  HIP_TRY(c, hipEventSynchronize(s.ev[4]));
  return slot_kernel_ms(c, s, ms4);
}

int txv_slot_verify_ms(txv_ctx* c, uint32_t slot, float* ms2) {
  if (!c || !ms2 || slot >= kStagedSlots) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  Slot& s = c->slots[slot];
  if (!s.launched) { c->err = "slot never ran"; return TXV_ESTATE; }
  HIP_TRY(c, hipEventSynchronize(s.ev[4]));
  if (TXV_K1A_ON_KEY_STREAM) {
    HIP_TRY(c, hipEventElapsedTime(&ms2[0], s.ev[8], s.ev[1]));
    HIP_TRY(c, hipEventElapsedTime(&ms2[1], s.ev[7], s.ev[2]));
  } else {
    HIP_TRY(c, hipEventElapsedTime(&ms2[0], s.ev[7], s.ev[8]));
    HIP_TRY(c, hipEventElapsedTime(&ms2[1], s.ev[8], s.ev[2]));
  }
  return TXV_OK;
}

int txv_commit_bitmap(txv_ctx* c, void** dev_ptr, uint64_t* bytes) {
  if (!c || !dev_ptr || !bytes) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (!c->d_ctr) { c->err = "no validator set"; return TXV_ESTATE; }
  const FlowState fs = flow_state(c);   // derived from the stake sums after every submitted batch
  HIP_TRY(c, txv_flow_bitmap(&fs, c->d_bitmap, (c->cfg.max_txs + 31) / 32, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  *dev_ptr = c->d_bitmap;
  *bytes = (uint64_t)(c->cfg.max_txs + 31) / 32 * 4;
  return TXV_OK;
}

int txv_host_register(txv_ctx* c, void* ptr, uint64_t bytes) {
  if (!c || !ptr || !bytes) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipHostRegister(ptr, bytes, hipHostRegisterDefault));
  std::lock_guard<std::mutex> rg(c->reg_mu);
  c->registered.emplace_back((uintptr_t)ptr, bytes);
  return TXV_OK;
}

int txv_host_unregister(txv_ctx* c, void* ptr) {
  if (!c || !ptr) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  for (size_t k = 0; k < c->registered.size(); ++k)
    if (c->registered[k].first == (uintptr_t)ptr) {
      // no DMA of an in-flight batch may still read it
      HIP_TRY(c, hipStreamSynchronize(c->copy_stream));
      HIP_TRY(c, hipHostUnregister(ptr));
      std::lock_guard<std::mutex> rg(c->reg_mu);
      c->registered.erase(c->registered.begin() + (long)k);
      return TXV_OK;
    }
  c->err = "pointer was not registered";
  return TXV_EINVAL;
}

uint64_t txv_commit_state_bytes(uint32_t n_sets_cap) {
  return 8ull + (uint64_t)(n_sets_cap + 31) / 32 * 4 + 8ull * n_sets_cap + 16ull * n_sets_cap;
}

int txv_pack_commit_state(txv_ctx* c, void* dst_dev, uint32_t n_sets_cap) {
  if (!c || !dst_dev) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (!c->d_ctr) { c->err = "no validator set"; return TXV_ESTATE; }
  const FlowState fs = flow_state(c);
  HIP_TRY(c, txv_flow_pack(&fs, static_cast<uint32_t*>(dst_dev), (n_sets_cap + 31) / 32, n_sets_cap, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return TXV_OK;
}

int txv_read_commit_state(txv_ctx* c, void* dst_host, uint32_t n_sets_cap) {
  if (!c || !dst_host) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (!c->d_ctr) { c->err = "no validator set"; return TXV_ESTATE; }
  const uint64_t bytes = txv_commit_state_bytes(n_sets_cap);
  if (bytes > c->q_cap) {
    int r;
    if ((r = dalloc(c, &c->d_q, bytes))) return r;
    c->q_cap = bytes;
  }
  const FlowState fs = flow_state(c);
  HIP_TRY(c, txv_flow_pack(&fs, reinterpret_cast<uint32_t*>(c->d_q), (n_sets_cap + 31) / 32, n_sets_cap, c->stream));
  HIP_TRY(c, hipMemcpyAsync(dst_host, c->d_q, bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return TXV_OK;
}

int txv_commit_state_pack_host(uint32_t n_sets, const uint8_t* committed, const int64_t* sums, const uint8_t* digests,
                               uint32_t n_sets_cap, void* dst) {
  if (!dst || n_sets > n_sets_cap || (n_sets && (!committed || !sums))) return TXV_EINVAL;
  uint32_t* d = static_cast<uint32_t*>(dst);
  const uint32_t bm = (n_sets_cap + 31) / 32;
  memset(d, 0, txv_commit_state_bytes(n_sets_cap));
  d[0] = n_sets;
  d[1] = 1;
  uint8_t* dg = reinterpret_cast<uint8_t*>(d + 2 + bm + 2 * (size_t)n_sets_cap);
  for (uint32_t s = 0; s < n_sets; ++s) {
    if (committed[s]) d[2 + s / 32] |= 1u << (s % 32);
    memcpy(d + 2 + bm + 2 * s, &sums[s], 8);
    if (digests) memcpy(dg + 16 * (size_t)s, digests + 16 * (size_t)s, 16);
  }
  return TXV_OK;
}

int txv_commit_state_unpack(const void* src, uint32_t n_sets_cap, uint32_t* n_sets, uint8_t* committed, int64_t* sums,
                            uint8_t* digests, uint32_t cap) {
  if (!src || !n_sets) return TXV_EINVAL;
  const uint32_t* d = static_cast<const uint32_t*>(src);
  const uint32_t bm = (n_sets_cap + 31) / 32;
  if (d[0] > n_sets_cap || d[1] != 1) return TXV_EINVAL;
  *n_sets = d[0];
  const uint8_t* dg = reinterpret_cast<const uint8_t*>(d + 2 + bm + 2 * (size_t)n_sets_cap);
  for (uint32_t s = 0; s < d[0] && s < cap; ++s) {
    if (committed) committed[s] = (uint8_t)((d[2 + s / 32] >> (s % 32)) & 1u);
    if (sums) memcpy(&sums[s], d + 2 + bm + 2 * s, 8);
    if (digests) memcpy(digests + 16 * (size_t)s, dg + 16 * (size_t)s, 16);
  }
  return TXV_OK;
}

int txv_shard_of(const uint8_t* txhash, const uint32_t* off, const uint32_t* len, uint32_t n, uint32_t n_shards,
                 uint32_t* shard_out) {
  if (!n_shards || (n && (!txhash || !off || !len || !shard_out))) return TXV_EINVAL;
  const uint32_t nt = std::max(1u, std::min<uint32_t>(16, n / 4096));
  std::vector<std::thread> th;
  auto work = [&](uint32_t t) {
    for (uint32_t i = (uint32_t)((uint64_t)n * t / nt); i < (uint32_t)((uint64_t)n * (t + 1) / nt); ++i) {
      uint8_t h[32];
      txv_sha256_bytes(txhash + off[i], len[i], h);
      shard_out[i] = h[0] % n_shards;
    }
  };
  for (uint32_t t = 1; t < nt; ++t) {
    try {
      th.emplace_back(work, t);
    } catch (const std::system_error&) {
      work(t);   // no thread to spare: the range runs here
    }
  }
  work(0);
  for (auto& x : th) x.join();
  return TXV_OK;
}

}  // extern "C"

namespace {

// ---- the multi-GPU ingest route (include/txvote.h txv_route_admitted; kernels_route.hip) ----
uint32_t route_flags(const txv_votes* v) {
  return (v->txkey ? TXV_ROUTE_TXKEY : 0u) | (v->is_nil ? TXV_ROUTE_NIL : 0u);
}

// txv_route_admitted's steps (route_mu held by the caller).  Stage: the batch's columns into the
// route slot (without its signatures when sig_later: txv_route_checked takes them from the pool's
// flight slot), c->mu held inside.
int route_stage(txv_ctx* c, const txv_votes* v, bool sig_later, uint64_t stride) {
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  txv_votes w = *v;
  if (sig_later) w.sig = nullptr;
  int r;
  if ((r = stage_add(c, kRouteSlot, &w, true))) return r;
  Slot& s = c->slots[kRouteSlot];
  const uint64_t need = txv_route_bytes(v->n, s.arena_end, route_flags(v));
  if (stride < need) {
    c->err = "route stride below txv_route_bytes(n, TxHash arena extent, flags) = " + std::to_string(need);
    return TXV_EINVAL;
  }
  return TXV_OK;
}

// Launch: the pool's statuses either given on the host (st: uploaded beside the columns, with the
// signatures too when they were left out) or already in the slot's pre-check column (st null,
// dev_status: txv_route_checked), then the three route kernels; waits for the metas.
int route_launch(txv_ctx* c, const txv_votes* v, const uint8_t* st, bool dev_status, bool sig_later, uint32_t G,
                 void* dst, uint64_t stride, txv_route_meta* meta) {
  const uint32_t n = v->n;
  const uint32_t flags = route_flags(v);
  int r;
  hipEvent_t done;
  {
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(c, hipSetDevice(c->device));
    Slot& s = c->slots[kRouteSlot];
    if (st && n) {   // the pool's statuses beside the columns (the slot's pre-check column is free here)
      memcpy(s.h_status, st, n);
      HIP_TRY(c, hipMemcpyAsync(s.d_pre, s.h_status, n, hipMemcpyHostToDevice, c->copy_stream));
      if (sig_later) {          // the signatures the pool's slot no longer holds, from the caller
        const bool reg = is_registered(c, v->sig, (uint64_t)n * 64);
        if (!reg) c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
          memcpy(s.h_sigraw + (size_t)lo * 64, v->sig + (size_t)lo * 64, (size_t)(hi - lo) * 64);
        }, 4096);
        HIP_TRY(c, hipMemcpyAsync(s.d_sigraw, reg ? (const void*)v->sig : (const void*)s.h_sigraw, (size_t)n * 64,
                                  hipMemcpyHostToDevice, c->copy_stream));
      }
      HIP_TRY(c, hipEventRecord(s.ev[3], c->copy_stream));
    }
    const uint32_t nw = (n + 63) / 64;
    if (n > c->route_n_cap) {
      if ((r = dalloc(c, &c->d_rshard, std::max<uint32_t>(n, 64)))) return r;
      c->route_n_cap = n;
    }
    if ((uint64_t)nw * G > c->route_w_cap) {
      if ((r = dalloc(c, &c->d_rw, 2 * (size_t)std::max<uint32_t>(nw, 1) * G))) return r;
      c->route_w_cap = std::max<uint32_t>(nw, 1) * G;
    }
    if (!c->d_rmax) {
      if ((r = dalloc(c, &c->d_rmax, 256)) || (r = dalloc(c, &c->d_rtot, 512)) ||
          (r = halloc_mapped(c, &c->h_rmeta, &c->m_rmeta, 256)))
        return r;
      HIP_TRY(c, hipEventCreateWithFlags(&c->route_ev, hipEventDisableTiming));
    }
    RouteArgs a{};
    a.n = n; a.G = G; a.nw = nw;
    a.height = s.d_fh; a.ts_sec = s.d_fs; a.ts_nanos = s.d_fn; a.th_off = s.d_fo; a.th_len = s.d_fl; a.th = s.d_arena_th;
    a.addr = s.d_addr; a.addr_len = s.d_addr_len; a.sig = s.d_sigraw; a.sig_len = s.d_sig_len;
    a.txkey = s.has_txkey ? s.d_txkey : nullptr;
    a.nil = s.has_nil ? s.d_nil : nullptr;
    a.status = (st || dev_status) ? s.d_pre : nullptr;
    a.flags = flags;
    a.shard = c->d_rshard; a.wcnt = c->d_rw; a.wbytes = c->d_rw + (size_t)std::max<uint32_t>(nw, 1) * G;
    a.maxhl = c->d_rmax; a.tot = c->d_rtot;
    a.dst = static_cast<uint8_t*>(dst); a.stride = stride; a.meta = c->m_rmeta;
    // on the key stream (CheckTx's engine and the batches' prep run there too): after the uploads
    HIP_TRY(c, hipStreamWaitEvent(c->key_stream, s.ev[3], 0));
    HIP_TRY(c, txv_launch_route(&a, c->key_stream));
    HIP_TRY(c, hipEventRecord(s.ev[4], c->key_stream));   // the slot's next staging waits for it
    HIP_TRY(c, hipEventRecord(c->route_ev, c->key_stream));
    s.launched = true;
    s.staged = false;
    done = c->route_ev;
  }
  HIP_TRY(c, hipEventSynchronize(done));
  memcpy(meta, c->h_rmeta, (size_t)G * sizeof(txv_route_meta));
  return TXV_OK;
}

int route_admitted(txv_ctx* c, const txv_votes* v, const uint8_t* st, uint32_t G, void* dst, uint64_t stride,
                   txv_route_meta* meta) {
  int r;
  if ((r = route_stage(c, v, false, stride))) return r;
  return route_launch(c, v, st, false, false, G, dst, stride, meta);
}

// the receiving rank: a route buffer (on this context's device) into AddVote slot `slot`, by
// device-to-device copies on the copy stream (stage_add's counterpart: nothing crosses PCIe)
int stage_routed(txv_ctx* c, uint32_t slot, const uint8_t* buf, const txv_route_meta* m) {
  if (!c->n_vals) { c->err = "no validator set"; return TXV_ESTATE; }
  if (m->n > c->cfg.max_batch) { c->err = "batch exceeds max_batch"; return TXV_ECAPACITY; }
  if (c->poisoned) { c->err = "a TxFlow capacity was exceeded: txv_reset_flow first"; return TXV_ECAPACITY; }
  if (m->arena_bytes >= (1ull << 32)) { c->err = "TxHash arena >= 4 GiB"; return TXV_EINVAL; }
  Slot& s = c->slots[slot];
  const uint32_t n = m->n;
  uint64_t off[txv_route::kNCols];
  if (txv_route::layout(n, m->arena_bytes, m->flags, off) != m->bytes) { c->err = "route meta: inconsistent sizes"; return TXV_EINVAL; }
  const uint32_t mw = (signbytes_bound(m->max_txhash_len, (uint32_t)c->chain.size()) + 7) / 8;
  int r;
  if ((r = ensure_slot(c, s, n, mw)) || (r = ensure_flow_slot(c, s, n))) return r;
  const uint64_t ae = m->arena_bytes;
  if (ae + 16 > s.arena_cap) {
    const size_t cap = std::max<size_t>((size_t)ae + 16, s.arena_cap * 2);
    if ((r = halloc(c, &s.h_arena, cap)) || (r = dalloc(c, &s.d_arena_th, cap))) return r;
    s.arena_cap = cap;
  }
  s.n = n; s.n_pad = (n + 63) / 64 * 64; s.msg_words = mw;
  s.has_nil = (m->flags & TXV_ROUTE_NIL) != 0;
  s.has_txkey = (m->flags & TXV_ROUTE_TXKEY) != 0;
  s.host_val = false;
  s.arena_end = ae;
  s.seq_base = c->seq_next;
  c->seq_next += n;
  if (s.launched) HIP_TRY(c, hipStreamWaitEvent(c->copy_stream, s.ev[4], 0));   // its last chain has ended
  struct { int col; void* dev; size_t elem; } cols[] = {
      {txv_route::kHeight, s.d_fh, 8}, {txv_route::kSec, s.d_fs, 8}, {txv_route::kNanos, s.d_fn, 4},
      {txv_route::kOff, s.d_fo, 4}, {txv_route::kLen, s.d_fl, 4}, {txv_route::kAddrLen, s.d_addr_len, 4},
      {txv_route::kSigLen, s.d_sig_len, 4}, {txv_route::kAddr, s.d_addr, 20}, {txv_route::kSig, s.d_sigraw, 64},
      {txv_route::kTxKey, s.has_txkey ? s.d_txkey : nullptr, 32}, {txv_route::kNil, s.has_nil ? s.d_nil : nullptr, 1}};
  for (const auto& k : cols)
    if (k.dev && n) HIP_TRY(c, hipMemcpyAsync(k.dev, buf + off[k.col], (size_t)n * k.elem, hipMemcpyDeviceToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_arena_th, buf + off[txv_route::kArena], ae + 16, hipMemcpyDeviceToDevice, c->copy_stream));
  c->staged_bytes = 0;
  HIP_TRY(c, hipEventRecord(s.ev[3], c->copy_stream));   // run_slot's kernels wait for this
  s.staged = true; s.ran = false; s.fill_mask = 0; s.fill_key = false;
  return TXV_OK;
}

// host: shard of every admitted vote, then each rank's buffer in arrival order (route.h)
int route_pack_host(const txv_votes* v, const uint8_t* st, uint32_t G, uint8_t* dst, uint64_t stride,
                    txv_route_meta* meta) {
  const uint32_t n = v->n;
  const uint32_t flags = route_flags(v);
  std::vector<uint8_t> shard(n, 0xFF);
  std::vector<uint32_t> cnt(G, 0), mx(G, 0);
  std::vector<uint64_t> ab(G, 0);
  uint64_t ae = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (!(v->is_nil && v->is_nil[i])) ae = std::max<uint64_t>(ae, (uint64_t)v->txhash_off[i] + v->txhash_len[i]);
    if (st && st[i] != TXV_POOL_OK) continue;
    const uint32_t len = (v->is_nil && v->is_nil[i]) ? 0u : v->txhash_len[i];
    uint8_t h[32];
    txv_sha256_bytes(len ? v->txhash + v->txhash_off[i] : nullptr, len, h);
    const uint32_t r = h[0] % G;
    shard[i] = (uint8_t)r;
    ++cnt[r];
    ab[r] += len;
    mx[r] = std::max(mx[r], len);
  }
  if (stride < txv_route_bytes(n, ae, flags)) return TXV_EINVAL;
  std::vector<uint64_t> pos(G, 0), bpos(G, 0);
  for (uint32_t r = 0; r < G; ++r) {
    uint64_t off[txv_route::kNCols];
    const uint64_t total = txv_route::layout(cnt[r], ab[r], flags, off);
    uint8_t* b = dst + (size_t)r * stride;
    memset(b, 0, total);
    const uint64_t hdr[8] = {txv_route::kMagic, cnt[r], ab[r], flags, mx[r], total, 0, 0};
    memcpy(b, hdr, 64);
    meta[r] = txv_route_meta{cnt[r], mx[r], flags, 0, ab[r], total};
  }
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t r = shard[i];
    if (r == 0xFF) continue;
    uint64_t off[txv_route::kNCols];
    (void)txv_route::layout(cnt[r], ab[r], flags, off);
    uint8_t* b = dst + (size_t)r * stride;
    const uint64_t j = pos[r]++;
    const bool nil = v->is_nil && v->is_nil[i];
    const uint32_t len = nil ? 0u : v->txhash_len[i];
    const uint32_t bo = (uint32_t)bpos[r];
    memcpy(b + off[txv_route::kHeight] + 8 * j, &v->height[i], 8);
    memcpy(b + off[txv_route::kSec] + 8 * j, &v->ts_sec[i], 8);
    memcpy(b + off[txv_route::kNanos] + 4 * j, &v->ts_nanos[i], 4);
    memcpy(b + off[txv_route::kOff] + 4 * j, &bo, 4);
    memcpy(b + off[txv_route::kLen] + 4 * j, &len, 4);
    memcpy(b + off[txv_route::kAddrLen] + 4 * j, &v->addr_len[i], 4);
    memcpy(b + off[txv_route::kSigLen] + 4 * j, &v->sig_len[i], 4);
    memcpy(b + off[txv_route::kAddr] + 20 * j, v->addr + (size_t)i * 20, 20);
    memcpy(b + off[txv_route::kSig] + 64 * j, v->sig + (size_t)i * 64, 64);
    if (flags & TXV_ROUTE_TXKEY) memcpy(b + off[txv_route::kTxKey] + 32 * j, v->txkey + (size_t)i * 32, 32);
    if (flags & TXV_ROUTE_NIL) b[off[txv_route::kNil] + j] = nil ? 1 : 0;
    if (len) memcpy(b + off[txv_route::kArena] + bo, v->txhash + v->txhash_off[i], len);
    bpos[r] += len;
  }
  return TXV_OK;
}

}  // namespace

extern "C" {

uint64_t txv_route_bytes(uint32_t n, uint64_t arena_bytes, uint32_t flags) {
  uint64_t off[txv_route::kNCols];
  return txv_route::layout(n, arena_bytes, flags, off);
}

int txv_route_admitted(txv_ctx* c, const txv_votes* v, const uint8_t* pool_status, uint32_t n_shards, void* dst_dev,
                       uint64_t stride, txv_route_meta* meta_out) {
  if (!c || !v || !dst_dev || !meta_out || !n_shards || n_shards > 255) return TXV_EINVAL;
  if (v->n && (!v->height || !v->txhash || !v->txhash_off || !v->txhash_len || !v->ts_sec || !v->ts_nanos || !v->addr ||
               !v->addr_len || !v->sig || !v->sig_len))
    return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->route_mu);
  return route_admitted(c, v, pool_status, n_shards, dst_dev, stride, meta_out);
}

int txv_route_pack_host(const txv_votes* v, const uint8_t* pool_status, uint32_t n_shards, void* dst, uint64_t stride,
                        txv_route_meta* meta_out) {
  if (!v || !dst || !meta_out || !n_shards || n_shards > 255) return TXV_EINVAL;
  if (v->n && (!v->height || !v->txhash || !v->txhash_off || !v->txhash_len || !v->ts_sec || !v->ts_nanos || !v->addr ||
               !v->addr_len || !v->sig || !v->sig_len))
    return TXV_EINVAL;
  return route_pack_host(v, pool_status, n_shards, static_cast<uint8_t*>(dst), stride, meta_out);
}

int txv_route_view(const void* buf, uint64_t bytes, txv_votes* out) {
  if (!buf || !out || bytes < 64) return TXV_EINVAL;
  const uint8_t* b = static_cast<const uint8_t*>(buf);
  uint64_t h[8];
  memcpy(h, b, 64);
  if (h[0] != txv_route::kMagic || h[1] > 0xFFFFFFFFull) return TXV_EINVAL;
  uint64_t off[txv_route::kNCols];
  const uint64_t total = txv_route::layout(h[1], h[2], (uint32_t)h[3], off);
  if (total != h[5] || total > bytes) return TXV_EINVAL;
  const uint32_t flags = (uint32_t)h[3];
  out->n = (uint32_t)h[1];
  out->height = reinterpret_cast<const int64_t*>(b + off[txv_route::kHeight]);
  out->ts_sec = reinterpret_cast<const int64_t*>(b + off[txv_route::kSec]);
  out->ts_nanos = reinterpret_cast<const int32_t*>(b + off[txv_route::kNanos]);
  out->txhash_off = reinterpret_cast<const uint32_t*>(b + off[txv_route::kOff]);
  out->txhash_len = reinterpret_cast<const uint32_t*>(b + off[txv_route::kLen]);
  out->addr_len = reinterpret_cast<const uint32_t*>(b + off[txv_route::kAddrLen]);
  out->sig_len = reinterpret_cast<const uint32_t*>(b + off[txv_route::kSigLen]);
  out->addr = b + off[txv_route::kAddr];
  out->sig = b + off[txv_route::kSig];
  out->txkey = (flags & TXV_ROUTE_TXKEY) ? b + off[txv_route::kTxKey] : nullptr;
  out->is_nil = (flags & TXV_ROUTE_NIL) ? b + off[txv_route::kNil] : nullptr;
  out->txhash = b + off[txv_route::kArena];
  return TXV_OK;
}

int txv_submit_routed(txv_ctx* c, const void* buf_dev, const txv_route_meta* meta, uint64_t* ticket) {
  if (!c || !buf_dev || !meta || !ticket) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  const uint64_t t = c->next_ticket;
  const uint32_t slot = (uint32_t)((t - 1) % kSubmitRing);
  Slot& s = c->slots[slot];
  if (s.ticket) { c->err = "four batches already in flight: wait for the oldest one first"; return TXV_ESTATE; }
  int r;
  if ((r = stage_routed(c, slot, static_cast<const uint8_t*>(buf_dev), meta))) return r;
  if ((r = run_slot(c, slot, nullptr))) return r;
  s.ticket = t;
  c->next_ticket = t + 1;
  *ticket = t;
  return TXV_OK;
}

int txv_reset_tally(txv_ctx* c) {
  if (!c) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (!c->n_vals) return TXV_OK;
  return reset_tally(c, true);
}

// SHA-256 of an arbitrary byte string on the host (signatures longer than 64 bytes only)
static void sha256_host(const uint8_t* p, uint64_t n, uint8_t out[32]) {
  uint32_t st[8], w[16];
  txv::sha256_init(st);
  const uint64_t total = n + 9, nblk = (total + 63) / 64;
  for (uint64_t b = 0; b < nblk; ++b) {
    uint8_t blk[64];
    for (int j = 0; j < 64; ++j) {
      const uint64_t g = b * 64 + (uint64_t)j;
      blk[j] = g < n ? p[g] : (g == n ? 0x80 : 0);
    }
    if (b == nblk - 1)
      for (int j = 0; j < 8; ++j) blk[56 + j] = (uint8_t)((n * 8) >> (56 - 8 * j));
    for (int t = 0; t < 16; ++t)
      w[t] = ((uint32_t)blk[4 * t] << 24) | ((uint32_t)blk[4 * t + 1] << 16) | ((uint32_t)blk[4 * t + 2] << 8) | blk[4 * t + 3];
    txv::sha256_block(st, w);
  }
  for (int j = 0; j < 8; ++j)
    for (int b = 0; b < 4; ++b) out[4 * j + b] = (uint8_t)(st[j] >> (24 - 8 * b));
}

}  // extern "C"

// internal (pool.cpp): SHA-256 on the host
void txv_sha256_bytes(const uint8_t* p, uint64_t n, uint8_t out[32]) { sha256_host(p, n, out); }

// the context's persistent host workers for pool.cpp's order-independent passes (no thread
// creation per call)
void txv_host_parallel_for(txv_ctx* c, uint32_t n, const std::function<void(uint32_t, uint32_t)>& fn,
                           uint32_t min_chunk) {
  if (c && c->pool) c->pool->parallel_for(n, fn, min_chunk);
  else if (n) fn(0, n);
}

// a worker pool of its own for a TxVotePool used without a context (TXV_HOST_THREADS, else
// min(16, hardware threads)), created on its first batch-path call
std::shared_ptr<void> txv_host_workers_new() {
  unsigned nt = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  if (const char* e = getenv("TXV_HOST_THREADS")) nt = (unsigned)std::max(1, std::min(256, atoi(e)));
  return std::shared_ptr<void>(new txv_host::WorkerPool(nt),
                               [](void* w) { delete static_cast<txv_host::WorkerPool*>(w); });
}
void txv_host_workers_for(void* w, uint32_t n, const std::function<void(uint32_t, uint32_t)>& fn,
                          uint32_t min_chunk) {
  static_cast<txv_host::WorkerPool*>(w)->parallel_for(n, fn, min_chunk);
}

int txv_sig_keys_overlap(txv_ctx* c, const txv_votes* v, const uint8_t* sig_full, const uint64_t* sig_full_off,
                         uint8_t* keys_out, const std::function<void()>& overlap);
extern "C" {

int txv_sig_keys(txv_ctx* c, const txv_votes* v, const uint8_t* sig_full, const uint64_t* sig_full_off,
                 uint8_t* keys_out) {
  return txv_sig_keys_overlap(c, v, sig_full, sig_full_off, keys_out, nullptr);
}

}  // extern "C"

// txv_sig_keys, running `overlap` (host work of the caller's, e.g. the pool's TxVote.Size pass)
// while the key stream hashes
int txv_sig_keys_overlap(txv_ctx* c, const txv_votes* v, const uint8_t* sig_full, const uint64_t* sig_full_off,
                         uint8_t* keys_out, const std::function<void()>& overlap) {
  if (!c || !v || (v->n && (!v->sig || !v->sig_len || !keys_out))) return TXV_EINVAL;
  const uint32_t n = v->n;
  // its own lock: the pool's keys (TxVotePool.CheckTx on the ingest thread) must not wait for a
  // txv_submit_votes staging on another thread, nor hold it up over the key stream's round trip;
  // the key stream takes both threads' work in enqueue order, the worker pool both threads' passes
  std::lock_guard<std::mutex> g(c->pk_mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (!n) return TXV_OK;
  if (n > c->pk_cap) {
    int r;
    if ((r = dalloc(c, &c->d_pk_sig, (size_t)n * 16)) || (r = dalloc(c, &c->d_pk_len, n)) ||
        (r = dalloc(c, &c->d_pk_keys, (size_t)n * 8)) || (r = halloc(c, &c->h_pk_sig, (size_t)n * 16)) ||
        (r = halloc(c, &c->h_pk_len, n)) || (r = halloc(c, &c->h_pk_keys, (size_t)n * 8)))
      return r;
    c->pk_cap = n;
  }
  if (!c->pk_ev) HIP_TRY(c, hipEventCreateWithFlags(&c->pk_ev, hipEventDisableTiming));
  static const bool prof = getenv("TXV_PROFILE_HOST") != nullptr;
  std::chrono::steady_clock::time_point tp[5];
  if (prof) tp[0] = std::chrono::steady_clock::now();
  if (!sig_full || !sig_full_off) {   // a signature > 64 bytes cannot be hashed: reject before any GPU work
    std::atomic<bool> lg{false};
    c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
      bool l = false;
      for (uint32_t i = lo; i < hi; ++i) l |= v->sig_len[i] > 64;
      if (l) lg.store(true, std::memory_order_relaxed);
    }, 8192);
    if (lg.load()) { c->err = "signature > 64 bytes without sig_full"; return TXV_EINVAL; }
  }
  // a failure after the first enqueue drains the key stream before returning: its copies read
  // the pinned buffers the next call overwrites
#define PK_TRY(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      c->err = std::string(#x) + ": " + hipGetErrorString(e_);                            \
      (void)hipStreamSynchronize(c->key_stream);                                           \
      return TXV_EDEVICE;                                                                  \
    }                                                                                      \
  } while (0)
  // in up to 4 chunks: chunk k+1 is staged into pinned memory while chunk k is uploaded, hashed
  // and read back on the key stream (a signature longer than 64 bytes is hashed on the host below)
  // (every chunk is four queued operations of ~10-20 us launch / DMA latency each: a C5 batch of
  // 64k keys -- 4 MB up, 2 MB down -- waited 0.35-0.43 ms in four chunks, so chunking starts at
  // 256k votes, where the staging copy it overlaps is worth it; TXV_KEYS_CHUNKS overrides)
  static const uint32_t forced_k = getenv("TXV_KEYS_CHUNKS") ? (uint32_t)std::max(1, std::min(8, atoi(getenv("TXV_KEYS_CHUNKS")))) : 0u;
  const uint32_t K = forced_k ? std::min(forced_k, std::max(n, 1u)) : (n >= 262144 ? 4u : 1u);
  std::atomic<bool> long_sig{false};
  // signature / length columns inside caller memory registered with txv_host_register are DMA'd
  // from there (no staging copy)
  bool reg;
  {
    std::lock_guard<std::mutex> lk(c->reg_mu);
    reg = is_registered(c, v->sig, (uint64_t)n * 64) && is_registered(c, v->sig_len, (uint64_t)n * 4);
  }
  for (uint32_t k = 0; k < K; ++k) {
    const uint32_t c0 = (uint32_t)((uint64_t)n * k / K), c1 = (uint32_t)((uint64_t)n * (k + 1) / K);
    c->pool->parallel_for(c1 - c0, [&](uint32_t lo, uint32_t hi) {
      lo += c0; hi += c0;
      if (!reg) {
        memcpy(c->h_pk_sig + (size_t)lo * 16, v->sig + (size_t)lo * 64, (size_t)(hi - lo) * 64);
        memcpy(c->h_pk_len + lo, v->sig_len + lo, (size_t)(hi - lo) * 4);
      }
      bool lg = false;
      for (uint32_t i = lo; i < hi; ++i) lg |= v->sig_len[i] > 64;
      if (lg) long_sig.store(true, std::memory_order_relaxed);
    }, 2048);
    const void* src_sig = reg ? (const void*)(v->sig + (size_t)c0 * 64) : (const void*)(c->h_pk_sig + (size_t)c0 * 16);
    const void* src_len = reg ? (const void*)(v->sig_len + c0) : (const void*)(c->h_pk_len + c0);
    PK_TRY(hipMemcpyAsync(c->d_pk_sig + (size_t)c0 * 16, src_sig, (size_t)(c1 - c0) * 64, hipMemcpyHostToDevice,
                          c->key_stream));
    PK_TRY(hipMemcpyAsync(c->d_pk_len + c0, src_len, (size_t)(c1 - c0) * 4, hipMemcpyHostToDevice, c->key_stream));
    PK_TRY(txv_launch_sig_keys(c->d_pk_sig + (size_t)c0 * 16, c->d_pk_len + c0, c1 - c0,
                                   c->d_pk_keys + (size_t)c0 * 8, c->key_stream));
    PK_TRY(hipMemcpyAsync(c->h_pk_keys + (size_t)c0 * 8, c->d_pk_keys + (size_t)c0 * 8, (size_t)(c1 - c0) * 32,
                              hipMemcpyDeviceToHost, c->key_stream));
  }
  // the wait below is for this event, not the stream: a batch's prep / SignBytes that another
  // thread's txv_submit_votes enqueues on the key stream after these keys is not waited for
  // (work enqueued before them still is: the stream is in order)
  PK_TRY(hipEventRecord(c->pk_ev, c->key_stream));
  if (prof) tp[1] = std::chrono::steady_clock::now();
  if (overlap) overlap();
  if (prof) tp[2] = std::chrono::steady_clock::now();
  PK_TRY(hipEventSynchronize(c->pk_ev));
#undef PK_TRY
  if (prof) tp[3] = std::chrono::steady_clock::now();
  c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
    memcpy(keys_out + (size_t)lo * 32, c->h_pk_keys + (size_t)lo * 8, (size_t)(hi - lo) * 32);
    if (long_sig.load(std::memory_order_relaxed))
      for (uint32_t i = lo; i < hi; ++i)
        if (v->sig_len[i] > 64) sha256_host(sig_full + sig_full_off[i], v->sig_len[i], keys_out + (size_t)i * 32);
  }, 2048);
  if (prof) {
    tp[4] = std::chrono::steady_clock::now();
    auto ms = [&](int a) { return std::chrono::duration<double, std::milli>(tp[a + 1] - tp[a]).count(); };
    fprintf(stderr, "[txv keys] stage+enqueue=%.3f overlap=%.3f sync=%.3f copy_out=%.3f ms\n", ms(0), ms(1), ms(2), ms(3));
  }
  return TXV_OK;
}

extern "C" {

// CPUs of the NUMA node the GPU hangs off (sysfs local_cpulist of its PCI function)
static bool gpu_local_cpuset(int dev, cpu_set_t* out) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, dev) != hipSuccess) return false;
  for (char* p = bus; *p; ++p) *p = (char)tolower(*p);
  std::string path = std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist";
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  char line[4096] = {0};
  const bool got = fgets(line, sizeof line, f) != nullptr;
  fclose(f);
  if (!got) return false;
  CPU_ZERO(out);
  int n = 0;
  for (char* tok = strtok(line, ",\n"); tok; tok = strtok(nullptr, ",\n")) {
    int a = -1, b = -1;
    if (sscanf(tok, "%d-%d", &a, &b) == 2) { for (int i = a; i <= b && i < CPU_SETSIZE; ++i) { CPU_SET(i, out); ++n; } }
    else if (sscanf(tok, "%d", &a) == 1 && a < CPU_SETSIZE) { CPU_SET(a, out); ++n; }
  }
  return n > 0;
}

int txv_bind_host_numa(txv_ctx* c) {
  if (!c) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  cpu_set_t local, allowed, both;
  if (!gpu_local_cpuset(c->device, &local)) { c->err = "GPU NUMA locality unknown"; return TXV_ESTATE; }
  if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) { c->err = "sched_getaffinity failed"; return TXV_ESTATE; }
  CPU_AND(&both, &local, &allowed);
  if (CPU_COUNT(&both) == 0) { c->err = "no allowed CPU on the GPU's NUMA node"; return TXV_ESTATE; }
  if (sched_setaffinity(0, sizeof both, &both) != 0 || !c->pool->set_affinity(both)) {
    c->err = "setting the CPU affinity failed";
    return TXV_ESTATE;
  }
  return TXV_OK;
}

int txv_reset_flow(txv_ctx* c) {
  if (!c) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (!c->n_vals) return TXV_OK;
  return reset_tally(c, false);
}

void* txv_flow_stream(txv_ctx* c) { return c ? (void*)c->stream : nullptr; }

int txv_sync(txv_ctx* c) {
  if (!c) return TXV_EINVAL;
  HIP_TRY(c, hipStreamSynchronize(c->vstream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return TXV_OK;
}

int txv_copy_commit_bitmap(txv_ctx* c, void* dst_dev, uint64_t bytes) {
  if (!c || !dst_dev) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (!c->d_ctr) { c->err = "no validator set"; return TXV_ESTATE; }
  const uint64_t have = (uint64_t)(c->cfg.max_txs + 31) / 32 * 4;
  const FlowState fs = flow_state(c);
  HIP_TRY(c, txv_flow_bitmap(&fs, static_cast<uint32_t*>(dst_dev), (uint32_t)(std::min(bytes, have) / 4), c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return TXV_OK;
}

int txv_copy_set_sums(txv_ctx* c, void* dst_dev, uint32_t n_sets) {
  if (!c || (!dst_dev && n_sets)) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  const uint32_t n = std::min(n_sets, c->cfg.max_txs);
  if (n) HIP_TRY(c, hipMemcpyAsync(dst_dev, c->d_set_sum, (size_t)n * 8, hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return TXV_OK;
}

int txv_valu_probe(txv_ctx* c, double* add_lane_ops_per_s, double* mad_lane_ops_per_s) {
  if (!c) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  const uint32_t blocks = (uint32_t)c->n_cus * 8;   // 32 waves per CU
  const int iters = 1 << 14;
  uint32_t* d = nullptr;
  int r;
  if ((r = dalloc(c, &d, (size_t)blocks * 256))) return r;
  hipEvent_t e0, e1;
  HIP_TRY(c, hipEventCreate(&e0));
  HIP_TRY(c, hipEventCreate(&e1));
  double* outs[2] = {add_lane_ops_per_s, mad_lane_ops_per_s};
  for (int op = 0; op < 2; ++op) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      HIP_TRY(c, hipEventRecord(e0, c->stream));
      HIP_TRY(c, txv_launch_valu_probe(op, d, blocks, iters, c->stream));
      HIP_TRY(c, hipEventRecord(e1, c->stream));
      HIP_TRY(c, hipEventSynchronize(e1));
      float ms;
      HIP_TRY(c, hipEventElapsedTime(&ms, e0, e1));
      if (rep && ms < best) best = ms;   // first launch is warm-up
    }
    const double lane_ops = (double)blocks * 256.0 * iters * 8.0;
    if (outs[op]) *outs[op] = lane_ops / (best * 1e-3);
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  dfree(d);
  return TXV_OK;
}

int txv_table_window(txv_ctx* c) { return c ? c->tab_w : TXV_EINVAL; }
int txv_validator_tables_built(txv_ctx* c) { return c ? (int)c->tables_built : TXV_EINVAL; }
int64_t txv_staged_bytes(txv_ctx* c) { return c ? (int64_t)c->staged_bytes : TXV_EINVAL; }
int txv_base_window(txv_ctx* c) { return c ? c->b_w : TXV_EINVAL; }

int txv_fe_selftest(txv_ctx* c, const uint32_t* a, const uint32_t* b, uint32_t* out, uint32_t n, int op) {
  if (!c || !a || !b || !out) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  uint32_t *da = nullptr, *db = nullptr, *dout = nullptr;
  int r;
  if ((r = dalloc(c, &da, (size_t)n * 8)) || (r = dalloc(c, &db, (size_t)n * 8)) || (r = dalloc(c, &dout, (size_t)n * 8)))
    return r;
  HIP_TRY(c, hipMemcpyAsync(da, a, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(db, b, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, txv_launch_fe_selftest(da, db, dout, n, op, c->stream));
  HIP_TRY(c, hipMemcpyAsync(out, dout, (size_t)n * 32, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  dfree(da); dfree(db); dfree(dout);
  return TXV_OK;
}

}  // extern "C"

// ---- TxVoteMessage wire decode (Reactor.Receive / decodeMsg, txvotepool/reactor.go:170-190, 278-284) ----

namespace {

// records of txv_k_decode_msgs (TXV_WIRE_REC_WORDS u32 per message, txv_device.h)
size_t wire_out_bytes(uint32_t cap) { return (size_t)cap * TXV_WIRE_REC_WORDS * 4; }

// amino nameToDisfix("tendermint/txvotepool/TxVoteMessage") (go-amino, external): SHA-256 of the
// registered name, leading zero bytes skipped, 3 disambiguation bytes, zero bytes skipped, 4 prefix bytes
void txvote_msg_disfix(uint32_t* disamb, uint32_t* prefix) {
  static const char name[] = "tendermint/txvotepool/TxVoteMessage";
  uint8_t h[32];
  sha256_host(reinterpret_cast<const uint8_t*>(name), sizeof name - 1, h);
  int i = 0;
  while (h[i] == 0) ++i;
  *disamb = (uint32_t)h[i] | ((uint32_t)h[i + 1] << 8) | ((uint32_t)h[i + 2] << 16);
  i += 3;
  while (h[i] == 0) ++i;
  *prefix = le32(h + i);
}

}  // namespace

extern "C" {

int txv_decode_stage(txv_ctx* c, const uint8_t* wire, uint64_t wire_bytes, const uint64_t* msg_off,
                     const uint32_t* msg_len, uint32_t n) {
  if (!c || (n && (!wire || !msg_off || !msg_len))) return TXV_EINVAL;
  if (wire_bytes >= (1ull << 32)) { c->err = "wire buffer >= 4 GiB"; return TXV_EINVAL; }
  for (uint32_t i = 0; i < n; ++i)   // every message inside the buffer: the kernel trusts these
    if (msg_off[i] > wire_bytes || msg_len[i] > wire_bytes - msg_off[i]) {
      c->err = "message " + std::to_string(i) + " outside the wire buffer";
      return TXV_EINVAL;
    }
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  int r;
  if (n > c->wd_cap) {
    const uint32_t cap = std::max<uint32_t>(n, 1024);
    if ((r = dalloc(c, &c->d_wd_off, cap)) || (r = halloc(c, &c->h_wd_off, cap)) || (r = dalloc(c, &c->d_wd_len, cap)) ||
        (r = halloc(c, &c->h_wd_len, cap)) || (r = dalloc(c, &c->d_wd_out, wire_out_bytes(cap))) ||
        (r = halloc(c, &c->h_wd_out, wire_out_bytes(cap))) ||
        (r = dalloc(c, &c->d_wd_span, (size_t)2 * ((cap + TXV_WIRE_BLOCK - 1) / TXV_WIRE_BLOCK))) ||
        (r = halloc(c, &c->h_wd_span, (size_t)2 * ((cap + TXV_WIRE_BLOCK - 1) / TXV_WIRE_BLOCK))))
      return r;
    c->wd_cap = cap;
  }
  if (wire_bytes + 128 > c->wd_bytes_cap) {   // 128 bytes of padding: kernels_wire.hip row reads
    const uint64_t cap = std::max<uint64_t>(wire_bytes + 128, 1u << 20);
    if ((r = dalloc(c, &c->d_wd_wire, cap)) || (r = halloc(c, &c->h_wd_wire, cap))) return r;
    c->wd_bytes_cap = cap;
  }
  if (!c->wd_ev[0]) { HIP_TRY(c, hipEventCreate(&c->wd_ev[0])); HIP_TRY(c, hipEventCreate(&c->wd_ev[1])); }
  c->pool->parallel_for((uint32_t)((wire_bytes + 65535) / 65536), [&](uint32_t lo, uint32_t hi) {
    const uint64_t a = (uint64_t)lo * 65536, b = std::min<uint64_t>((uint64_t)hi * 65536, wire_bytes);
    memcpy(c->h_wd_wire + a, wire + a, b - a);
  }, 16);
  memset(c->h_wd_wire + wire_bytes, 0, 128);
  memcpy(c->h_wd_off, msg_off, (size_t)n * 8);
  memcpy(c->h_wd_len, msg_len, (size_t)n * 4);
  // per-chunk byte spans (the kernel stages a chunk into LDS when its span fits)
  const uint32_t n_chunks = (n + TXV_WIRE_BLOCK - 1) / TXV_WIRE_BLOCK;
  c->pool->parallel_for(n_chunks, [&](uint32_t lo_c, uint32_t hi_c) {
    for (uint32_t k = lo_c; k < hi_c; ++k) {
      uint64_t lo = ~0ull, hi = 0;
      for (uint32_t i = k * TXV_WIRE_BLOCK; i < std::min<uint32_t>(n, (k + 1) * TXV_WIRE_BLOCK); ++i)
        if (msg_len[i]) { lo = std::min(lo, msg_off[i]); hi = std::max(hi, msg_off[i] + msg_len[i]); }
      if (hi == 0) lo = 0;
      c->h_wd_span[2 * k] = lo & ~15ull;
      c->h_wd_span[2 * k + 1] = hi;
    }
  }, 64);
  HIP_TRY(c, hipMemcpyAsync(c->d_wd_wire, c->h_wd_wire, wire_bytes + 128, hipMemcpyHostToDevice, c->key_stream));
  if (n) {
    HIP_TRY(c, hipMemcpyAsync(c->d_wd_off, c->h_wd_off, (size_t)n * 8, hipMemcpyHostToDevice, c->key_stream));
    HIP_TRY(c, hipMemcpyAsync(c->d_wd_len, c->h_wd_len, (size_t)n * 4, hipMemcpyHostToDevice, c->key_stream));
    HIP_TRY(c, hipMemcpyAsync(c->d_wd_span, c->h_wd_span, (size_t)n_chunks * 16, hipMemcpyHostToDevice, c->key_stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->key_stream));
  c->wd_n = n;
  c->wd_bytes = wire_bytes;
  c->wd_ran = false;
  return TXV_OK;
}

int txv_decode_run(txv_ctx* c, uint32_t max_msg_bytes, uint32_t reps, float* kernel_ms_avg) {
  if (!c) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (!c->wd_ev[0]) { c->err = "txv_decode_run before txv_decode_stage"; return TXV_ESTATE; }
  WireArgs a{};
  a.n = c->wd_n;
  a.max_msg_bytes = max_msg_bytes;
  txvote_msg_disfix(&a.disamb, &a.prefix);
  a.wire = c->d_wd_wire; a.off = c->d_wd_off; a.len = c->d_wd_len;
  a.rec = reinterpret_cast<uint32_t*>(c->d_wd_out);
  a.n_chunks = (a.n + TXV_WIRE_BLOCK - 1) / TXV_WIRE_BLOCK;
  a.span = c->d_wd_span;
  // persistent grid: 5 resident blocks per CU (LDS: 28.7 KB of staging per 128-message block)
  const uint32_t grid = (uint32_t)c->n_cus * (getenv("TXV_WIRE_BPC") ? (uint32_t)atoi(getenv("TXV_WIRE_BPC")) : 5u);
  if (!reps) reps = 1;
  HIP_TRY(c, hipEventRecord(c->wd_ev[0], c->key_stream));
  for (uint32_t k = 0; k < reps; ++k) HIP_TRY(c, txv_launch_decode_msgs(&a, grid, c->key_stream));
  HIP_TRY(c, hipEventRecord(c->wd_ev[1], c->key_stream));
  HIP_TRY(c, hipEventSynchronize(c->wd_ev[1]));
  if (kernel_ms_avg) {
    float ms = 0;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->wd_ev[0], c->wd_ev[1]));
    *kernel_ms_avg = ms / (float)reps;
  }
  c->wd_ran = true;
  return TXV_OK;
}

int txv_decode_fetch(txv_ctx* c, const txv_wire_votes* out) {
  if (!c || !out) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (!c->wd_ran) { c->err = "txv_decode_fetch before txv_decode_run"; return TXV_ESTATE; }
  const uint32_t n = c->wd_n;
  if (!n) return TXV_OK;
  HIP_TRY(c, hipMemcpyAsync(c->h_wd_out, c->d_wd_out, wire_out_bytes(n), hipMemcpyDeviceToHost, c->key_stream));
  HIP_TRY(c, hipStreamSynchronize(c->key_stream));
  const uint32_t* rec = reinterpret_cast<const uint32_t*>(c->h_wd_out);
  c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {   // records -> the caller's columns
    for (uint32_t i = lo; i < hi; ++i) {
      const uint32_t* r = rec + (size_t)i * TXV_WIRE_REC_WORDS;
      if (out->status) out->status[i] = (uint8_t)r[0];
      if (out->height) out->height[i] = (int64_t)((uint64_t)r[1] | ((uint64_t)r[2] << 32));
      if (out->ts_sec) out->ts_sec[i] = (int64_t)((uint64_t)r[3] | ((uint64_t)r[4] << 32));
      if (out->ts_nanos) out->ts_nanos[i] = (int32_t)r[5];
      if (out->txhash_off) out->txhash_off[i] = r[6];
      if (out->txhash_len) out->txhash_len[i] = r[7];
      if (out->addr_len) out->addr_len[i] = r[8];
      if (out->sig_off) out->sig_off[i] = r[9];
      if (out->sig_len) out->sig_len[i] = r[10];
      if (out->txkey) memcpy(out->txkey + (size_t)i * 32, r + 11, 32);
      if (out->addr) memcpy(out->addr + (size_t)i * 20, r + 19, 20);
      if (out->sig) memcpy(out->sig + (size_t)i * 64, r + 24, 64);
    }
  }, 8192);
  return TXV_OK;
}

int txv_decode_msgs(txv_ctx* c, const uint8_t* wire, uint64_t wire_bytes, const uint64_t* msg_off,
                    const uint32_t* msg_len, uint32_t n, uint32_t max_msg_bytes, const txv_wire_votes* out) {
  if (!c || !out) return TXV_EINVAL;
  int r = txv_decode_stage(c, wire, wire_bytes, msg_off, msg_len, n);
  if (!r) r = txv_decode_run(c, max_msg_bytes, 1, nullptr);
  if (!r) r = txv_decode_fetch(c, out);
  return r;
}

}  // extern "C"

uint32_t txv_pool_max_msg_bytes(txv_pool* p);  // pool.cpp
int txv_pool_check_dev_submit(txv_pool* p, txv_ctx* ctx, const uint32_t* d_keys, const uint32_t* d_sizes,
                              const uint8_t* d_valid, uint8_t valid_ok, uint32_t n, uint64_t bytes_bound, void* after,
                              uint8_t* d_status_copy, void* then_stream, uint64_t* ticket, bool* done);   // pool.cpp
int txv_pool_check_dev(txv_pool* p, txv_ctx* ctx, const uint32_t* d_keys, const uint32_t* d_sizes,
                       const uint8_t* d_valid, const uint8_t* h_keys, const uint32_t* h_sizes, uint8_t valid_ok,
                       uint32_t n, uint64_t bytes_bound, void* after, uint8_t* status_out, bool* done);   // pool.cpp

namespace {

// Reactor.Receive -> CheckTxWithInfo -> TryAddVote for one batch of received messages, with the
// decoded votes kept in HBM, in three phases a node runs on its goroutines' threads:
//   decode (txv_ingest_decode; c->ing_dec_mu, c->mu around the enqueue) the wire bytes -> ring
//          slot j's arena (DMA'd straight from registered caller memory, else through pinned
//          staging), decodeMsg (kernels_wire.hip) into records in HBM, then per decoded message its
//          pool key, TxVote.Size() and status, whose copies back are enqueued; returns at once
//   admit  (txv_ingest_admit; c->ing_adm_mu, tickets in order) wait for those keys, CheckTxWithInfo
//          over the decoded messages in arrival order on the host (pool.cpp), then (c->mu) the
//          admitted votes' TxVote columns built on the device from the same records and the AddVote
//          chain of txv_add_votes enqueued (run_slot), not waited for
//   wait   (txv_ingest_wait) the chain's statuses and commit events
// so batch k+2 decodes while batch k+1 is in the pool stage and batch k's TxFlow chain runs, and
// other threads may submit or wait AddVote batches meanwhile (c->mu is not held by the waits for
// keys or for chains, nor by the pool stage).  An error after the pool stage (its votes are in the
// pool already) is kept for the wait, which reports TXV_FLOW_NOT_RUN for the admitted votes
// instead of dropping them silently.
int ingest_alloc(txv_ctx* c, txv_ctx::Ingest& g, Slot& s, uint64_t wire_bytes, uint32_t n) {
  int r;
  if (n > g.cap) {
    const uint32_t cap = std::max<uint32_t>(n, 1024);
    const size_t nch = (size_t)2 * ((cap + TXV_WIRE_BLOCK - 1) / TXV_WIRE_BLOCK);
    if ((r = dalloc(c, &g.d_off, cap)) || (r = halloc(c, &g.h_off, cap)) || (r = dalloc(c, &g.d_len, cap)) ||
        (r = halloc(c, &g.h_len, cap)) || (r = dalloc(c, &g.d_rec, wire_out_bytes(cap))) ||
        (r = dalloc(c, &g.d_span, nch)) || (r = halloc(c, &g.h_span, nch)) ||
        (r = dalloc(c, &g.d_status, cap)) || (r = halloc(c, &g.h_status, cap)) ||
        (r = dalloc(c, &g.d_keys, (size_t)cap * 8)) || (r = halloc(c, &g.h_keys, (size_t)cap * 8)) ||
        (r = dalloc(c, &g.d_sizes, cap)) || (r = halloc(c, &g.h_sizes, cap)) ||
        (r = dalloc(c, &g.d_list, cap)) || (r = halloc(c, &g.h_list, cap)) || (r = dalloc(c, &g.d_pstat, cap)) ||
        (r = dalloc(c, &g.d_max, 1)) || (r = halloc(c, &g.h_max, 1)))
      return r;
    g.cap = cap;
  }
  if (!g.kev) HIP_TRY(c, hipEventCreateWithFlags(&g.kev, hipEventDisableTiming));
  if (!g.uev) HIP_TRY(c, hipEventCreateWithFlags(&g.uev, hipEventDisableTiming));
  // the wire bytes go straight into the slot's TxHash arena: the decoded TxHash offsets index it
  if (wire_bytes + 128 > s.arena_cap) {
    const size_t cap = std::max<size_t>((size_t)wire_bytes + 128, s.arena_cap * 2);
    if ((r = halloc(c, &s.h_arena, cap)) || (r = dalloc(c, &s.d_arena_th, cap))) return r;
    s.arena_cap = cap;
  }
  return ensure_flow_slot(c, s, n);
}

int ingest_decode(txv_ctx* c, txv_pool* p, const uint8_t* wire, uint64_t wire_bytes, const uint64_t* msg_off,
                  const uint32_t* msg_len, uint32_t n, uint64_t* ticket) {
  if (wire_bytes >= (1ull << 32)) { c->err = "wire buffer >= 4 GiB"; return TXV_EINVAL; }
  uint32_t max_len = 0;
  for (uint32_t i = 0; i < n; ++i) {   // every message inside the buffer: the kernels trust these
    if (msg_off[i] > wire_bytes || msg_len[i] > wire_bytes - msg_off[i]) {
      c->err = "message " + std::to_string(i) + " outside the wire buffer";
      return TXV_EINVAL;
    }
    max_len = std::max(max_len, msg_len[i]);
  }
  // the pool's lock is taken before the context's everywhere (pool.cpp calls into the context with
  // its own lock held): its MaxMsgBytes is read here, before c->mu
  const uint32_t max_msg = p ? txv_pool_max_msg_bytes(p) : 0u;
  std::lock_guard<std::mutex> order(c->ing_dec_mu);
  HostTimer ht(c->profile_host);
  uint64_t t;
  uint32_t j;
  bool wire_reg;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(c, hipSetDevice(c->device));
    if (!c->n_vals) { c->err = "no validator set"; return TXV_ESTATE; }
    if (n > c->cfg.max_batch) { c->err = "batch exceeds max_batch"; return TXV_ECAPACITY; }
    if (c->poisoned) { c->err = "a TxFlow capacity was exceeded: txv_reset_flow first"; return TXV_ECAPACITY; }
    t = c->ing_next;
    j = (uint32_t)((t - 1) % kIngestRing);
    if (c->ing[j].phase) { c->err = "three ingest batches already in flight: wait for the oldest first"; return TXV_ESTATE; }
    // registered receive buffers are DMA'd from caller memory (until the batch's admit returns)
    wire_reg = wire_bytes && is_registered(c, wire, wire_bytes);
  }
  // ring slot j is free (its last ticket was waited: no DMA or kernel of it is pending), and only
  // this decoder (c->ing_dec_mu) touches it until its ticket is published
  txv_ctx::Ingest& g = c->ing[j];
  Slot& s = c->slots[kIngestSlot + j];
  int r;
  if ((r = ingest_alloc(c, g, s, wire_bytes, n))) return r;
  g.n = n; g.n_adm = 0; g.flow_err = 0; g.flow_msg.clear(); g.pool = p; g.wire_bytes = wire_bytes;
  g.max_len = max_len; g.early = false;
  const uint32_t n_chunks = (n + TXV_WIRE_BLOCK - 1) / TXV_WIRE_BLOCK;
  if (n) {
    if (!wire_reg) {
      c->pool->parallel_for((uint32_t)((wire_bytes + 65535) / 65536), [&](uint32_t lo, uint32_t hi) {
        const uint64_t a = (uint64_t)lo * 65536, b = std::min<uint64_t>((uint64_t)hi * 65536, wire_bytes);
        memcpy(s.h_arena + a, wire + a, b - a);
      }, 16);
      memset(s.h_arena + wire_bytes, 0, 128);
    }
    memcpy(g.h_off, msg_off, (size_t)n * 8);
    memcpy(g.h_len, msg_len, (size_t)n * 4);
    c->pool->parallel_for(n_chunks, [&](uint32_t lo_c, uint32_t hi_c) {
      for (uint32_t k = lo_c; k < hi_c; ++k) {
        uint64_t lo = ~0ull, hi = 0;
        for (uint32_t i = k * TXV_WIRE_BLOCK; i < std::min<uint32_t>(n, (k + 1) * TXV_WIRE_BLOCK); ++i)
          if (msg_len[i]) { lo = std::min(lo, msg_off[i]); hi = std::max(hi, msg_off[i] + msg_len[i]); }
        if (hi == 0) lo = 0;
        g.h_span[2 * k] = lo & ~15ull;
        g.h_span[2 * k + 1] = hi;
      }
    }, 64);
    *g.h_max = 0;
    ht.mark("stage");
  }
  std::lock_guard<std::mutex> lk(c->mu);
  if (n) {
    // the uploads run on the copy stream, which then carries DMA only (these, the Update entries'
    // signatures, the statuses back), the decode kernels on the key stream after them, in order with
    // the pool's device decisions and the TxFlow chains' prep that follow there.
    // TXV_WIRE_DECODE_STREAM (experiment): "copy" -- uploads and kernels on the copy stream, "key" --
    // both on the key stream (round 5)
    static const char* dsv = getenv("TXV_WIRE_DECODE_STREAM");
    static const int dmode = !dsv ? 0 : !strcmp(dsv, "copy") ? 1 : !strcmp(dsv, "key") ? 2 : 0;
    hipStream_t us = dmode == 2 ? c->key_stream : c->copy_stream;   // uploads
    hipStream_t ks = dmode == 1 ? c->copy_stream : c->key_stream;   // decode kernels
    if (s.launched) HIP_TRY(c, hipStreamWaitEvent(us, s.ev[4], 0));   // the slot's last chain ended
    if (wire_reg) {
      HIP_TRY(c, hipMemcpyAsync(s.d_arena_th, wire, wire_bytes, hipMemcpyHostToDevice, us));
      HIP_TRY(c, hipMemsetAsync(s.d_arena_th + wire_bytes, 0, 128, us));
    } else {
      HIP_TRY(c, hipMemcpyAsync(s.d_arena_th, s.h_arena, wire_bytes + 128, hipMemcpyHostToDevice, us));
    }
    HIP_TRY(c, hipMemcpyAsync(g.d_off, g.h_off, (size_t)n * 8, hipMemcpyHostToDevice, us));
    HIP_TRY(c, hipMemcpyAsync(g.d_len, g.h_len, (size_t)n * 4, hipMemcpyHostToDevice, us));
    HIP_TRY(c, hipMemcpyAsync(g.d_span, g.h_span, (size_t)n_chunks * 16, hipMemcpyHostToDevice, us));
    HIP_TRY(c, hipMemcpyAsync(g.d_max, g.h_max, 4, hipMemcpyHostToDevice, us));
    if (us != ks) {
      HIP_TRY(c, hipEventRecord(g.uev, us));
      HIP_TRY(c, hipStreamWaitEvent(ks, g.uev, 0));
    }
    WireArgs a{};
    a.n = n;
    a.max_msg_bytes = max_msg;
    txvote_msg_disfix(&a.disamb, &a.prefix);
    a.wire = s.d_arena_th; a.off = g.d_off; a.len = g.d_len;
    a.rec = reinterpret_cast<uint32_t*>(g.d_rec);
    a.n_chunks = n_chunks;
    a.span = g.d_span;
    HIP_TRY(c, txv_launch_decode_msgs(&a, (uint32_t)c->n_cus * 5u, ks));
    HIP_TRY(c, txv_launch_rec_keys(a.rec, s.d_arena_th, n, g.d_status, g.d_keys, g.d_sizes, g.d_max, ks));
    // back: the wire statuses and the longest TxHash; the keys and sizes only if the admission
    // takes the host path (ingest_admit_submit)
    HIP_TRY(c, hipMemcpyAsync(g.h_status, g.d_status, n, hipMemcpyDeviceToHost, ks));
    HIP_TRY(c, hipMemcpyAsync(g.h_max, g.d_max, 4, hipMemcpyDeviceToHost, ks));
    HIP_TRY(c, hipEventRecord(g.kev, ks));
  }
  ht.mark("decode_enqueue");
  g.ticket = t;
  g.phase = 1;
  c->ing_next = t + 1;
  *ticket = t;
  return TXV_OK;
}

// the admitted votes' TxFlow chain (the second half of an admission): their TxVote columns built
// on the device from the decode records, run_slot enqueued; c->mu held by the caller.  From here
// on the admitted votes are in the pool: the batch keeps its ticket whatever happens, and an
// error is reported by its wait together with the votes it concerns
void ingest_flow_stage(txv_ctx* c, uint64_t t, uint32_t n_adm) {
  const uint32_t j = (uint32_t)((t - 1) % kIngestRing);
  txv_ctx::Ingest& g = c->ing[j];
  Slot& s = c->slots[kIngestSlot + j];
  g.n_adm = n_adm;
  auto flow_stage = [&]() -> int {
    if (!n_adm) return TXV_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    if (c->poisoned) { c->err = "a TxFlow capacity was exceeded: txv_reset_flow first"; return TXV_ECAPACITY; }
    const uint32_t chain_len = (uint32_t)c->chain.size();
    const uint32_t mw = (signbytes_bound(*g.h_max, chain_len) + 7) / 8;
    int rr;
    if ((rr = ensure_slot(c, s, n_adm, mw))) return rr;
    hipStream_t ks = c->key_stream;
    HIP_TRY(c, hipMemcpyAsync(g.d_list, g.h_list, (size_t)n_adm * 4, hipMemcpyHostToDevice, ks));
    FlowCols fc{s.d_fh, s.d_fs, s.d_fn, s.d_fo, s.d_fl, s.d_addr, s.d_addr_len, s.d_sigraw, s.d_sig_len, s.d_txkey};
    HIP_TRY(c, txv_launch_rec_to_flow(reinterpret_cast<const uint32_t*>(g.d_rec), g.d_list, n_adm, &fc, ks));
    HIP_TRY(c, hipEventRecord(s.ev[3], ks));   // run_slot's kernels wait for this
    s.n = n_adm; s.n_pad = (n_adm + 63) / 64 * 64; s.msg_words = mw;
    s.has_nil = false;
    s.has_txkey = true;
    s.seq_base = c->seq_next;
    c->seq_next += n_adm;
    s.staged = true; s.ran = false; s.fill_mask = 0; s.fill_key = false;
    return run_slot(c, kIngestSlot + j, nullptr);
  };
  if (const int rf = flow_stage()) {
    g.flow_err = rf;
    g.flow_msg = c->err.copy();
  }
  g.phase = 2;
}

// The early TxFlow chain of a batch whose CheckTx was handed to the device: every message enters
// it, the pool's rejections and the messages that did not decode as nil entries built on the
// device from the statuses the pool's chain writes to g.d_pstat (the key stream waits for them:
// txv_pool_check_dev_submit), so the chain is enqueued without those statuses' host round trip.
// The SignBytes column is sized by the longest message (it bounds every TxHash).  c->mu held;
// an error is kept for the wait, as ingest_flow_stage's.
constexpr uint32_t kEarlyMaxLen = 1024;   // longer messages in a batch: ingest_flow_stage at finish
void ingest_flow_stage_early(txv_ctx* c, uint64_t t) {
  const uint32_t j = (uint32_t)((t - 1) % kIngestRing);
  txv_ctx::Ingest& g = c->ing[j];
  Slot& s = c->slots[kIngestSlot + j];
  g.early = true;
  auto flow_stage = [&]() -> int {
    HIP_TRY(c, hipSetDevice(c->device));
    if (c->poisoned) { c->err = "a TxFlow capacity was exceeded: txv_reset_flow first"; return TXV_ECAPACITY; }
    const uint32_t n = g.n;
    const uint32_t mw = (signbytes_bound(g.max_len, (uint32_t)c->chain.size()) + 7) / 8;
    int rr;
    if ((rr = ensure_slot(c, s, n, mw))) return rr;
    hipStream_t ks = c->key_stream;
    FlowCols fc{s.d_fh, s.d_fs, s.d_fn, s.d_fo, s.d_fl, s.d_addr, s.d_addr_len, s.d_sigraw, s.d_sig_len, s.d_txkey};
    HIP_TRY(c, txv_launch_rec_to_flow_nil(reinterpret_cast<const uint32_t*>(g.d_rec), g.d_pstat, n, &fc, s.d_nil, ks));
    HIP_TRY(c, hipEventRecord(s.ev[3], ks));   // run_slot's kernels wait for this
    s.n = n; s.n_pad = (n + 63) / 64 * 64; s.msg_words = mw;
    s.has_nil = true;
    s.has_txkey = true;
    s.seq_base = c->seq_next;
    c->seq_next += n;
    s.staged = true; s.ran = false; s.fill_mask = 0; s.fill_key = false;
    return run_slot(c, kIngestSlot + j, nullptr);
  };
  if (const int rf = flow_stage()) {
    g.flow_err = rf;
    g.flow_msg = c->err.copy();
  }
}

// the ticket ends without TxFlow (CheckTx failed before touching the pool); c->mu held
void ingest_drop(txv_ctx* c, txv_ctx::Ingest& g, uint64_t t) {
  g.phase = 0;
  g.ticket = 0;
  if (c->ing_admit_next == t) c->ing_admit_next = t + 1;
}

// an earlier ticket's admission is submitted to the device but not finished (c->mu held)
bool ingest_earlier_pending(const txv_ctx* c, uint64_t t) {
  for (const auto& o : c->ing)
    if (o.phase == 3 && o.ticket && o.ticket < t) return true;
  return false;
}

// First half of an admission (tickets in decode order): with TXV_POOL_DEVICE_CACHE and caps that
// cannot bind, CheckTx for every decoded message is enqueued on the device from the keys, sizes
// and decode statuses the decode left in HBM, behind the decode (txv_pool_check_dev_submit), and
// the call returns (phase 3) -- ingest_admit_finish collects the statuses.  Otherwise the whole
// admission runs here on the host path (phase 2 when it returns).
int ingest_admit_submit(txv_ctx* c, uint64_t t, uint8_t* wire_status, uint8_t* pool_status, bool* pending) {
  *pending = false;
  if (!t) return TXV_EINVAL;
  std::lock_guard<std::mutex> order(c->ing_adm_mu);
  HostTimer ht(c->profile_host);
  const uint32_t j = (uint32_t)((t - 1) % kIngestRing);
  txv_ctx::Ingest& g = c->ing[j];
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if (g.ticket != t || g.phase != 1) { c->err = "unknown ingest ticket, or not in the decoded phase"; return TXV_ESTATE; }
    if (t != c->ing_admit_next) { c->err = "ingest tickets must be admitted in decode order"; return TXV_ESTATE; }
  }
  const uint32_t n = g.n;
  if (n) {
    bool dev = false;
    uint64_t pt = 0;
    const bool early = g.max_len <= kEarlyMaxLen;
    const int rd = txv_pool_check_dev_submit(g.pool, c, g.d_keys, g.d_sizes, g.d_status, TXV_WIRE_OK, n, g.wire_bytes,
                                             (void*)g.kev, early ? g.d_pstat : nullptr,
                                             early ? (void*)c->key_stream : nullptr, &pt, &dev);
    if (rd) {   // the pool is unchanged: the ticket ends here (no wait)
      (void)hipEventSynchronize(g.kev);
      std::lock_guard<std::mutex> lk(c->mu);
      ingest_drop(c, g, t);
      return rd;
    }
    if (dev) {
      std::lock_guard<std::mutex> lk(c->mu);
      g.pool_ticket = pt;
      g.phase = 3;
      c->ing_admit_next = t + 1;
      *pending = true;
      ht.mark("pool_submit");
      if (early) {                 // TxFlow order = pool order: enqueued here, in ticket order
        ingest_flow_stage_early(c, t);
        ht.mark("flow_enqueue");
      }
      return TXV_OK;
    }
  }
  // the host path: CheckTxWithInfo over the decoded messages in arrival order on the host (the
  // others never reach it), every earlier submitted admission finished first (pool order)
  {
    std::lock_guard<std::mutex> fin(c->ing_fin_mu);
    {
      std::lock_guard<std::mutex> lk(c->mu);
      if (ingest_earlier_pending(c, t)) { c->err = "finish the earlier ingest admissions before a host-path batch"; return TXV_ESTATE; }
    }
    if (n) {
      {   // the keys and sizes back (the decode left them in HBM): after the decode, on the copy stream
        std::lock_guard<std::mutex> lk(c->mu);
        HIP_TRY(c, hipStreamWaitEvent(c->copy_stream, g.kev, 0));
        HIP_TRY(c, hipMemcpyAsync(g.h_keys, g.d_keys, (size_t)n * 32, hipMemcpyDeviceToHost, c->copy_stream));
        HIP_TRY(c, hipMemcpyAsync(g.h_sizes, g.d_sizes, (size_t)n * 4, hipMemcpyDeviceToHost, c->copy_stream));
        HIP_TRY(c, hipEventRecord(g.kev, c->copy_stream));
      }
      HIP_TRY(c, hipEventSynchronize(g.kev));   // no lock held: the keys' round trip only
    }
    ht.mark("keys_wait");
    if (wire_status && n) memcpy(wire_status, g.h_status, n);
    std::atomic<uint32_t> bad{0};
    c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
      uint32_t b = 0;
      for (uint32_t i = lo; i < hi; ++i) b += g.h_status[i] != TXV_WIRE_OK;
      if (b) bad.fetch_add(b, std::memory_order_relaxed);
    }, 16384);
    const bool all_ok = bad.load() == 0;
    std::vector<uint32_t> ok;
    std::vector<uint8_t> keys_c;
    std::vector<uint32_t> sizes_c;
    const uint8_t* keys = reinterpret_cast<const uint8_t*>(g.h_keys);
    const uint32_t* sizes = g.h_sizes;
    uint32_t m = n;
    if (!all_ok) {
      ok.reserve(n);
      for (uint32_t i = 0; i < n; ++i)
        if (g.h_status[i] == TXV_WIRE_OK) ok.push_back(i);
      m = (uint32_t)ok.size();
      keys_c.resize((size_t)m * 32);
      sizes_c.resize(m);
      c->pool->parallel_for(m, [&](uint32_t lo, uint32_t hi) {
        for (uint32_t q = lo; q < hi; ++q) {
          memcpy(keys_c.data() + (size_t)q * 32, g.h_keys + (size_t)ok[q] * 8, 32);
          sizes_c[q] = g.h_sizes[ok[q]];
        }
      }, 8192);
      keys = keys_c.data();
      sizes = sizes_c.data();
    }
    std::unique_ptr<uint8_t[]> pst(new uint8_t[std::max<uint32_t>(m, 1)]);
    int r = txv_pool_check_keys(g.pool, c, keys, sizes, m, pst.get());
    if (r) {   // the pool is unchanged: the ticket ends here (no wait)
      std::lock_guard<std::mutex> lk(c->mu);
      ingest_drop(c, g, t);
      return r;
    }
    uint32_t n_adm = 0;
    if (all_ok) {
      if (pool_status && m) memcpy(pool_status, pst.get(), m);
      for (uint32_t q = 0; q < m; ++q) {
        g.h_list[n_adm] = q;
        n_adm += pst[q] == TXV_POOL_OK;
      }
    } else {
      if (pool_status) memset(pool_status, TXV_POOL_NOT_CHECKED, n);
      for (uint32_t q = 0; q < m; ++q) {
        if (pool_status) pool_status[ok[q]] = pst[q];
        if (pst[q] == TXV_POOL_OK) g.h_list[n_adm++] = ok[q];
      }
    }
    ht.mark("pool");
    std::lock_guard<std::mutex> lk(c->mu);
    ingest_flow_stage(c, t, n_adm);
    c->ing_admit_next = t + 1;
    ht.mark("flow_enqueue");
  }
  return TXV_OK;
}

// Second half (tickets in order): the submitted CheckTx's statuses (txv_pool_check_wait, no
// context lock held while the GPU finishes), the admitted messages listed, their TxFlow chain
// enqueued (phase 2).  A batch the first half admitted on the host is finished already.
int ingest_admit_finish(txv_ctx* c, uint64_t t, uint8_t* wire_status, uint8_t* pool_status) {
  if (!t) return TXV_EINVAL;
  std::lock_guard<std::mutex> order(c->ing_fin_mu);
  HostTimer ht(c->profile_host);
  const uint32_t j = (uint32_t)((t - 1) % kIngestRing);
  txv_ctx::Ingest& g = c->ing[j];
  uint64_t pt;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if (g.ticket != t || (g.phase != 3 && g.phase != 2)) { c->err = "unknown ingest ticket, or not submitted for admission"; return TXV_ESTATE; }
    if (g.phase == 2) return TXV_OK;
    if (ingest_earlier_pending(c, t)) { c->err = "ingest admissions must be finished in ticket order"; return TXV_ESTATE; }
    pt = g.pool_ticket;
  }
  const uint32_t n = g.n;
  std::unique_ptr<uint8_t[]> dst(new uint8_t[std::max<uint32_t>(n, 1)]);
  const int rw = txv_pool_check_wait(g.pool, pt, dst.get());
  ht.mark("pool_wait");
  HIP_TRY(c, hipEventSynchronize(g.kev));   // (ended before the decisions began)
  if (wire_status && n) memcpy(wire_status, g.h_status, n);
  if (rw) {   // the device decisions failed: nothing of the batch reached TxFlow
    std::lock_guard<std::mutex> lk(c->mu);
    c->err = "ingest: the device CheckTx of the batch failed";
    // an early chain read statuses the failed decisions left: TxFlow's state is unknown from here
    if (g.early && !g.flow_err) c->poisoned = true;
    ingest_drop(c, g, t);
    return rw;
  }
  if (pool_status) memcpy(pool_status, dst.get(), n);
  uint32_t n_adm = 0;
  for (uint32_t i = 0; i < n; ++i) {
    g.h_list[n_adm] = i;
    n_adm += dst[i] == TXV_POOL_OK;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  if (g.early) {              // the chain runs already (every message, the rejected ones nil)
    g.n_adm = n_adm;
    g.phase = 2;
    ht.mark("list");
    return TXV_OK;
  }
  ingest_flow_stage(c, t, n_adm);
  ht.mark("flow_enqueue");
  return TXV_OK;
}

int ingest_admit(txv_ctx* c, uint64_t t, uint8_t* wire_status, uint8_t* pool_status) {
  bool pending = false;
  int r = ingest_admit_submit(c, t, wire_status, pool_status, &pending);
  if (r || !pending) return r;
  return ingest_admit_finish(c, t, wire_status, pool_status);
}

int ingest_wait(txv_ctx* c, uint64_t ticket, uint8_t* flow_status, txv_commit_event* ev_out, uint32_t ev_cap,
                uint32_t* n_ev) {
  if (n_ev) *n_ev = 0;
  if (!ticket) return TXV_EINVAL;
  const uint32_t j = (uint32_t)((ticket - 1) % kIngestRing);
  txv_ctx::Ingest& g = c->ing[j];
  Slot& s = c->slots[kIngestSlot + j];
  hipEvent_t done = nullptr;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if (g.ticket != ticket || g.phase != 2) { c->err = "unknown, unadmitted or already waited ingest ticket"; return TXV_ESTATE; }
    for (const auto& o : c->ing)
      if (o.phase == 2 && o.ticket < ticket) { c->err = "ingest tickets must be waited in submission order"; return TXV_ESTATE; }
    if (!g.flow_err && (g.n_adm || g.early) && s.ran) done = s.ev[4];
  }
  // the batch's chain ends without c->mu held (another thread's stages may run meanwhile); the
  // slot is not reused before this ticket is released below
  if (done) HIP_TRY(c, hipEventSynchronize(done));
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  int r = g.flow_err;
  // an early chain ran over every message (its statuses by message index), a late one over the
  // admitted ones (by their place in h_list)
  std::vector<uint8_t> fst(g.early ? g.n : g.n_adm);
  std::vector<txv_commit_event> evs;
  uint32_t ne = 0;
  if (!r && (g.n_adm || (g.early && s.ran))) {
    evs.resize(ev_out ? std::min(ev_cap, g.n_adm) : 0);
    r = fetch_slot(c, kIngestSlot + j, fst.data(), evs.data(), (uint32_t)evs.size(), &ne);
  } else if (r) {
    c->err = g.flow_msg;
  }
  if (flow_status) {
    for (uint32_t i = 0; i < g.n; ++i) flow_status[i] = TXV_FLOW_NOT_ADDED;
    for (uint32_t q = 0; q < g.n_adm; ++q)
      flow_status[g.h_list[q]] = r ? (uint8_t)TXV_FLOW_NOT_RUN : fst[g.early ? g.h_list[q] : q];
  }
  if (!r) {
    for (uint32_t e = 0; e < std::min<uint32_t>(ne, (uint32_t)evs.size()); ++e) {   // batch index -> message index
      txv_commit_event x = evs[e];
      if (!g.early) x.vote_index = g.h_list[x.vote_index];
      ev_out[e] = x;
    }
    if (n_ev) *n_ev = ne;
  }
  g.ticket = 0;
  g.phase = 0;
  return r;
}

int ingest_submit(txv_ctx* c, txv_pool* p, const uint8_t* wire, uint64_t wire_bytes, const uint64_t* msg_off,
                  const uint32_t* msg_len, uint32_t n, uint8_t* wire_status, uint8_t* pool_status, uint64_t* ticket) {
  // decode + admit back to back (a decode of another thread may slip in between: admits keep
  // ticket order, so this thread's admit then waits for the other batch's)
  uint64_t t = 0;
  int r = ingest_decode(c, p, wire, wire_bytes, msg_off, msg_len, n, &t);
  if (r) return r;
  for (;;) {
    r = ingest_admit(c, t, wire_status, pool_status);
    if (r != TXV_ESTATE) break;
    uint64_t next;
    {
      std::lock_guard<std::mutex> lk(c->mu);
      next = c->ing_admit_next;
    }
    if (next > t) break;            // a real state error
    std::this_thread::yield();      // an older ticket of another thread is still to be admitted
  }
  if (r) return r;
  *ticket = t;
  return TXV_OK;
}

}  // namespace

extern "C" {

int txv_ingest_decode(txv_ctx* c, txv_pool* p, const uint8_t* wire, uint64_t wire_bytes, const uint64_t* msg_off,
                      const uint32_t* msg_len, uint32_t n, uint64_t* ticket) {
  if (!c || !p || !ticket || (n && (!wire || !msg_off || !msg_len))) return TXV_EINVAL;
  *ticket = 0;
  return ingest_decode(c, p, wire, wire_bytes, msg_off, msg_len, n, ticket);
}

int txv_ingest_admit(txv_ctx* c, uint64_t ticket, uint8_t* wire_status, uint8_t* pool_status) {
  if (!c) return TXV_EINVAL;
  return ingest_admit(c, ticket, wire_status, pool_status);
}

int txv_ingest_admit_submit(txv_ctx* c, uint64_t ticket, uint8_t* wire_status, uint8_t* pool_status) {
  if (!c) return TXV_EINVAL;
  bool pending = false;
  return ingest_admit_submit(c, ticket, wire_status, pool_status, &pending);
}

int txv_ingest_admit_finish(txv_ctx* c, uint64_t ticket, uint8_t* wire_status, uint8_t* pool_status) {
  if (!c) return TXV_EINVAL;
  return ingest_admit_finish(c, ticket, wire_status, pool_status);
}

int txv_ingest_submit(txv_ctx* c, txv_pool* p, const uint8_t* wire, uint64_t wire_bytes, const uint64_t* msg_off,
                      const uint32_t* msg_len, uint32_t n, uint8_t* wire_status, uint8_t* pool_status, uint64_t* ticket) {
  if (!c || !p || !ticket || (n && (!wire || !msg_off || !msg_len))) return TXV_EINVAL;
  *ticket = 0;
  return ingest_submit(c, p, wire, wire_bytes, msg_off, msg_len, n, wire_status, pool_status, ticket);
}

int txv_ingest_wait(txv_ctx* c, uint64_t ticket, uint8_t* flow_status, txv_commit_event* ev_out, uint32_t ev_cap,
                    uint32_t* n_ev) {
  if (!c) return TXV_EINVAL;
  return ingest_wait(c, ticket, flow_status, ev_out, ev_cap, n_ev);
}

int txv_ingest_msgs(txv_ctx* c, txv_pool* p, const uint8_t* wire, uint64_t wire_bytes, const uint64_t* msg_off,
                    const uint32_t* msg_len, uint32_t n, uint8_t* wire_status, uint8_t* pool_status,
                    uint8_t* flow_status, txv_commit_event* ev_out, uint32_t ev_cap, uint32_t* n_ev) {
  if (!c || !p || (n && (!wire || !msg_off || !msg_len))) return TXV_EINVAL;
  if (n_ev) *n_ev = 0;
  uint64_t t = 0;
  const int r = ingest_submit(c, p, wire, wire_bytes, msg_off, msg_len, n, wire_status, pool_status, &t);
  if (r) {
    if (flow_status)
      for (uint32_t i = 0; i < n; ++i) flow_status[i] = TXV_FLOW_NOT_ADDED;
    return r;
  }
  return ingest_wait(c, t, flow_status, ev_out, ev_cap, n_ev);
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// TxVotePool's cache on the GPU (TXV_POOL_DEVICE_CACHE; pool_dev.h, kernels_pool.hip): the
// engine pool.cpp drives.  Its buffers are plain hipMalloc / hipHostMalloc allocations owned by
// the pool (freed by pooldev_free, whatever became of the context), on the device of the context
// first used; the work runs on that context's key stream.
#include "pool_dev.h"
extern "C" size_t txv_pooldev_tmp_bytes(uint32_t n, uint32_t C);
extern "C" hipError_t txv_pooldev_run(const PoolDevArgs* a, hipStream_t st);
extern "C" hipError_t txv_pooldev_index(const uint32_t* ck, uint32_t L, uint32_t* ci, uint32_t icap, uint64_t seed,
                                        hipStream_t st);
extern "C" size_t txv_poollist_tmp_bytes(uint32_t cap);
extern "C" hipError_t txv_poollist_compact(const uint32_t* lk, const uint32_t* lsz, const uint8_t* lfl,
                                           const unsigned long long* li, uint32_t ocap, uint32_t oicap, uint32_t* nk,
                                           uint32_t* nsz, uint8_t* nfl, unsigned long long* ni, uint32_t ncap,
                                           uint32_t nicap, uint32_t* npos, void* tmp, size_t tmp_bytes,
                                           uint32_t* tail_out, uint64_t seed, hipStream_t st);
extern "C" hipError_t txv_poollist_upload_index(const uint32_t* lk, const uint8_t* ins, uint32_t L,
                                                unsigned long long* li, uint32_t icap, uint64_t seed, hipStream_t st);

struct PoolDev {
  int device = -1;
  uint32_t C = 0, icap = 0, cap_n = 0, cur = 0;
  uint64_t seed = 0;                       // secret hash seed of every key placement (kernels_pool.hip)
  uint32_t* ck[2] = {nullptr, nullptr};
  uint32_t* ci[2] = {nullptr, nullptr};
  uint32_t* clen = nullptr;                        // [2]: length, staged new length
  uint32_t *push = nullptr, *aidx = nullptr, *hkey = nullptr, *hidx = nullptr, *skey = nullptr, *sidx = nullptr;
  uint32_t *last = nullptr, *lpos = nullptr, *far = nullptr, *nfar = nullptr, *surv = nullptr, *spos = nullptr;
  uint8_t *dec = nullptr, *detached = nullptr, *d_status = nullptr;
  uint64_t *pst = nullptr, *pend = nullptr;
  uint32_t *xs = nullptr, *xn = nullptr;   // per 1024-vote block: sorted pair starts, pair count
  uint64_t* tiles = nullptr;               // look-back words of the fused scans (kernels_pool.hip)
  uint32_t* tk = nullptr;                  // [4] their tile tickets
  uint32_t epoch = 0;                      // batches run: the look-back words' tag
  uint32_t* d_err = nullptr;               // sticky look-back timeout flag (kernels_pool.hip) ...
  uint32_t *h_err = nullptr, *m_err = nullptr;   // ... copied into mapped memory by each chain's last launch
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  uint32_t* okpos = nullptr;               // [cap_n] the list appends' ranks
  // the pool list (pool_dev.h PoolListArgs): two buffers, the current one `lcur` (a compaction
  // moves the live entries into the other), each with its own capacity; the tail in a pair of
  // words, ltp the current one (an append writes the other)
  struct ListBuf {
    uint32_t *k = nullptr, *sz = nullptr;
    uint8_t* fl = nullptr;
    unsigned long long* ix = nullptr;
    uint32_t cap = 0, icap = 0;
  } lb[2];
  int lcur = 0, ltp = 0;
  uint32_t* ltail = nullptr;               // [2]
  uint32_t* lnpos = nullptr;               // compaction scratch [lnpos_cap]
  uint32_t lnpos_cap = 0;
  void* ltmp = nullptr;
  size_t ltmp_bytes = 0;
  uint64_t tail_ub = 0;                    // host: an upper bound of the tail (the appends enqueued)
  uint64_t list_hint = 0;                  // entries the list is expected to hold (the pool's Size cap, clamped)
  // per batch in flight (kPdRing): its inputs, statuses and keys, and the event that ends it
  static constexpr int kPdRing = 8;
  struct Flight {
    uint32_t *d_sig = nullptr, *d_len = nullptr, *d_keys = nullptr, *d_sizes = nullptr;
    uint8_t* d_status = nullptr;
    uint32_t *h_sig = nullptr, *h_len = nullptr, *h_keys = nullptr, *h_sizes = nullptr;
    uint8_t *h_status = nullptr, *m_status = nullptr;   // mapped: pd_status writes the batch's statuses here
    uint64_t *h_res = nullptr, *m_res = nullptr;        // mapped, per tile (entries, bytes): [2 ntm] appended, [2 ntm] removed
    uint32_t nt_app = 0, nt_rm = 0;                // tiles of the batch in flight with partials there
    hipEvent_t ev = nullptr;
    hipEvent_t up_ev = nullptr;                    // the slot's signature uploads done (copy stream)
    // a CheckTx batch whose signatures and statuses a TxFlow chain reads straight from this slot
    // (txv_submit_checked): the pool ticket holding them (0 once anything else is staged here),
    // its Update entries ahead of it and its votes; cons_ev ends the reads (every later write to
    // the slot waits for it on the GPU)
    uint64_t occ = 0;
    uint32_t occ_upd = 0, occ_n = 0;
    hipEvent_t cons_ev = nullptr;
    bool cons = false;
  } fl[kPdRing];
  uint32_t* h_clen = nullptr;
  hipEvent_t ev = nullptr;
  hipStream_t st = nullptr;                        // cache uploads / downloads
  int on_ctx = 0;                                  // batches run on a context stream: 2 key, 3 copy (0: st)
  hipStream_t last_ks = nullptr;                   // the stream of the last batch enqueued, and its end
  hipEvent_t last_ev = nullptr;
  void quiesce() {                                 // every batch enqueued has ended (on_ctx: not on st)
    for (Flight& f : fl)
      if (f.ev) (void)hipEventSynchronize(f.ev);
  }
  ~PoolDev() {
    if (device < 0) return;
    (void)hipSetDevice(device);
    for (int b = 0; b < 2; ++b) { dfree(ck[b]); dfree(ci[b]); }
    dfree(clen); dfree(push); dfree(aidx); dfree(hkey); dfree(hidx); dfree(skey); dfree(sidx);
    dfree(last); dfree(lpos); dfree(far); dfree(nfar); dfree(surv); dfree(spos); dfree(dec);
    dfree(detached); dfree(pst); dfree(pend); dfree(xs); dfree(xn); dfree(tiles); dfree(tk); dfree(okpos);
    for (ListBuf& b : lb) { dfree(b.k); dfree(b.sz); dfree(b.fl); dfree(b.ix); }
    dfree(ltail); dfree(lnpos); dfree(d_err); hfree(h_err);
    if (ltmp) (void)hipFree(ltmp);
    for (Flight& f : fl) {
      dfree(f.d_sig); dfree(f.d_len); dfree(f.d_keys); dfree(f.d_sizes); dfree(f.d_status);
      hfree(f.h_sig); hfree(f.h_len); hfree(f.h_keys); hfree(f.h_sizes); hfree(f.h_status); hfree(f.h_res);
      if (f.ev) (void)hipEventDestroy(f.ev);
      if (f.up_ev) (void)hipEventDestroy(f.up_ev);
      if (f.cons_ev) (void)hipEventDestroy(f.cons_ev);
    }
    if (tmp) (void)hipFree(tmp);
    hfree(h_clen);
    if (ev) (void)hipEventDestroy(ev);
    if (st) (void)hipStreamDestroy(st);
  }
};

void pooldev_free(PoolDev* s) { delete s; }
bool pooldev_same_device(const txv_ctx* c, const PoolDev* s) { return c && s && c->device == s->device; }
uint32_t pooldev_cap(const PoolDev* s) { return s ? s->cap_n : 0; }

// the list partials of a flight: (entries, bytes) per 1024-vote tile, appended then removed
size_t res_words(uint32_t m) { return 4 * (((size_t)m + 1023) / 1024); }

// look-back words: per 1024 votes the push, last and list-append chains, per 1024 cache entries
// the survivors' chain
size_t pooldev_tile_words(uint32_t m, uint32_t C) {
  return 3 * (((size_t)m + 1023) / 1024) + ((size_t)std::max<uint32_t>(C, 1) + 1023) / 1024;
}

// (re)binds the engine to c's device with capacity C and room for n-vote batches; a new cache
// starts empty (length 0)
int pooldev_bind(txv_ctx* c, PoolDev** sp, uint32_t C, uint32_t n) {
  HIP_TRY(c, hipSetDevice(c->device));
  PoolDev* s = *sp;
  if (s && (s->device != c->device || s->C != C)) { delete s; s = *sp = nullptr; }
  const bool fresh = !s;
  if (fresh) {
    s = new (std::nothrow) PoolDev();
    if (!s) return TXV_ENOMEM;
    *sp = s;
    s->device = c->device;
    s->C = C;
    s->seed = ((uint64_t)std::random_device{}() << 32 | std::random_device{}()) ^ 0x706f6f6c6b657973ULL;
    s->icap = 16;
    while (s->icap < 2 * std::max<uint32_t>(C, 1)) s->icap *= 2;
    int r;
    const size_t cw = (size_t)std::max<uint32_t>(C, 1);
    if ((r = dalloc(c, &s->ck[0], cw * 8)) || (r = dalloc(c, &s->ck[1], cw * 8)) || (r = dalloc(c, &s->ci[0], s->icap)) ||
        (r = dalloc(c, &s->ci[1], s->icap)) || (r = dalloc(c, &s->clen, 2)) || (r = dalloc(c, &s->detached, cw)) ||
        (r = dalloc(c, &s->surv, cw)) || (r = dalloc(c, &s->spos, cw)) || (r = dalloc(c, &s->nfar, 2)) ||
        (r = halloc(c, &s->h_clen, 2)) || (r = dalloc(c, &s->tk, 4)) || (r = dalloc(c, &s->ltail, 2)) ||
        (r = dalloc(c, &s->d_err, 1)) || (r = halloc_mapped(c, &s->h_err, &s->m_err, 1)))
      return r;
    HIP_TRY(c, hipMemset(s->d_err, 0, 4));
    *s->h_err = 0;
    HIP_TRY(c, hipMemset(s->tk, 0, 16));
    HIP_TRY(c, hipMemset(s->ltail, 0, 8));
    HIP_TRY(c, hipMemset(s->ci[0], 0, (size_t)s->icap * 4));
    HIP_TRY(c, hipMemset(s->clen, 0, 8));
    HIP_TRY(c, hipMemset(s->detached, 0, cw));
    HIP_TRY(c, hipEventCreateWithFlags(&s->ev, hipEventDisableTiming));
    for (PoolDev::Flight& f : s->fl) {
      HIP_TRY(c, hipEventCreateWithFlags(&f.ev, hipEventDisableTiming));
      HIP_TRY(c, hipEventCreateWithFlags(&f.up_ev, hipEventDisableTiming));
    }
    // the batches run on the context's key stream: no HSA queue of the engine's own.  Measured on
    // C5 with Update (profiles/r05/c5_ab): an own high-priority stream 49-66M votes/s, an own
    // normal one 44-88M, the key stream 97-103M -- a fifth queue beside the context's four is
    // time-sliced by the hardware scheduler, and every launch of the engine's chain waits for it.
    // TXV_POOL_STREAM (experiment): 0 own high-priority stream, 1 own normal-priority stream,
    // 2 (default) the key stream, 3 the copy stream; the engine's own stream serves its synchronous
    // uploads either way
    static const int mode = getenv("TXV_POOL_STREAM") ? atoi(getenv("TXV_POOL_STREAM")) : 2;
    s->on_ctx = (mode == 2 || mode == 3) ? mode : 0;
    if (mode == 0) {
      int lo = 0, hi = 0;
      HIP_TRY(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIP_TRY(c, hipStreamCreateWithPriority(&s->st, hipStreamNonBlocking, hi));
    } else {
      HIP_TRY(c, hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
    }
  }
  if (n > s->cap_n) {
    int r;
    // geometric growth: an Update riding with a batch makes n vary, and every growth reallocates
    // (hipFree synchronises the device)
    const uint32_t m = std::max<uint32_t>(std::max<uint32_t>(n, 1024), s->cap_n ? 2 * s->cap_n : 0u);
    if (getenv("TXV_PROFILE_HOST")) fprintf(stderr, "[txv pool] engine grows %u -> %u entries\n", s->cap_n, m);
    if ((r = dalloc(c, &s->push, m)) || (r = dalloc(c, &s->aidx, m)) || (r = dalloc(c, &s->hkey, m)) ||
        (r = dalloc(c, &s->hidx, m)) || (r = dalloc(c, &s->skey, m)) || (r = dalloc(c, &s->sidx, m)) ||
        (r = dalloc(c, &s->last, m)) ||
        (r = dalloc(c, &s->lpos, m)) || (r = dalloc(c, &s->far, m)) || (r = dalloc(c, &s->dec, m)) ||
        (r = dalloc(c, &s->pst, m)) || (r = dalloc(c, &s->pend, m)) ||
        (r = dalloc(c, &s->xs, ((size_t)m + 1023) / 1024 * 1024)) || (r = dalloc(c, &s->xn, ((size_t)m + 1023) / 1024)) ||
        (r = dalloc(c, &s->tiles, pooldev_tile_words(m, C))) || (r = dalloc(c, &s->okpos, m)))
      return r;
    HIP_TRY(c, hipMemset(s->tiles, 0, pooldev_tile_words(m, C) * 8));
    for (PoolDev::Flight& f : s->fl)
      if ((r = dalloc(c, &f.d_sig, (size_t)m * 16)) || (r = dalloc(c, &f.d_len, m)) || (r = dalloc(c, &f.d_keys, (size_t)m * 8)) ||
          (r = dalloc(c, &f.d_sizes, m)) || (r = dalloc(c, &f.d_status, m)) || (r = halloc(c, &f.h_sig, (size_t)m * 16)) ||
          (r = halloc(c, &f.h_len, m)) || (r = halloc(c, &f.h_keys, (size_t)m * 8)) || (r = halloc(c, &f.h_sizes, m)) ||
          (r = halloc_mapped(c, &f.h_status, &f.m_status, m)) || (r = halloc_mapped(c, &f.h_res, &f.m_res, res_words(m))))
        return r;
    s->cap_n = m;
    const size_t tb = txv_pooldev_tmp_bytes(m, std::max<uint32_t>(C, 1));
    if (tb > s->tmp_bytes) {
      if (s->tmp) (void)hipFree(s->tmp);
      s->tmp = nullptr;
      HIP_TRY(c, hipMalloc(&s->tmp, tb));
      s->tmp_bytes = tb;
    }
  }
  return TXV_OK;
}

// HIP status -> TXV_EDEVICE (the message into c->err when there is a context)
#define PD_TRY(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      if (c) c->err = std::string(#x) + ": " + hipGetErrorString(e_);                     \
      return TXV_EDEVICE;                                                                  \
    }                                                                                      \
  } while (0)

// the host's cache (L keys, front to back) becomes the device's (synchronous, on the engine's
// own stream: every batch is waited for before its call returns; c may be NULL)
int pooldev_put_cache(txv_ctx* c, PoolDev* s, const uint8_t* keys, uint32_t L) {
  PD_TRY(hipSetDevice(s->device));
  if (L > s->C) { if (c) c->err = "pool cache longer than its capacity"; return TXV_EINVAL; }
  if (!s->st) PD_TRY(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
  s->quiesce();
  if (L) PD_TRY(hipMemcpyAsync(s->ck[s->cur], keys, (size_t)L * 32, hipMemcpyHostToDevice, s->st));
  s->h_clen[0] = L;
  s->h_clen[1] = L;
  PD_TRY(hipMemcpyAsync(s->clen, s->h_clen, 8, hipMemcpyHostToDevice, s->st));
  PD_TRY(txv_pooldev_index(s->ck[s->cur], L, s->ci[s->cur], s->icap, s->seed, s->st));
  PD_TRY(hipStreamSynchronize(s->st));
  return TXV_OK;
}

// the device's cache, front to back, into keys (synchronous; c may be NULL)
int pooldev_get_cache(txv_ctx* c, PoolDev* s, std::vector<uint8_t>& keys) {
  PD_TRY(hipSetDevice(s->device));
  if (!s->st) PD_TRY(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
  s->quiesce();
  PD_TRY(hipMemcpyAsync(s->h_clen, s->clen, 8, hipMemcpyDeviceToHost, s->st));
  PD_TRY(hipStreamSynchronize(s->st));
  const uint32_t L = s->h_clen[0];
  keys.resize((size_t)L * 32);
  if (L) {
    PD_TRY(hipMemcpyAsync(keys.data(), s->ck[s->cur], (size_t)L * 32, hipMemcpyDeviceToHost, s->st));
    PD_TRY(hipStreamSynchronize(s->st));
  }
  return TXV_OK;
}
#undef PD_TRY

// ---- the pool list in HBM (pool_dev.h PoolListArgs) ----
int list_buf_alloc(txv_ctx* c, PoolDev::ListBuf& b, uint32_t cap) {
  uint32_t icap = 16;
  while (icap < 2 * cap) icap *= 2;
  int r;
  if ((r = dalloc(c, &b.k, (size_t)cap * 8)) || (r = dalloc(c, &b.sz, cap)) || (r = dalloc(c, &b.fl, cap)) ||
      (r = dalloc(c, &b.ix, icap)))
    return r;
  b.cap = cap;
  b.icap = icap;
  return TXV_OK;
}
uint32_t list_cap_for(uint64_t need) {   // a power of two >= need, >= 64k
  uint64_t cap = 1u << 16;
  while (cap < need) cap *= 2;
  return cap > (1u << 30) ? 0u : (uint32_t)cap;
}

// the list's expected size (pool.cpp: the Size cap, clamped): both buffers are sized for it up front,
// so the compactions of a running pipeline do not reallocate (hipFree synchronises the device)
void pooldev_list_hint(PoolDev* s, uint64_t entries) { s->list_hint = std::min<uint64_t>(entries, 1u << 22); }
uint32_t list_cap_initial(const PoolDev* s) { return list_cap_for(2 * (s->list_hint + 4 * (uint64_t)s->cap_n)); }

// the current buffer exists (first use: empty, room for the hinted size and four batches; the
// other buffer allocated alike)
int list_ready(txv_ctx* c, PoolDev* s) {
  PoolDev::ListBuf& b = s->lb[s->lcur];
  if (b.cap) return TXV_OK;
  int r;
  const uint32_t cap = list_cap_initial(s);
  if ((r = list_buf_alloc(c, b, cap))) return r;
  if (s->lb[s->lcur ^ 1].cap < cap && (r = list_buf_alloc(c, s->lb[s->lcur ^ 1], cap))) return r;
  // the compaction's scratch too: a compaction at this capacity then neither allocates nor
  // synchronises the stream it runs on
  if (s->lnpos_cap < cap) {
    if ((r = dalloc(c, &s->lnpos, cap))) return r;
    s->lnpos_cap = cap;
  }
  if (const size_t tb = txv_poollist_tmp_bytes(cap); s->ltmp_bytes < tb) {
    if (s->ltmp) (void)hipFree(s->ltmp);
    s->ltmp = nullptr;
    HIP_TRY(c, hipMalloc(&s->ltmp, tb));
    s->ltmp_bytes = tb;
  }
  HIP_TRY(c, hipMemset(b.fl, 0, b.cap));
  HIP_TRY(c, hipMemset(b.ix, 0, (size_t)b.icap * 8));
  HIP_TRY(c, hipMemset(s->ltail, 0, 8));
  s->tail_ub = 0;
  return TXV_OK;
}

// positions ran out (the tail bound + n past the capacity): the live entries (at most live_ub)
// move, in order, into the other buffer, sized so that at least half of it is free after; the
// index is rebuilt there without its tombstones
int list_compact(txv_ctx* c, PoolDev* s, hipStream_t ks, uint64_t live_ub, uint32_t n) {
  PoolDev::ListBuf& o = s->lb[s->lcur];
  PoolDev::ListBuf& nb = s->lb[s->lcur ^ 1];
  const uint32_t ncap = std::max(o.cap, list_cap_for(2 * (live_ub + n)));
  if (getenv("TXV_PROFILE_HOST"))
    fprintf(stderr, "[txv pool] list compaction: cap %u -> %u, live <= %llu\n", o.cap, ncap, (unsigned long long)live_ub);
  if (!ncap) { c->err = "pool list above 2^30 entries"; return TXV_ECAPACITY; }
  const size_t tb = txv_poollist_tmp_bytes(o.cap);
  if (nb.cap < ncap || s->lnpos_cap < o.cap || s->ltmp_bytes < tb) {
    HIP_TRY(c, hipStreamSynchronize(ks));                // earlier work may still read the buffers
    int r;
    if (nb.cap < ncap && (r = list_buf_alloc(c, nb, ncap))) return r;
    if (s->lnpos_cap < o.cap) {
      if ((r = dalloc(c, &s->lnpos, o.cap))) return r;
      s->lnpos_cap = o.cap;
    }
    if (s->ltmp_bytes < tb) {
      if (s->ltmp) (void)hipFree(s->ltmp);
      s->ltmp = nullptr;
      HIP_TRY(c, hipMalloc(&s->ltmp, tb));
      s->ltmp_bytes = tb;
    }
  }
  HIP_TRY(c, txv_poollist_compact(o.k, o.sz, o.fl, o.ix, o.cap, o.icap, nb.k, nb.sz, nb.fl, nb.ix, nb.cap, nb.icap,
                                  s->lnpos, s->ltmp, s->ltmp_bytes, s->ltail + (s->ltp ^ 1), s->seed, ks));
  s->ltp ^= 1;
  s->lcur ^= 1;
  s->tail_ub = live_ub;
  return TXV_OK;
}

// the host's pool list becomes the device's: L entries in order (keys [L][32], sizes), ins[e] = 1
// for the entries txsMap indexes (synchronous, on the engine's own stream)
int pooldev_list_put(txv_ctx* c, PoolDev* s, const uint8_t* keys, const uint32_t* sizes, const uint8_t* ins, uint32_t L) {
  HIP_TRY(c, hipSetDevice(s->device));
  s->quiesce();
  int r;
  const uint32_t cap = std::max(list_cap_for(2 * ((uint64_t)L + 4 * (uint64_t)s->cap_n)), list_cap_initial(s));
  if (!cap) { c->err = "pool list above 2^30 entries"; return TXV_ECAPACITY; }
  PoolDev::ListBuf& b = s->lb[s->lcur];
  if (b.cap < cap && (r = list_buf_alloc(c, b, cap))) return r;
  if (s->lb[s->lcur ^ 1].cap < cap && (r = list_buf_alloc(c, s->lb[s->lcur ^ 1], cap))) return r;
  uint8_t* d_ins = nullptr;
  if (L && (r = dalloc(c, &d_ins, L))) return r;
  HIP_TRY(c, hipMemsetAsync(b.fl, 0, b.cap, s->st));
  if (L) {
    HIP_TRY(c, hipMemcpyAsync(b.k, keys, (size_t)L * 32, hipMemcpyHostToDevice, s->st));
    HIP_TRY(c, hipMemcpyAsync(b.sz, sizes, (size_t)L * 4, hipMemcpyHostToDevice, s->st));
    HIP_TRY(c, hipMemcpyAsync(d_ins, ins, L, hipMemcpyHostToDevice, s->st));
    HIP_TRY(c, hipMemsetAsync(b.fl, 1, L, s->st));
  }
  HIP_TRY(c, txv_poollist_upload_index(b.k, d_ins, L, b.ix, b.icap, s->seed, s->st));
  s->h_clen[0] = L;                                    // (staging word)
  HIP_TRY(c, hipMemcpyAsync(s->ltail + s->ltp, s->h_clen, 4, hipMemcpyHostToDevice, s->st));
  HIP_TRY(c, hipStreamSynchronize(s->st));
  dfree(d_ins);
  s->tail_ub = L;
  return TXV_OK;
}

// the device's pool list, in order: its live entries' keys, sizes and whether txsMap indexes
// them (synchronous; c may be NULL)
int pooldev_list_get(txv_ctx* c, PoolDev* s, std::vector<uint8_t>& keys, std::vector<uint32_t>& sizes,
                     std::vector<uint8_t>& ins) {
  keys.clear(); sizes.clear(); ins.clear();
  const PoolDev::ListBuf& b = s->lb[s->lcur];
  if (!b.cap) return TXV_OK;
  if (hipSetDevice(s->device) != hipSuccess) return TXV_EDEVICE;
  s->quiesce();
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess && c) c->err = std::string("pool list download: ") + hipGetErrorString(e);
    return e == hipSuccess;
  };
  if (!ok(hipMemcpyAsync(s->h_clen, s->ltail + s->ltp, 4, hipMemcpyDeviceToHost, s->st)) || !ok(hipStreamSynchronize(s->st)))
    return TXV_EDEVICE;
  const uint32_t T = s->h_clen[0];
  std::vector<uint8_t> k((size_t)T * 32), fl(T);
  std::vector<uint32_t> sz(T);
  std::vector<unsigned long long> ix(b.icap);
  if ((T && (!ok(hipMemcpyAsync(k.data(), b.k, (size_t)T * 32, hipMemcpyDeviceToHost, s->st)) ||
             !ok(hipMemcpyAsync(sz.data(), b.sz, (size_t)T * 4, hipMemcpyDeviceToHost, s->st)) ||
             !ok(hipMemcpyAsync(fl.data(), b.fl, T, hipMemcpyDeviceToHost, s->st)))) ||
      !ok(hipMemcpyAsync(ix.data(), b.ix, (size_t)b.icap * 8, hipMemcpyDeviceToHost, s->st)) ||
      !ok(hipStreamSynchronize(s->st)))
    return TXV_EDEVICE;
  std::vector<uint8_t> indexed(T, 0);
  for (unsigned long long v : ix)
    if (v && (uint32_t)v != kListTomb && (uint32_t)v - 1 < T) indexed[(uint32_t)v - 1] = 1;
  for (uint32_t e = 0; e < T; ++e) {
    if (!fl[e]) continue;
    keys.insert(keys.end(), k.begin() + (size_t)e * 32, k.begin() + (size_t)e * 32 + 32);
    sizes.push_back(sz[e]);
    ins.push_back(indexed[e]);
  }
  return TXV_OK;
}

// slot's finished batch: (entries appended, their bytes, entries removed, their bytes)
void pooldev_result(const PoolDev* s, int slot, int64_t res[4]) {
  const PoolDev::Flight& f = s->fl[slot];
  const size_t half = res_words(s->cap_n) / 2;
  uint64_t ac = 0, ab = 0, rc = 0, rb = 0;
  for (uint32_t t = 0; t < f.nt_app; ++t) { ac += f.h_res[2 * t]; ab += f.h_res[2 * t + 1]; }
  for (uint32_t t = 0; t < f.nt_rm; ++t) { rc += f.h_res[half + 2 * t]; rb += f.h_res[half + 2 * t + 1]; }
  res[0] = (int64_t)ac; res[1] = (int64_t)ab; res[2] = (int64_t)rc; res[3] = (int64_t)rb;
}

// the stream the engine's batches run on
hipStream_t engine_stream(txv_ctx* c, const PoolDev* s) {
  return s->on_ctx == 2 ? c->key_stream : s->on_ctx == 3 ? c->copy_stream : s->st;
}

// n votes of a txv_votes batch into flight f's entries [off, off + n): signatures uploaded -- from
// caller memory registered with txv_host_register (which must stay valid until the finish) or
// through the slot's pinned staging -- on the context's copy stream (the DMA does not hold up the
// kernels queued on the engine's stream meanwhile; f.up_ev marks it done), h_sizes = their
// TxVote.Size(); with key, keyed on stream ks once uploaded
int upload_votes(txv_ctx* c, PoolDev::Flight& f, hipStream_t ks, const txv_votes* v, uint32_t off, uint32_t n,
                 const uint32_t* h_sizes, bool key) {
  // TXV_POOL_UPLOAD_STREAM (experiment): 1 (default) the copy stream, 0 the engine's stream itself
  static const int up_mode = getenv("TXV_POOL_UPLOAD_STREAM") ? atoi(getenv("TXV_POOL_UPLOAD_STREAM")) : 1;
  hipStream_t us = up_mode ? c->copy_stream : ks;
  bool reg;
  {
    std::lock_guard<std::mutex> lk(c->reg_mu);
    reg = is_registered(c, v->sig, (uint64_t)n * 64) && is_registered(c, v->sig_len, (uint64_t)n * 4);
  }
  if (!reg)
    c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
      memcpy(f.h_sig + (size_t)(off + lo) * 16, v->sig + (size_t)lo * 64, (size_t)(hi - lo) * 64);
      memcpy(f.h_len + off + lo, v->sig_len + lo, (size_t)(hi - lo) * 4);
    }, 4096);
  memcpy(f.h_sizes + off, h_sizes, (size_t)n * 4);
  f.occ = 0;
  if (f.cons) HIP_TRY(c, hipStreamWaitEvent(us, f.cons_ev, 0));   // a TxFlow chain's reads of the slot first
  HIP_TRY(c, hipMemcpyAsync(f.d_sig + (size_t)off * 16, reg ? (const void*)v->sig : (const void*)(f.h_sig + (size_t)off * 16),
                            (size_t)n * 64, hipMemcpyHostToDevice, us));
  HIP_TRY(c, hipMemcpyAsync(f.d_len + off, reg ? (const void*)v->sig_len : (const void*)(f.h_len + off), (size_t)n * 4,
                            hipMemcpyHostToDevice, us));
  HIP_TRY(c, hipMemcpyAsync(f.d_sizes + off, f.h_sizes + off, (size_t)n * 4, hipMemcpyHostToDevice, us));
  HIP_TRY(c, hipEventRecord(f.up_ev, us));
  if (key) {
    HIP_TRY(c, hipStreamWaitEvent(ks, f.up_ev, 0));
    HIP_TRY(c, txv_launch_sig_keys(f.d_sig + (size_t)off * 16, f.d_len + off, n, f.d_keys + (size_t)off * 8, ks));
  }
  return TXV_OK;
}

// Update's committed votes staged into flight slot `slot` (finished by the caller) at entries
// [off, off + n): uploaded now on the engine's stream, keyed and decided with the slot's next
// enqueue -- the CheckTx batch after them (one SHA-256 launch over both), their pushes and
// removals first (n_upd), or alone
int pooldev_stage(txv_ctx* c, PoolDev* s, int slot, uint32_t off, const txv_votes* v, const uint32_t* h_sizes) {
  HIP_TRY(c, hipSetDevice(c->device));
  if (!v->n) return TXV_OK;
  if ((uint64_t)off + v->n > s->cap_n) { c->err = "pool device batch above its capacity"; return TXV_ECAPACITY; }
  return upload_votes(c, s->fl[slot], engine_stream(c, s), v, off, v->n, h_sizes, false);
}

// one batch's decisions enqueued on the engine's stream into flight slot `slot` (whose previous
// batch the caller has finished), either from a txv_votes batch (v, keyed here; h_sizes = their
// TxVote.Size()), from keys / sizes given on the host (h_keys_in), or from keys / sizes / validity
// already in HBM (d_keys, d_sizes, d_valid == valid_ok for a decoded message; `after` = the event
// that ends their producer).  n_upd Update entries staged in the slot (pooldev_stage) go first:
// pushed, removed from the pool list, no statuses.  With list_on the batch's admitted votes are
// appended to the pool list in HBM (live_ub: a bound of its live entries, for a compaction).  The
// statuses, and with keys_back the keys, come back into the slot's pinned buffers (pooldev_finish).
int pooldev_enqueue(txv_ctx* c, PoolDev* s, int slot, const txv_votes* v, const uint8_t* h_keys_in,
                    const uint32_t* h_sizes, const uint32_t* d_keys, const uint32_t* d_sizes, const uint8_t* d_valid,
                    uint32_t valid_ok, uint32_t n, int64_t max_tx, bool wal, bool keys_back, void* after_ev,
                    bool list_on, uint64_t live_ub, uint32_t n_upd, uint8_t* d_status_copy, void* then_stream) {
  hipEvent_t after = (hipEvent_t)after_ev;
  HIP_TRY(c, hipSetDevice(c->device));
  const uint32_t total = n_upd + n;
  if (!total) return TXV_OK;
  if (total > s->cap_n) { c->err = "pool device batch above its capacity"; return TXV_ECAPACITY; }
  if (2 * ((uint64_t)s->C + total) >= 0xFFFFFFFFull) { c->err = "pool device batch: S positions exceed 32 bits"; return TXV_ECAPACITY; }
  PoolDev::Flight& f = s->fl[slot];
  hipStream_t ks = engine_stream(c, s);
  f.occ = 0;
  if (f.cons) HIP_TRY(c, hipStreamWaitEvent(ks, f.cons_ev, 0));   // a TxFlow chain's reads of the slot first
  // every batch runs on the key stream: the wire ingest's uploads and decodes are on the copy
  // stream (ingest_decode), so its decisions overlap the next batch's upload there.  Round 5 ran
  // the wire batches' decisions on the copy stream while the decode sat on the key stream (74-76M
  // votes/s); with the decode moved, the copy stream serialised each batch's 19 MB of uploads with
  // its decisions (79-81M), the key stream overlaps them (98-100M, C5 from wire bytes, round 6).
  // TXV_POOL_DEV_STREAM=3 (experiment): the wire batches' decisions on the copy stream.
  static const int dev_stream = getenv("TXV_POOL_DEV_STREAM") ? atoi(getenv("TXV_POOL_DEV_STREAM")) : 2;
  if (!v && !h_keys_in && d_keys && n && dev_stream == 3 && s->on_ctx == 2) ks = c->copy_stream;
  // each batch reads the cache and pool list the previous one wrote, on whichever stream it ran
  if (s->last_ks && s->last_ks != ks) HIP_TRY(c, hipStreamWaitEvent(ks, s->last_ev, 0));
  if (after) HIP_TRY(c, hipStreamWaitEvent(ks, after, 0));   // device-resident inputs: their producer first
  if (v) {   // the batch's votes beside the staged ones, every signature keyed by one launch
    if (n) {
      int r;
      if ((r = upload_votes(c, f, ks, v, n_upd, n, h_sizes, false))) return r;
    }
    HIP_TRY(c, hipStreamWaitEvent(ks, f.up_ev, 0));       // the staged and the batch's uploads (copy stream, in order)
    HIP_TRY(c, txv_launch_sig_keys(f.d_sig, f.d_len, total, f.d_keys, ks));
    d_keys = f.d_keys;
    d_sizes = f.d_sizes;
    d_valid = nullptr;
  } else if (h_keys_in) {   // keys and sizes given on the host (txv_pool_check_keys)
    if (n_upd) {
      HIP_TRY(c, hipStreamWaitEvent(ks, f.up_ev, 0));
      HIP_TRY(c, txv_launch_sig_keys(f.d_sig, f.d_len, n_upd, f.d_keys, ks));
    }
    c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
      memcpy(f.h_keys + (size_t)(n_upd + lo) * 8, h_keys_in + (size_t)lo * 32, (size_t)(hi - lo) * 32);
      memcpy(f.h_sizes + n_upd + lo, h_sizes + lo, (size_t)(hi - lo) * 4);
    }, 8192);
    if (n) {
      HIP_TRY(c, hipMemcpyAsync(f.d_keys + (size_t)n_upd * 8, f.h_keys + (size_t)n_upd * 8, (size_t)n * 32,
                                hipMemcpyHostToDevice, ks));
      HIP_TRY(c, hipMemcpyAsync(f.d_sizes + n_upd, f.h_sizes + n_upd, (size_t)n * 4, hipMemcpyHostToDevice, ks));
    }
    d_keys = f.d_keys;
    d_sizes = f.d_sizes;
    d_valid = nullptr;
  } else if (n_upd) {       // staged Update entries, alone or before keys already in HBM (moved beside them)
    HIP_TRY(c, hipStreamWaitEvent(ks, f.up_ev, 0));
    HIP_TRY(c, txv_launch_sig_keys(f.d_sig, f.d_len, n_upd, f.d_keys, ks));
    if (n) {
      HIP_TRY(c, hipMemcpyAsync(f.d_keys + (size_t)n_upd * 8, d_keys, (size_t)n * 32, hipMemcpyDeviceToDevice, ks));
      HIP_TRY(c, hipMemcpyAsync(f.d_sizes + n_upd, d_sizes, (size_t)n * 4, hipMemcpyDeviceToDevice, ks));
    }
    d_keys = f.d_keys;
    d_sizes = f.d_sizes;
  }
  PoolDevArgs a{};
  a.n = total; a.n_force = n_upd; a.keys = d_keys; a.sizes = d_sizes; a.valid = d_valid; a.valid_ok = valid_ok;
  a.max_tx = n ? max_tx : INT64_MAX;                     // Update alone: no statuses, no far decisions
  a.C = s->C; a.wal = wal ? 1u : 0u;
  a.ck_old = s->ck[s->cur]; a.ck_new = s->ck[s->cur ^ 1]; a.ci_old = s->ci[s->cur]; a.ci_new = s->ci[s->cur ^ 1];
  a.icap = s->icap; a.clen = s->clen;
  a.push = s->push; a.aidx = s->aidx; a.hkey = s->hkey; a.hidx = s->hidx; a.skey = s->skey; a.sidx = s->sidx;
  a.last = s->last; a.lpos = s->lpos; a.dec = s->dec; a.pst = s->pst;
  a.pend = s->pend; a.xs = s->xs; a.xn = s->xn; a.far = s->far; a.nfar = s->nfar; a.detached = s->detached; a.surv = s->surv; a.spos = s->spos;
  a.tmp = s->tmp; a.tmp_bytes = s->tmp_bytes; a.status = f.d_status; a.status_out = f.m_status; a.status_copy = d_status_copy;
  a.tiles = s->tiles; a.tk = s->tk; a.err = s->d_err; a.err_host = s->m_err; a.seed = s->seed;
  if (((++s->epoch) & 0x3FFFFFFFu) == 0) {          // the tag wrapped: no word may match by accident
    HIP_TRY(c, hipMemsetAsync(s->tiles, 0, pooldev_tile_words(s->cap_n, s->C) * 8, ks));
    ++s->epoch;
  }
  a.epoch = s->epoch;
  f.nt_app = f.nt_rm = 0;
  if (list_on) {
    int r;
    if ((r = list_ready(c, s))) return r;
    if (s->tail_ub + n > s->lb[s->lcur].cap && (r = list_compact(c, s, ks, live_ub, n))) return r;
    const PoolDev::ListBuf& b = s->lb[s->lcur];
    a.list_on = 1;
    a.okpos = s->okpos;
    a.res = f.m_res;
    a.res_rm = f.m_res + res_words(s->cap_n) / 2;
    a.l.lk = b.k; a.l.lsz = b.sz; a.l.lfl = b.fl; a.l.li = b.ix; a.l.imask = b.icap - 1; a.l.seed = s->seed;
    a.l.tail_in = s->ltail + s->ltp; a.l.tail_out = s->ltail + (s->ltp ^ 1);
    f.nt_app = (total + 1023) / 1024;
    f.nt_rm = (n_upd + 1023) / 1024;
  }
  HIP_TRY(c, txv_pooldev_run(&a, ks));
  if (s->C) s->cur ^= 1;                                  // the next batch on this stream reads the new cache
  if (list_on) {                                          // pd_status wrote the tail's other word
    s->ltp ^= 1;
    s->tail_ub += n;
  }
  if (keys_back && d_keys == f.d_keys && v && n)
    HIP_TRY(c, hipMemcpyAsync(f.h_keys, f.d_keys + (size_t)n_upd * 8, (size_t)n * 32, hipMemcpyDeviceToHost, ks));
  HIP_TRY(c, hipEventRecord(f.ev, ks));
  // a consumer of the statuses in HBM (the wire ingest's TxFlow chain) waits for them on its stream
  if (then_stream) HIP_TRY(c, hipStreamWaitEvent((hipStream_t)then_stream, f.ev, 0));
  s->last_ks = ks;
  s->last_ev = f.ev;
  return TXV_OK;
}

// waits for slot's batch; its statuses, keys ([n][32]: the v and h_keys_in paths) and sizes (same)
// in pinned memory, valid until the slot is enqueued again
int pooldev_finish(txv_ctx* c, PoolDev* s, int slot, const uint8_t** status, const uint8_t** keys,
                   const uint32_t** sizes) {
  PoolDev::Flight& f = s->fl[slot];
  if (c) HIP_TRY(c, hipEventSynchronize(f.ev));
  else if (hipEventSynchronize(f.ev) != hipSuccess) return TXV_EDEVICE;
  if (*(volatile uint32_t*)s->h_err) {   // a look-back scan of this or an earlier chain timed out (sticky)
    if (c) c->err = "pool engine: look-back scan timed out (device error; statuses not trusted)";
    return TXV_EDEVICE;
  }
  if (status) *status = f.h_status;
  if (keys) *keys = reinterpret_cast<const uint8_t*>(f.h_keys);
  if (sizes) *sizes = f.h_sizes;
  return TXV_OK;
}

// flight slot `slot` holds pool ticket `id`'s batch (n votes after n_upd Update entries): a TxFlow
// chain may read its signatures and statuses from HBM (pooldev_consume) until the slot is reused
void pooldev_set_occupant(PoolDev* s, int slot, uint64_t id, uint32_t n_upd, uint32_t n) {
  PoolDev::Flight& f = s->fl[slot];
  f.occ = id;
  f.occ_upd = n_upd;
  f.occ_n = n;
}

// txv_submit_checked: pool ticket `id`'s signatures ([n][64] bytes) into sig_out and its statuses
// as the nil column (nil_out[i] = status != TXV_POOL_OK, or-ed into the column's caller values
// when or_nil) on stream st, behind the batch's decisions; the slot's next writer waits for these
// reads.  1: the ticket's batch is no longer in any slot (the caller takes its host statuses).
int pooldev_consume(txv_ctx* c, PoolDev* s, uint64_t id, uint32_t n, hipStream_t st, uint8_t* sig_out, uint8_t* nil_out,
                    bool or_nil, bool raw_status) {
  if (!s || !id) return 1;
  for (PoolDev::Flight& f : s->fl) {
    if (f.occ != id) continue;
    if (f.occ_n != n) { c->err = "txv_submit_checked: the batch differs from the pool ticket's"; return TXV_EINVAL; }
    if (!f.cons_ev) HIP_TRY(c, hipEventCreateWithFlags(&f.cons_ev, hipEventDisableTiming));
    HIP_TRY(c, hipStreamWaitEvent(st, f.ev, 0));
    HIP_TRY(c, hipMemcpyAsync(sig_out, f.d_sig + (size_t)f.occ_upd * 16, (size_t)n * 64, hipMemcpyDeviceToDevice, st));
    if (raw_status)   // the statuses themselves (txv_route_checked: the route kernels read TXV_POOL_*)
      HIP_TRY(c, hipMemcpyAsync(nil_out, f.d_status + f.occ_upd, n, hipMemcpyDeviceToDevice, st));
    else
      HIP_TRY(c, txv_launch_nil_from_status(f.d_status + f.occ_upd, n, nil_out, or_nil ? 1u : 0u, st));
    HIP_TRY(c, hipEventRecord(f.cons_ev, st));
    f.cons = true;
    return 0;
  }
  return 1;
}

bool pooldev_holds(const PoolDev* s, uint64_t id) {
  if (!s || !id) return false;
  for (const PoolDev::Flight& f : s->fl)
    if (f.occ == id) return true;
  return false;
}

// txv_submit_checked's context half, in three steps (pool.cpp drives them, one submitter at a
// time under txv_ctx::sub_mu): stage the batch's columns but its signatures, then -- the pool's
// lock held -- take the signatures and nil column from the CheckTx batch still in the pool
// engine's flight slot (pooldev_consume), or else upload them from the caller's columns with the
// ticket's host statuses as the nil column, then enqueue the AddVote chain.
std::mutex& txv_ctx_submit_mu(txv_ctx* c) { return c->sub_mu; }

int submit_checked_stage(txv_ctx* c, const txv_votes* v, uint32_t* slot_out) {
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  const uint32_t slot = (uint32_t)((c->next_ticket - 1) % kSubmitRing);
  if (c->slots[slot].ticket) { c->err = "four batches already in flight: wait for the oldest one first"; return TXV_ESTATE; }
  txv_votes w = *v;
  w.sig = nullptr;                 // from the pool's flight slot (or uploaded late)
  w.is_nil = nullptr;              // written on the device (or uploaded late)
  if (int r = stage_add(c, slot, &w)) return r;
  *slot_out = slot;
  return TXV_OK;
}

// the device source (the pool's lock held): 1 = the batch is no longer in the engine
int submit_checked_consume(txv_ctx* c, uint32_t slot, PoolDev* dev, uint64_t pool_ticket, const txv_votes* v) {
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  Slot& s = c->slots[slot];
  if (!v->n) return TXV_OK;
  // behind the uploads (and the slot's previous chain: stage_add's copy stream waited for it), on
  // the key stream, which carries the pool's decisions too
  hipStream_t ks = c->key_stream;
  HIP_TRY(c, hipStreamWaitEvent(ks, s.ev[3], 0));
  if (v->is_nil) {                 // the caller's nil column first, or-ed into below
    memcpy(s.h_nil, v->is_nil, v->n);
    HIP_TRY(c, hipMemcpyAsync(s.d_nil, s.h_nil, v->n, hipMemcpyHostToDevice, ks));
  }
  const int r = pooldev_consume(c, dev, pool_ticket, v->n, ks, s.d_sigraw, s.d_nil, v->is_nil != nullptr, false);
  if (r) return r;
  HIP_TRY(c, hipEventRecord(s.ev[3], ks));   // run_slot's streams wait for the columns here
  return TXV_OK;
}

// the host source / the chain: why 1 = unknown pool ticket, 2 = another batch size; host_st (or
// null after a device consume) = the ticket's statuses
int submit_checked_run(txv_ctx* c, uint32_t slot, const txv_votes* v, const uint8_t* host_st, int why, uint64_t* ticket) {
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (why == 1) { c->err = "txv_submit_checked: unknown pool ticket (already waited?)"; return TXV_ESTATE; }
  if (why == 2) { c->err = "txv_submit_checked: the batch differs from the pool ticket's"; return TXV_EINVAL; }
  Slot& s = c->slots[slot];
  const uint32_t n = v->n;
  if (host_st && n) {              // the signatures and nil column from the host after all
    for (uint32_t i = 0; i < n; ++i) s.h_nil[i] = (host_st[i] != TXV_POOL_OK || (v->is_nil && v->is_nil[i])) ? 1 : 0;
    const bool reg = is_registered(c, v->sig, (uint64_t)n * 64);
    if (!reg) c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
      memcpy(s.h_sigraw + (size_t)lo * 64, v->sig + (size_t)lo * 64, (size_t)(hi - lo) * 64);
    }, 4096);
    HIP_TRY(c, hipMemcpyAsync(s.d_sigraw, reg ? (const void*)v->sig : (const void*)s.h_sigraw, (size_t)n * 64,
                              hipMemcpyHostToDevice, c->copy_stream));
    HIP_TRY(c, hipMemcpyAsync(s.d_nil, s.h_nil, n, hipMemcpyHostToDevice, c->copy_stream));
    HIP_TRY(c, hipEventRecord(s.ev[3], c->copy_stream));
  }
  s.has_nil = true;
  int r;
  if ((r = run_slot(c, slot, nullptr))) return r;
  const uint64_t t = c->next_ticket;
  s.ticket = t;
  c->next_ticket = t + 1;
  *ticket = t;
  return TXV_OK;
}

// txv_route_checked's device source (the pool's lock held): the CheckTx batch's signatures and
// statuses into the route slot, on the key stream behind the decisions; 1 = no longer in the engine
int route_checked_consume(txv_ctx* c, PoolDev* dev, uint64_t pool_ticket, uint32_t n) {
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  if (!n) return TXV_OK;
  Slot& s = c->slots[kRouteSlot];
  hipStream_t ks = c->key_stream;
  HIP_TRY(c, hipStreamWaitEvent(ks, s.ev[3], 0));
  const int r = pooldev_consume(c, dev, pool_ticket, n, ks, s.d_sigraw, s.d_pre, false, true);
  if (r) return r;
  HIP_TRY(c, hipEventRecord(s.ev[3], ks));
  return TXV_OK;
}

std::mutex& txv_ctx_route_mu(txv_ctx* c) { return c->route_mu; }
int route_checked_stage(txv_ctx* c, const txv_votes* v, uint64_t stride) { return route_stage(c, v, true, stride); }
int route_checked_launch(txv_ctx* c, const txv_votes* v, const uint8_t* host_st, uint32_t G, void* dst, uint64_t stride,
                         txv_route_meta* meta) {
  return route_launch(c, v, host_st, host_st == nullptr, true, G, dst, stride, meta);
}
int txv_ctx_fail(txv_ctx* c, int code, const char* msg) {
  std::lock_guard<std::mutex> g(c->mu);
  c->err = msg;
  return code;
}

// enqueue + finish in one call (synchronous): statuses into status_out, keys (v path) into keys_out
int pooldev_check(txv_ctx* c, PoolDev* s, const txv_votes* v, const uint8_t* h_keys_in, const uint32_t* h_sizes,
                  const uint32_t* d_keys, const uint32_t* d_sizes, const uint8_t* d_valid, uint32_t valid_ok, uint32_t n,
                  int64_t max_tx, bool wal, uint8_t* keys_out, uint8_t* status_out, void* after_ev, bool list_on,
                  uint64_t live_ub, int slot, uint32_t n_upd) {
  if (!n) return TXV_OK;
  HostTimer ht(c->profile_host);
  int r = pooldev_enqueue(c, s, slot, v, h_keys_in, h_sizes, d_keys, d_sizes, d_valid, valid_ok, n, max_tx, wal,
                          keys_out != nullptr, after_ev, list_on, live_ub, n_upd, nullptr, nullptr);
  if (r) return r;
  ht.mark("enqueue");
  const uint8_t* st;
  const uint8_t* kp;
  if ((r = pooldev_finish(c, s, slot, &st, &kp, nullptr))) return r;
  ht.mark("device");
  memcpy(status_out, st, n);
  if (v && keys_out)
    c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
      memcpy(keys_out + (size_t)lo * 32, kp + (size_t)lo * 32, (size_t)(hi - lo) * 32);
    }, 8192);
  ht.mark("out");
  return TXV_OK;
}
