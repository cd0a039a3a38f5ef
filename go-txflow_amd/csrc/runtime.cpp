// runtime.cpp — host runtime behind include/txvote.h (libtxvote.so).
//
// Responsibilities (the parts of the reference path that stay on the host):
//   * validator registry: address -> index (ValidatorSet.GetByAddress, ext, called at
//     types/vote_set.go:102), powers, quorum = Total*2/3 + 1 (types/vote_set.go:158)
//   * TxVoteSets routing: TxHash -> dense set id, created on first sight
//     (txflow/service.go:200-209); host mirror of sum / maj23 for the readers
//   * amino SignBytes encoding (amino.hpp) and the SoA pack into pinned buffers
//   * device buffers, one HIP stream per context, launch order K1 verify -> K2 tally
// Everything numeric about a vote's verdict runs on the GPU; there is no CPU verify path.
#include "../../include/txvote.h"
#include "txv_device.h"
#include "txv_tally.h"
#include "amino.hpp"
#include "host_pack.hpp"
#include "sha2.h"

#include <hip/hip_runtime.h>
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
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

// fixed-base table words per point for window W: ceil(256/W) positions x (2^(W-1)+1) entries x 24
inline size_t table_words(int w) { return (size_t)((256 + w - 1) / w) * ((1u << (w - 1)) + 1) * 24; }
constexpr uint32_t kTableWords4 = 64 * 9 * 24;
inline bool valid_window(int w) { return w == 4 || w == 8 || w == 10 || w == 12 || w == 14 || w == 16 || w == 18 || w == 20; }
constexpr uint32_t kSlots = 4;

struct Slot {
  uint32_t cap = 0, n = 0, n_pad = 0, msg_words = 0, msg_cap_words = 0;
  uint32_t n_touched = 0, touched_cap = 0;
  bool staged = false, ran = false;
  // device
  uint32_t* d_sig = nullptr; uint64_t* d_msg = nullptr; uint32_t* d_msg_len = nullptr;
  uint32_t* d_val = nullptr; uint32_t* d_set = nullptr; uint8_t* d_flags = nullptr;
  uint8_t* d_status = nullptr; uint8_t* d_ok = nullptr; uint8_t* d_pre = nullptr;
  uint32_t* d_kbuf = nullptr; uint32_t* d_rpts = nullptr; uint32_t* d_order = nullptr; uint32_t* h_order = nullptr;
  uint32_t n_work = 0;
  // set-major tally order: pending votes grouped by (set, validator), arrival order inside
  uint32_t* d_toff = nullptr; uint32_t* h_toff = nullptr;
  uint32_t* d_tvote = nullptr; uint32_t* h_tvote = nullptr;
  uint32_t* d_tval = nullptr; uint32_t* h_tval = nullptr;
  uint32_t* d_ent_vote = nullptr; int64_t* d_ent_power = nullptr; uint32_t* d_ent_val = nullptr;
  uint32_t* d_touched = nullptr; int64_t* d_tsum = nullptr; uint8_t* d_tmaj = nullptr; uint32_t* d_tcross = nullptr;
  // pinned host
  uint32_t* h_sig = nullptr; uint64_t* h_msg = nullptr; uint32_t* h_msg_len = nullptr;
  uint32_t* h_val = nullptr; uint32_t* h_set = nullptr; uint8_t* h_flags = nullptr; uint8_t* h_status = nullptr;
  uint32_t* h_touched = nullptr; int64_t* h_tsum = nullptr; uint8_t* h_tmaj = nullptr; uint32_t* h_tcross = nullptr;
  // results, written by the tally kernels straight into mapped host memory (m_* = device views)
  uint8_t* h_out = nullptr; uint8_t* m_out = nullptr;
  int64_t* m_tsum = nullptr; uint8_t* m_tmaj = nullptr; uint32_t* m_tcross = nullptr;
  std::vector<uint8_t> tmp_msg;   // SignBytes arena (verify-only paths)
  std::vector<size_t> tmp_off;
  // device SignBytes inputs (kernels_signbytes.hip): pinned staging + device copies
  int64_t *h_fh = nullptr, *h_fs = nullptr, *d_fh = nullptr, *d_fs = nullptr;     // height, ts_sec
  int32_t *h_fn = nullptr, *d_fn = nullptr;                                        // ts_nanos
  uint32_t *h_fo = nullptr, *h_fl = nullptr, *d_fo = nullptr, *d_fl = nullptr;     // txhash off / len
  uint8_t *h_arena = nullptr, *d_arena_th = nullptr;                               // TxHash arena
  size_t arena_cap = 0;
  bool msg_on_device = false;      // this staging's SignBytes are built by txv_k_signbytes
  std::vector<int> lens;           // AddVote pack: SignBytes length (-1 amino error, -2 nil)
  std::vector<uint64_t> khash;     // AddVote pack: seeded hash of the TxHash bytes
  std::vector<uint32_t> vidx;      // AddVote pack: validator index or UINT32_MAX
  std::vector<uint32_t> miss;      // AddVote pack: votes whose TxHash has no set yet
  // 0..2 kernel timing, 3 = the slot's uploads are done (copy stream), 4 = its results are in
  // the pinned buffers (compute stream)
  hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  uint64_t ticket = 0;    // txv_submit_votes ticket in flight on this slot (0 = none)
};

}  // namespace

struct txv_ctx {
  txv_config cfg{};
  int device = 0;
  int n_cus = 256;
  hipStream_t stream = nullptr;        // compute: verify + tally kernels, result copies
  hipStream_t copy_stream = nullptr;   // batch uploads, so batch k+1's H2D overlaps batch k's kernels
  hipStream_t key_stream = nullptr;    // txv_sig_keys (pool ingest) runs beside in-flight batches
  uint64_t next_ticket = 1;            // txv_submit_votes ring over slots 0 and 1
  std::string err;
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
  uint32_t* d_park = nullptr;      // K1b parked points: [wave][V-1][32][64]
  size_t park_words = 0;
  // scratch registry for caller-supplied keys (txv_verify_batch with pubs32)
  uint32_t tmp_cap = 0;
  int tmp_w = 0;
  uint32_t* d_tmp_pubs = nullptr; uint8_t* d_tmp_ok = nullptr; uint32_t* d_tmp_tables = nullptr; uint32_t* d_tmp_addr = nullptr;
  // tally state
  txv_host::TxTable tx_tab{std::random_device{}() * 0x9e3779b97f4a7c15ULL + 0x7478};   // TxHash -> set id
  std::unique_ptr<txv_host::WorkerPool> pool;   // host pack threads
  bool profile_host = false;                    // TXV_PROFILE_HOST
  std::vector<int64_t> h_sum;
  std::vector<uint8_t> h_maj;
  std::vector<uint32_t> seen_stage, set_tidx;   // per set: last staging that touched it, its index there
  uint32_t stage_count = 0;
  uint32_t* d_acc_slot = nullptr; uint32_t* d_arena = nullptr;
  int64_t* d_set_sum = nullptr; uint32_t* d_bitmap = nullptr;
  uint64_t arena_used = 0;          // arena rows reserved by the batches run since the last reset
  // signer slots (load generator)
  uint32_t n_signers = 0;
  uint32_t *d_sk_scal = nullptr, *d_sk_araw = nullptr, *d_sk_prefix = nullptr, *d_sk_pub = nullptr;
  Slot slots[kSlots];
  // txv_sig_keys scratch: signatures [n][16] u32, lengths, keys [n][8] u32
  uint32_t pk_cap = 0;
  uint32_t *d_pk_sig = nullptr, *d_pk_len = nullptr, *d_pk_keys = nullptr;
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
};

#define HIP_TRY(ctx, x)                                                                    \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
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
  explicit HostTimer(bool o) : on(o), t(std::chrono::steady_clock::now()) {}
  void mark(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    char b[64];
    snprintf(b, sizeof b, " %s=%.3fms", what, std::chrono::duration<double, std::milli>(now - t).count());
    line += b;
    t = now;
  }
  ~HostTimer() { if (on && !line.empty()) fprintf(stderr, "[txv host]%s\n", line.c_str()); }
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
        (c->lane_votes == 1 && (r = dalloc(c, &s.d_rpts, (size_t)TXV_RPTS_WORDS * npad))) ||
        (r = dalloc(c, &s.d_order, npad)) || (r = halloc(c, &s.h_order, npad)) ||
        (r = dalloc(c, &s.d_tvote, npad)) || (r = halloc(c, &s.h_tvote, npad)) ||
        (r = dalloc(c, &s.d_tval, npad)) || (r = halloc(c, &s.h_tval, npad)) ||
        (r = dalloc(c, &s.d_ent_vote, npad)) || (r = dalloc(c, &s.d_ent_power, npad)) ||
        (r = dalloc(c, &s.d_ent_val, npad)) ||
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
  if (s.touched_cap < need) {
    int r;
    if ((r = dalloc(c, &s.d_touched, need)) || (r = dalloc(c, &s.d_tsum, need)) || (r = dalloc(c, &s.d_tmaj, need)) ||
        (r = dalloc(c, &s.d_toff, need + 1)) || (r = halloc(c, &s.h_toff, need + 1)) ||
        (r = dalloc(c, &s.d_tcross, need)) || (r = halloc(c, &s.h_touched, need)) ||
        (r = halloc_mapped(c, &s.h_tsum, &s.m_tsum, need)) || (r = halloc_mapped(c, &s.h_tmaj, &s.m_tmaj, need)) ||
        (r = halloc_mapped(c, &s.h_tcross, &s.m_tcross, need)))
      return r;
    s.touched_cap = need;
  }
  if (!s.ev[0])
    for (auto& e : s.ev) HIP_TRY(c, hipEventCreate(&e));
  return TXV_OK;
}

int alloc_tally(txv_ctx* c) {
  const size_t cells = (size_t)c->cfg.max_txs * std::max<uint32_t>(c->n_vals, 1);
  int r;
  if ((r = dalloc(c, &c->d_acc_slot, cells)) || (r = dalloc(c, &c->d_arena, (size_t)c->cfg.max_accepted * 16)) ||
      (r = dalloc(c, &c->d_set_sum, c->cfg.max_txs)) || (r = dalloc(c, &c->d_bitmap, (c->cfg.max_txs + 31) / 32)))
    return r;
  return TXV_OK;
}

int reset_tally(txv_ctx* c, bool keep_ids = false) {
  const size_t cells = (size_t)c->cfg.max_txs * std::max<uint32_t>(c->n_vals, 1);
  HIP_TRY(c, hipMemsetAsync(c->d_acc_slot, 0, cells * 4, c->stream));
  HIP_TRY(c, hipMemsetAsync(c->d_set_sum, 0, (size_t)c->cfg.max_txs * 8, c->stream));
  HIP_TRY(c, hipMemsetAsync(c->d_bitmap, 0, (size_t)(c->cfg.max_txs + 31) / 32 * 4, c->stream));
  c->arena_used = 0;
  if (keep_ids) {
    std::fill(c->h_sum.begin(), c->h_sum.end(), 0);
    std::fill(c->h_maj.begin(), c->h_maj.end(), 0);
    return TXV_OK;
  }
  c->tx_tab.clear();
  c->h_sum.clear();
  c->h_maj.clear();
  c->seen_stage.clear();
  c->set_tidx.clear();
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
  if (s.n_touched)
    HIP_TRY(c, hipMemcpyAsync(s.d_touched, s.h_touched, (size_t)s.n_touched * 4, hipMemcpyHostToDevice, c->copy_stream));
  if (s.n_work)
    HIP_TRY(c, hipMemcpyAsync(s.d_order, s.h_order, (size_t)s.n_work * 4, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipEventRecord(s.ev[3], c->copy_stream));   // kernels on c->stream wait for it
  return TXV_OK;
}

// set-major tally order (AddVote path): stable counting sort of the validator-sorted pending
// votes (h_order) by touched-set index gives (set, validator, arrival) order
int build_set_order(txv_ctx* c, Slot& s) {
  // stable by touched-set index over the validator-sorted pending votes
  txv_host::counting_sort(*c->pool, s.n_work, s.n_touched,
      [&](uint32_t q) { return c->set_tidx[s.h_set[s.h_order[q]]]; },
      [&](uint32_t p, uint32_t q) {
        const uint32_t i = s.h_order[q];
        s.h_tvote[p] = i;
        s.h_tval[p] = s.h_val[i] | ((s.h_flags[i] & TXV_FLAG_SIG64) ? 0x80000000u : 0u) |
                      ((s.h_flags[i] & TXV_FLAG_BADMSG) ? 0x40000000u : 0u);
      }, s.h_toff);
  HIP_TRY(c, hipMemcpyAsync(s.d_toff, s.h_toff, (size_t)(s.n_touched + 1) * 4, hipMemcpyHostToDevice, c->copy_stream));
  if (s.n_work) {
    HIP_TRY(c, hipMemcpyAsync(s.d_tvote, s.h_tvote, (size_t)s.n_work * 4, hipMemcpyHostToDevice, c->copy_stream));
    HIP_TRY(c, hipMemcpyAsync(s.d_tval, s.h_tval, (size_t)s.n_work * 4, hipMemcpyHostToDevice, c->copy_stream));
  }
  HIP_TRY(c, hipEventRecord(s.ev[3], c->copy_stream));   // run_slot's kernels wait for this
  return TXV_OK;
}

// Counting sort of the pending votes by validator (keys = validator or caller-key index <
// n_keys).  The tally's set-major order is built from it; K1b walks it only with the small
// tables (verify_args).
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
VerifyArgs verify_args(txv_ctx* c, Slot& s, const uint32_t* pubs, const uint8_t* dok, const uint32_t* tabs, int w) {
  VerifyArgs a{};
  a.n = s.n; a.n_pad = s.n_pad; a.msg_words = s.msg_words;
  a.sig = s.d_sig; a.msg = s.d_msg; a.msg_len = s.d_msg_len; a.val = s.d_val; a.flags = s.d_flags;
  const bool by_val = w <= 12;
  a.n_work = by_val || !s.n_work ? s.n_work : s.n; a.kbuf = s.d_kbuf;
  a.order = by_val ? s.d_order : nullptr; a.pubs_le = pubs; a.decode_ok = dok; a.atables = tabs; a.btable = c->d_btable;
  a.ok_out = s.d_ok;
  a.park = c->d_park;
  a.rpts = s.d_rpts;
  a.lane_votes = c->lane_votes;
  return a;
}

// K1b votes per lane for a launch with base window wb.  V = 8 halves the inversions per vote
// but also the waves; with the divstep inverse it wins once the batch still fills >= 1.5 waves
// per SIMD (C2, 1M votes: 517 vs 503-512M votes/s, profiles/r01/inv_var, profiles/r01/park);
// smaller batches (C5's 64k) keep V = 4.  V = 8 kernels exist for the radix-2^24 base table.
uint32_t launch_lane_votes(const txv_ctx* c, int wb, uint32_t n_work) {
  return (c->lane_auto && wb == 24 && n_work >= (3u << 18)) ? 8u : c->lane_votes;
}

// scratch for the parked results per K1b lane (V slots: the last one with TXV_PARK_LAST) (the grid never exceeds verify_grid's cap)
int ensure_park(txv_ctx* c) {
  if (c->lane_votes == 1) return TXV_OK;   // split mode parks nothing
  const size_t words = (size_t)(c->lane_auto ? 8u : c->lane_votes) * TXV_PARK_WORDS * (size_t)c->n_cus * 2 * TXV_VERIFY_BLOCK;
  if (words <= c->park_words) return TXV_OK;
  int r;
  if ((r = dalloc(c, &c->d_park, words))) return r;
  c->park_words = words;
  return TXV_OK;
}

TallyArgs tally_args(txv_ctx* c, Slot& s, uint32_t arena_base) {
  TallyArgs a{};
  a.n = s.n; a.n_pad = s.n_pad; a.n_vals = c->n_vals; a.n_touched = s.n_touched;
  a.quorum = c->quorum; a.arena_base = arena_base;
  a.sig = s.d_sig; a.ok = s.d_ok; a.pre = s.d_pre; a.status = s.d_status;
  a.touched = s.d_touched; a.toff = s.d_toff; a.tvote = s.d_tvote; a.tval = s.d_tval;
  a.ent_vote = s.d_ent_vote; a.ent_power = s.d_ent_power; a.ent_val = s.d_ent_val;
  a.acc_slot = c->d_acc_slot; a.arena = c->d_arena;
  a.power = c->d_power; a.set_sum = c->d_set_sum; a.commit_bitmap = c->d_bitmap;
  a.t_sum = s.m_tsum; a.t_maj = s.m_tmaj; a.t_cross = s.m_tcross;   // mapped host memory
  a.status_host = s.m_out;
  return a;
}

// stage for the AddVote path: routing, pre-checks, SignBytes, pack, upload
// Device SignBytes for slot s: stage the raw fields + the TxHash arena prefix
// [0, arena_end) into pinned buffers (parallel), upload them on the copy stream and build the
// column-major message words there with txv_k_signbytes.  s.h_msg_len must be set already.
int encode_signbytes_device(txv_ctx* c, Slot& s, const txv_votes* v, const uint8_t* d_chain, uint32_t chain_len,
                            uint64_t arena_end) {
  const uint32_t n = s.n, np = s.n_pad;
  if (arena_end + 1 > s.arena_cap) {
    int r;
    const size_t cap = std::max<size_t>((size_t)arena_end + 1, s.arena_cap * 2);
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
  HIP_TRY(c, hipMemcpyAsync(s.d_fh, s.h_fh, (size_t)n * 8, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_fs, s.h_fs, (size_t)n * 8, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_fn, s.h_fn, (size_t)n * 4, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_fo, s.h_fo, (size_t)n * 4, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipMemcpyAsync(s.d_fl, s.h_fl, (size_t)n * 4, hipMemcpyHostToDevice, c->copy_stream));
  if (arena_end) HIP_TRY(c, hipMemcpyAsync(s.d_arena_th, s.h_arena, (size_t)arena_end, hipMemcpyHostToDevice, c->copy_stream));
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
  if (len + 1 > *cap) {
    int r;
    if ((r = dalloc(c, d, (size_t)len + 1))) return r;
    *cap = len + 1;
  }
  if (len) HIP_TRY(c, hipMemcpyAsync(*d, chain, len, hipMemcpyHostToDevice, c->copy_stream));
  HIP_TRY(c, hipStreamSynchronize(c->copy_stream));
  return TXV_OK;
}

int stage_add(txv_ctx* c, uint32_t slot, const txv_votes* v) {
  if (!c->n_vals) { c->err = "no validator set"; return TXV_ESTATE; }
  if (v->n > c->cfg.max_batch) { c->err = "batch exceeds max_batch"; return TXV_ECAPACITY; }
  Slot& s = c->slots[slot];
  const uint32_t n = v->n;
  const uint32_t chain_len = (uint32_t)c->chain.size();
  HostTimer ht(c->profile_host);
  // phase A (parallel): SignBytes lengths, TxHash hashes, validator lookups
  s.lens.resize(n); s.khash.resize(n); s.vidx.resize(n);
  std::atomic<uint32_t> mx{0};
  std::atomic<uint64_t> arena_end{0};
  c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
    uint32_t m = 0;
    uint64_t ae = 0;
    for (uint32_t i = lo; i < hi; ++i) {
      if (v->is_nil && v->is_nil[i]) { s.lens[i] = -2; continue; }
      ae = std::max<uint64_t>(ae, (uint64_t)v->txhash_off[i] + v->txhash_len[i]);
      const int L = txv_host::sign_bytes_len(v->height[i], v->txhash_len[i], v->ts_sec[i], v->ts_nanos[i], chain_len);
      s.lens[i] = L;
      if (L > 0 && (uint32_t)L > m) m = (uint32_t)L;
      s.khash[i] = c->tx_tab.hash(v->txhash + v->txhash_off[i], v->txhash_len[i]);
      s.vidx[i] = v->addr_len[i] == 20 ? c->addr_tab.find(v->addr + (size_t)i * 20) : UINT32_MAX;
    }
    uint32_t cur = mx.load();
    while (m > cur && !mx.compare_exchange_weak(cur, m)) {}
    uint64_t ca = arena_end.load();
    while (ae > ca && !arena_end.compare_exchange_weak(ca, ae)) {}
  });
  const uint32_t mw = std::max<uint32_t>(1, (mx.load() + 7) / 8);
  ht.mark("A");
  int r = ensure_slot(c, s, n, mw);
  if (r) return r;
  s.n = n; s.n_pad = (n + 63) / 64 * 64; s.msg_words = mw;
  // phase B: TxHash -> set id, created on first sight in arrival order (txflow/service.go:200-209,
  // also for votes that then fail), touched-set list, the AddVote pre-checks (types/vote_set.go:92-105).
  // B1 (parallel): lookups of existing sets (read-only table) and the per-vote pre-checks;
  // B2 (sequential, arrival order): the misses are interned -- new sets get their ids in
  // first-seen order exactly as a sequential pass would assign them; B3: touched-set list.
  const uint32_t stage_id = ++c->stage_count;
  s.n_touched = 0;
  std::vector<uint32_t>& miss = s.miss;
  c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; ++i) {
      s.h_flags[i] = 0; s.h_val[i] = 0;
      if (s.lens[i] == -2) { s.h_status[i] = TXV_ERR_NIL; s.h_set[i] = UINT32_MAX - 1; continue; }
      s.h_set[i] = c->tx_tab.find(v->txhash + v->txhash_off[i], v->txhash_len[i], s.khash[i]);
      if (v->addr_len[i] == 0) { s.h_status[i] = TXV_ERR_EMPTY_ADDR; continue; }
      const uint32_t vi = s.vidx[i];
      if (vi == UINT32_MAX) { s.h_status[i] = TXV_ERR_UNKNOWN_VALIDATOR; continue; }
      s.h_val[i] = vi;
      // a SignBytes failure is only reached after the accepted-vote check (AddVote order), so
      // the vote stays pending with BADMSG: it never verifies and the tally resolves it
      s.h_status[i] = 0xFF;
      s.h_flags[i] = TXV_FLAG_PENDING | (v->sig_len[i] == 64 ? TXV_FLAG_SIG64 : 0) | (s.lens[i] < 0 ? TXV_FLAG_BADMSG : 0);
    }
  }, 4096);
  miss.clear();
  for (uint32_t i = 0; i < n; ++i)
    if (s.h_set[i] == UINT32_MAX) miss.push_back(i);
  for (const uint32_t i : miss) {
    bool created;
    const uint32_t sid = c->tx_tab.intern(v->txhash + v->txhash_off[i], v->txhash_len[i], s.khash[i], &created,
                                          c->cfg.max_txs);
    if (sid == UINT32_MAX) { c->err = "TxVoteSets exceed max_txs"; return TXV_ECAPACITY; }
    if (created) {
      c->h_sum.push_back(0); c->h_maj.push_back(0); c->seen_stage.push_back(0); c->set_tidx.push_back(0);
    }
    s.h_set[i] = sid;
  }
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t sid = s.h_set[i];
    if (sid == UINT32_MAX - 1) { s.h_set[i] = 0; continue; }   // nil vote: no set
    if (c->seen_stage[sid] != stage_id) {
      c->seen_stage[sid] = stage_id;
      c->set_tidx[sid] = s.n_touched;
      s.h_touched[s.n_touched++] = sid;
    }
  }
  ht.mark("B");
  // phase C (parallel): column-major signature words and lengths; the SignBytes words are
  // built on the device (encode_signbytes_device)
  const uint32_t np = s.n_pad;
  c->pool->parallel_for(np, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; ++i) {
      if (i >= n) {
        for (int j = 0; j < 16; ++j) s.h_sig[(size_t)j * np + i] = 0;
        s.h_msg_len[i] = 0; s.h_val[i] = 0; s.h_set[i] = 0; s.h_flags[i] = 0; s.h_status[i] = TXV_ERR_NIL;
        continue;
      }
      uint8_t sg[64];
      const uint32_t sl = v->sig_len[i] > 64 ? 64 : v->sig_len[i];
      memset(sg, 0, 64);
      memcpy(sg, v->sig + (size_t)i * 64, sl);
      for (int j = 0; j < 16; ++j) s.h_sig[(size_t)j * np + i] = le32(sg + 4 * j);
      s.h_msg_len[i] = s.lens[i] > 0 ? (uint32_t)s.lens[i] : 0;
    }
  }, 1024);
  ht.mark("C");
  build_order(c, s, c->n_vals);
  ht.mark("order");
  if ((r = encode_signbytes_device(c, s, v, c->d_chain, chain_len, arena_end.load()))) return r;
  ht.mark("signbytes");
  if ((r = upload_slot(c, s))) return r;
  ht.mark("upload");
  if ((r = build_set_order(c, s))) return r;
  ht.mark("set_order");
  s.staged = true; s.ran = false;
  return TXV_OK;
}

int run_slot(txv_ctx* c, uint32_t slot, float* ms) {
  Slot& s = c->slots[slot];
  if (!s.staged) { c->err = "slot not staged"; return TXV_ESTATE; }
  // arena rows [arena_used, arena_used + n) are this batch's (row = base + arrival index)
  if (c->arena_used + s.n > c->cfg.max_accepted) { c->err = "accepted-signature arena full"; return TXV_ECAPACITY; }
  const uint32_t arena_base = (uint32_t)c->arena_used;
  c->arena_used += s.n;
  int r;
  if ((r = ensure_park(c))) return r;
  HIP_TRY(c, hipStreamWaitEvent(c->stream, s.ev[3], 0));
  HIP_TRY(c, hipEventRecord(s.ev[0], c->stream));
  VerifyArgs va = verify_args(c, s, c->d_pubs, c->d_decode_ok, c->d_atables, c->tab_w);
  va.lane_votes = launch_lane_votes(c, c->b_w, va.n_work);
  HIP_TRY(c, txv_launch_verify(c->b_w, c->tab_w, &va, verify_grid(c, s.n), c->stream));
  HIP_TRY(c, hipEventRecord(s.ev[1], c->stream));
  TallyArgs ta = tally_args(c, s, arena_base);
  HIP_TRY(c, txv_launch_tally(&ta, c->stream));
  HIP_TRY(c, hipEventRecord(s.ev[2], c->stream));
  // the tally kernels wrote the statuses and per-set results into mapped host memory (no copy
  // engine in the loop); fetch_slot only waits for the kernels
  HIP_TRY(c, hipEventRecord(s.ev[4], c->stream));
  s.ran = true;
  if (ms) {
    HIP_TRY(c, hipEventSynchronize(s.ev[2]));
    HIP_TRY(c, hipEventElapsedTime(&ms[0], s.ev[0], s.ev[1]));
    HIP_TRY(c, hipEventElapsedTime(&ms[1], s.ev[1], s.ev[2]));
    ms[2] = ms[0] + ms[1];
  }
  return TXV_OK;
}

int fetch_slot(txv_ctx* c, uint32_t slot, uint8_t* status_out, txv_commit_event* ev, uint32_t ev_cap, uint32_t* n_ev) {
  Slot& s = c->slots[slot];
  if (!s.ran) { c->err = "slot not run"; return TXV_ESTATE; }
  HostTimer ht(c->profile_host);
  HIP_TRY(c, hipEventSynchronize(s.ev[4]));
  ht.mark("fetch_sync");
  if (status_out) memcpy(status_out, s.h_out, s.n);
  ht.mark("fetch_copy");
  uint32_t ne = 0;
  for (uint32_t t = 0; t < s.n_touched; ++t) {
    const uint32_t sid = s.h_touched[t];
    c->h_sum[sid] = s.h_tsum[t];
    c->h_maj[sid] = s.h_tmaj[t];
    if (s.h_tcross[t] != TXV_NO_CROSS) {
      if (ev && ne < ev_cap) ev[ne] = txv_commit_event{s.h_tcross[t], sid, s.h_tsum[t]};
      ++ne;
    }
  }
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

// make tab_w = w current: its B table exists; then the verify kernel's base-point window
// b_w: the requested one if the kernels support (b_w, w), else by default the 8.9 GB
// radix-2^24 table over radix-2^16 validator tables (11 instead of 16 additions for [s]B;
// measured 2.06 vs 2.23 ms per 1M-vote verify, W_B = 22: 2.11), falling back to b_w = w
// when the wide table cannot be allocated.  d_btable = table of b_w.
int select_window(txv_ctx* c, int w) {
  int r;
  // radix-2^18 / 2^20 validator tables only run against the radix-2^24 base table
  if (w != 4 && w <= 16 && (r = build_base_table(c, w))) return r;
  c->tab_w = w;
  c->d_btable = w == 4 ? c->d_btable4 : c->d_btable8;
  c->b_w = w;
  int bw = c->cfg_bw ? c->cfg_bw : (w >= 12 ? 24 : w);
  if ((c->lane_votes < 4 && c->lane_votes != 1) || !txv_verify_windows_supported(bw, w)) bw = w;
  if (bw != w) {
    if (c->btable_wide_w != bw) {
      dfree(c->d_btable_wide);
      c->btable_wide_w = 0;
      if (hipMalloc((void**)&c->d_btable_wide, table_words(bw) * 4) != hipSuccess) {
        (void)hipGetLastError();
        c->d_btable_wide = nullptr;
        return TXV_OK;                       // no room: stay at b_w = w
      }
      uint32_t* d_b = nullptr;
      if ((r = dalloc(c, &d_b, 8))) return r;
      const uint32_t bwords[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                                  0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
      HIP_TRY(c, hipMemcpyAsync(d_b, bwords, 32, hipMemcpyHostToDevice, c->stream));
      HIP_TRY(c, txv_launch_build_tables(bw, d_b, 1, c->d_btable_wide, nullptr, nullptr, c->stream));
      HIP_TRY(c, hipStreamSynchronize(c->stream));
      dfree(d_b);
      c->btable_wide_w = bw;
    }
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
};

KeySet registry_keys(const txv_ctx* c) { return KeySet{c->d_pubs, c->d_decode_ok, c->d_atables, c->tab_w}; }

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
  ks = KeySet{c->d_tmp_pubs, c->d_tmp_ok, c->d_tmp_tables, w_keys};
  return TXV_OK;
}

// Upload slot s and run K1 (verify only) against key set ks; ok[i] = 1 when vote i verified.
int run_verify(txv_ctx* c, Slot& s, const KeySet& ks, std::vector<uint8_t>& ok) {
  int r;
  if ((r = upload_slot(c, s)) || (r = ensure_park(c))) return r;
  HIP_TRY(c, hipStreamWaitEvent(c->stream, s.ev[3], 0));
  VerifyArgs va = verify_args(c, s, ks.pubs, ks.ok, ks.tables, ks.w);
  const bool reg_w = ks.w == c->tab_w;
  const int w_base = reg_w ? c->b_w : ks.w;
  va.btable = reg_w ? c->d_btable : (ks.w == 4 ? c->d_btable4 : c->d_btable8);
  va.lane_votes = launch_lane_votes(c, w_base, va.n_work);
  HIP_TRY(c, txv_launch_verify(w_base, ks.w, &va, verify_grid(c, s.n), c->stream));
  ok.resize(s.n);
  if (s.n) HIP_TRY(c, hipMemcpyAsync(ok.data(), s.d_ok, s.n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return TXV_OK;
}

// txv_submit_votes ring: ticket t runs in slot (t - 1) % 2; a slot is reused only after
// its ticket was waited for (its pinned and device buffers are free again)
int submit_votes(txv_ctx* c, const txv_votes* v, uint64_t* ticket) {
  const uint64_t t = c->next_ticket;
  const uint32_t slot = (uint32_t)((t - 1) % 2);
  Slot& s = c->slots[slot];
  if (s.ticket) { c->err = "two batches already in flight: wait for the older one first"; return TXV_ESTATE; }
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
  Slot& s = c->slots[(ticket - 1) % 2];
  if (s.ticket != ticket) { c->err = "unknown or already waited ticket"; return TXV_ESTATE; }
  const uint32_t other = (uint32_t)(ticket % 2);   // the other ring slot
  if (c->slots[other].ticket && c->slots[other].ticket < ticket) {
    c->err = "tickets must be waited in submission order";
    return TXV_ESTATE;
  }
  s.ticket = 0;
  return fetch_slot(c, (uint32_t)((ticket - 1) % 2), status_out, ev, ev_cap, n_ev);
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
  if (!c->cfg.max_accepted) c->cfg.max_accepted = (uint32_t)std::min<uint64_t>((uint64_t)c->cfg.max_txs * 128, 1u << 28);
  if (!c->cfg.max_msg_bytes) c->cfg.max_msg_bytes = 256;
  if (!c->cfg.table_budget_mb) c->cfg.table_budget_mb = 80u << 10;   // 80 GiB of the 288 GB HBM
  c->cfg_w = (c->cfg.flags & TXV_CFG_TABLE_W4) ? 4 : 0;
  if (TXV_CFG_WINDOW(c->cfg.flags)) c->cfg_w = (int)TXV_CFG_WINDOW(c->cfg.flags);
  if (c->cfg_w && !valid_window(c->cfg_w)) { delete c; return TXV_EINVAL; }
  if (TXV_CFG_LANE_VOTES(c->cfg.flags)) { c->lane_votes = TXV_CFG_LANE_VOTES(c->cfg.flags); c->lane_auto = false; }
  if (c->lane_votes != 1 && c->lane_votes != 2 && c->lane_votes != 4 && c->lane_votes != 8) { delete c; return TXV_EINVAL; }
  c->cfg_bw = (int)TXV_CFG_B_WINDOW(c->cfg.flags);
  if (c->cfg_bw && c->cfg_bw != 4 && !valid_window(c->cfg_bw) && c->cfg_bw != 20 && c->cfg_bw != 22 && c->cfg_bw != 24) {
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
  if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->key_stream, hipStreamNonBlocking) != hipSuccess) {
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
  for (auto& s : c->slots) {
    dfree(s.d_sig); dfree(s.d_msg); dfree(s.d_msg_len); dfree(s.d_val); dfree(s.d_set); dfree(s.d_flags);
    dfree(s.d_status); dfree(s.d_ok); dfree(s.d_pre); dfree(s.d_kbuf); dfree(s.d_rpts); dfree(s.d_order); hfree(s.h_order);
    dfree(s.d_toff); hfree(s.h_toff); dfree(s.d_tvote); hfree(s.h_tvote); dfree(s.d_tval); hfree(s.h_tval);
    dfree(s.d_ent_vote); dfree(s.d_ent_power); dfree(s.d_ent_val); dfree(s.d_touched); dfree(s.d_tsum); dfree(s.d_tmaj); dfree(s.d_tcross);
    hfree(s.h_sig); hfree(s.h_msg); hfree(s.h_msg_len); hfree(s.h_val); hfree(s.h_set); hfree(s.h_flags);
    hfree(s.h_status); hfree(s.h_touched); hfree(s.h_tsum); hfree(s.h_tmaj); hfree(s.h_tcross); hfree(s.h_out);
    hfree(s.h_fh); hfree(s.h_fs); hfree(s.h_fn); hfree(s.h_fo); hfree(s.h_fl); hfree(s.h_arena);
    dfree(s.d_fh); dfree(s.d_fs); dfree(s.d_fn); dfree(s.d_fo); dfree(s.d_fl); dfree(s.d_arena_th);
    for (auto& e : s.ev) if (e) (void)hipEventDestroy(e);
  }
  dfree(c->d_pubs); dfree(c->d_decode_ok); dfree(c->d_atables); dfree(c->d_addr); dfree(c->d_power);
  dfree(c->d_btable4); dfree(c->d_btable8); dfree(c->d_park); dfree(c->d_btable_wide); c->d_btable = nullptr; dfree(c->d_tmp_pubs); dfree(c->d_tmp_ok); dfree(c->d_tmp_tables); dfree(c->d_tmp_addr);
  dfree(c->d_acc_slot); dfree(c->d_arena); dfree(c->d_set_sum); dfree(c->d_bitmap);
  dfree(c->d_sk_scal); dfree(c->d_sk_araw); dfree(c->d_sk_prefix); dfree(c->d_sk_pub);
  dfree(c->d_chain); dfree(c->d_chain_sign);
  dfree(c->d_pk_sig); dfree(c->d_pk_len); dfree(c->d_pk_keys); hfree(c->h_pk_sig); hfree(c->h_pk_len); hfree(c->h_pk_keys);
  dfree(c->d_wd_wire); hfree(c->h_wd_wire); dfree(c->d_wd_off); hfree(c->h_wd_off); dfree(c->d_wd_len); hfree(c->h_wd_len);
  dfree(c->d_wd_out); hfree(c->h_wd_out); dfree(c->d_wd_span); hfree(c->h_wd_span);
  for (auto& e : c->wd_ev) if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->key_stream) (void)hipStreamDestroy(c->key_stream);
  delete c;
}

const char* txv_last_error(txv_ctx* c) { return c ? c->err.c_str() : "null context"; }

int txv_device_name(txv_ctx* c, char* buf, uint32_t cap) {
  if (!c || !buf || !cap) return TXV_EINVAL;
  hipDeviceProp_t p;
  HIP_TRY(c, hipGetDeviceProperties(&p, c->device));
  snprintf(buf, cap, "%s (%s, %d CUs)", p.name, p.gcnArchName, p.multiProcessorCount);
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
  if ((r = select_window(c, choose_window(c, n)))) return r;
  if ((r = dalloc(c, &c->d_pubs, (size_t)n * 8)) || (r = dalloc(c, &c->d_decode_ok, n)) ||
      (r = dalloc(c, &c->d_atables, (size_t)n * table_words(c->tab_w))) || (r = dalloc(c, &c->d_addr, (size_t)n * 5)) ||
      (r = dalloc(c, &c->d_power, n)))
    return r;
  if (n) {
    HIP_TRY(c, hipMemcpyAsync(c->d_pubs, pubs32, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->d_power, powers, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, txv_launch_build_tables(c->tab_w, c->d_pubs, n, c->d_atables, c->d_decode_ok, c->d_addr, c->stream));
  }
  c->addrs.resize((size_t)n * 20);
  c->decode_ok.resize(n);
  if (n) {
    HIP_TRY(c, hipMemcpyAsync(c->addrs.data(), c->d_addr, (size_t)n * 20, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->decode_ok.data(), c->d_decode_ok, n, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->addr_index.clear();
  for (uint32_t i = 0; i < n; ++i) c->addr_index.emplace(std::string((const char*)c->addrs.data() + 20 * i, 20), i);
  c->addr_tab.build(c->addrs.data(), n);
  if ((r = alloc_tally(c))) return r;
  return reset_tally(c);
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
  Slot& s = c->slots[kSlots - 1];
  std::vector<int> lens;
  const uint32_t mx = encode_all(c, s, v, c->chain.data(), (uint32_t)c->chain.size(), lens);
  const uint32_t mw = std::max<uint32_t>(1, (mx + 7) / 8);
  int r = ensure_slot(c, s, v->n, mw);
  if (r) return r;
  s.n = v->n; s.n_pad = (v->n + 63) / 64 * 64; s.msg_words = mw; s.n_touched = 0;
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
  Slot& s = c->slots[kSlots - 1];
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
  s.n = n; s.n_pad = (n + 63) / 64 * 64; s.msg_words = mw; s.n_touched = 0;
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
      const Slot& s = c->slots[(ticket - 1) % 2];
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

int txv_query_tx(txv_ctx* c, const uint8_t* txhash, uint32_t len, int64_t* sum, uint8_t* maj23) {
  if (!c) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!txhash && len) return TXV_EINVAL;
  const uint32_t sid = c->tx_tab.find(txhash, len, c->tx_tab.hash(txhash, len));
  if (sid == UINT32_MAX) return 0;
  if (sum) *sum = c->h_sum[sid];
  if (maj23) *maj23 = c->h_maj[sid];
  return 1;
}

int txv_get_votes(txv_ctx* c, const uint8_t* txhash, uint32_t len, uint32_t* val_out, uint64_t* seq_out,
                  uint8_t* sig_out, uint32_t cap, uint32_t* n_out) {
  if (!c || (!txhash && len) || !n_out) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  *n_out = 0;
  const uint32_t sid = c->tx_tab.find(txhash, len, c->tx_tab.hash(txhash, len));
  if (sid == UINT32_MAX || !c->n_vals) return TXV_OK;
  uint32_t *d_rows = nullptr, *d_sigs = nullptr;
  int r;
  if ((r = dalloc(c, &d_rows, c->n_vals)) || (r = dalloc(c, &d_sigs, (size_t)c->n_vals * 16))) { dfree(d_rows); return r; }
  std::vector<uint32_t> rows(c->n_vals), sigs((size_t)c->n_vals * 16);
  // stream order: after every batch already submitted on this context
  hipError_t e = txv_launch_set_votes(c->d_acc_slot + (size_t)sid * c->n_vals, c->n_vals, c->d_arena, d_rows, d_sigs,
                                      c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(rows.data(), d_rows, (size_t)c->n_vals * 4, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(sigs.data(), d_sigs, (size_t)c->n_vals * 64, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(d_rows); dfree(d_sigs);
  HIP_TRY(c, e);
  uint32_t k = 0;
  for (uint32_t v = 0; v < c->n_vals; ++v) {
    if (!rows[v]) continue;
    if (k < cap) {
      if (val_out) val_out[k] = v;
      if (seq_out) seq_out[k] = rows[v] - 1;
      if (sig_out) memcpy(sig_out + (size_t)k * 64, sigs.data() + (size_t)v * 16, 64);
    }
    ++k;
  }
  *n_out = k;
  return TXV_OK;
}

uint32_t txv_num_tx_sets(txv_ctx* c) { return c ? c->tx_tab.size() : 0; }
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
  Slot& s = c->slots[kSlots - 2];
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
  s.n = v->n; s.n_pad = (v->n + 63) / 64 * 64; s.msg_words = mw; s.n_touched = 0; s.n_work = 0;
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
  if (!c || !v || slot >= kSlots - 2) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  int r = stage_add(c, slot, v);
  if (r) return r;
  HIP_TRY(c, hipStreamSynchronize(c->copy_stream));   // resident before any timed run
  return TXV_OK;
}

int txv_run_staged(txv_ctx* c, uint32_t slot, float* ms) {
  if (!c || slot >= kSlots - 2) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  return run_slot(c, slot, ms);
}

int txv_fetch_staged(txv_ctx* c, uint32_t slot, uint8_t* status_out, txv_commit_event* ev, uint32_t ev_cap,
                     uint32_t* n_ev) {
  if (!c || slot >= kSlots - 2) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  return fetch_slot(c, slot, status_out, ev, ev_cap, n_ev);
}

int txv_commit_bitmap(txv_ctx* c, void** dev_ptr, uint64_t* bytes) {
  if (!c || !dev_ptr || !bytes) return TXV_EINVAL;
  *dev_ptr = c->d_bitmap;
  *bytes = (uint64_t)(c->cfg.max_txs + 31) / 32 * 4;
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

extern "C" {

int txv_sig_keys(txv_ctx* c, const txv_votes* v, const uint8_t* sig_full, const uint64_t* sig_full_off,
                 uint8_t* keys_out) {
  if (!c || !v || (v->n && (!v->sig || !v->sig_len || !keys_out))) return TXV_EINVAL;
  const uint32_t n = v->n;
  for (uint32_t i = 0; i < n; ++i)
    if (v->sig_len[i] > 64 && (!sig_full || !sig_full_off)) { c->err = "signature > 64 bytes without sig_full"; return TXV_EINVAL; }
  std::lock_guard<std::mutex> g(c->mu);
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
  c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
    memcpy(c->h_pk_sig + (size_t)lo * 16, v->sig + (size_t)lo * 64, (size_t)(hi - lo) * 64);
    memcpy(c->h_pk_len + lo, v->sig_len + lo, (size_t)(hi - lo) * 4);
  }, 8192);
  HIP_TRY(c, hipMemcpyAsync(c->d_pk_sig, c->h_pk_sig, (size_t)n * 64, hipMemcpyHostToDevice, c->key_stream));
  HIP_TRY(c, hipMemcpyAsync(c->d_pk_len, c->h_pk_len, (size_t)n * 4, hipMemcpyHostToDevice, c->key_stream));
  HIP_TRY(c, txv_launch_sig_keys(c->d_pk_sig, c->d_pk_len, n, c->d_pk_keys, c->key_stream));
  HIP_TRY(c, hipMemcpyAsync(c->h_pk_keys, c->d_pk_keys, (size_t)n * 32, hipMemcpyDeviceToHost, c->key_stream));
  HIP_TRY(c, hipStreamSynchronize(c->key_stream));
  c->pool->parallel_for(n, [&](uint32_t lo, uint32_t hi) {
    memcpy(keys_out + (size_t)lo * 32, c->h_pk_keys + (size_t)lo * 8, (size_t)(hi - lo) * 32);
    for (uint32_t i = lo; i < hi; ++i)
      if (v->sig_len[i] > 64) sha256_host(sig_full + sig_full_off[i], v->sig_len[i], keys_out + (size_t)i * 32);
  }, 8192);
  return TXV_OK;
}

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

int txv_sync(txv_ctx* c) {
  if (!c) return TXV_EINVAL;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return TXV_OK;
}

int txv_copy_commit_bitmap(txv_ctx* c, void* dst_dev, uint64_t bytes) {
  if (!c || !dst_dev) return TXV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(c, hipSetDevice(c->device));
  const uint64_t have = (uint64_t)(c->cfg.max_txs + 31) / 32 * 4;
  HIP_TRY(c, hipMemcpyAsync(dst_dev, c->d_bitmap, std::min(bytes, have), hipMemcpyDeviceToDevice, c->stream));
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
