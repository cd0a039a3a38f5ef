/*
 * txflow.c — sequential restatement of the reference's vote routing and stake tally.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 *   txflow/service.go:192-234   TxFlow.addVote: TxVoteSets[vote.TxHash] created on first
 *                               sight (also for votes that then fail), AddVote, commit
 *                               side effects whenever added && HasTwoThirdsMajority (:216)
 *   types/vote_set.go:81-131    TxVoteSet.AddVote/addVote check order:
 *                               nil -> empty address -> unknown validator -> existing vote
 *                               (same signature bytes: (false,nil); else ErrVoteNonDeterministicSignature)
 *                               -> Verify -> addVerifiedVote
 *   types/vote_set.go:143-166   addVerifiedVote: sum += power; maj23 |= sum >= Total*2/3 + 1
 *   types/tx_vote.go:110-119    TxVote.Verify (address check, then ed25519 over SignBytes)
 * Height and TxKey are never checked by the code.
 */
#include "oracle.h"
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define ORC_ERR_SIGNBYTES 8   /* amino rejects the timestamp: the reference panics in SignBytes */

typedef struct { uint8_t sig[64]; uint32_t len; } acc_sig;

struct orc_flow {
  uint32_t n_vals;
  uint8_t* pubs;        /* n_vals x 32 */
  uint8_t* addrs;       /* n_vals x 20 */
  int64_t* powers;
  uint32_t* by_addr;    /* validator indices sorted by address (ValidatorSet.GetByAddress) */
  int64_t total, quorum;
  uint8_t chain[256]; size_t chain_len;
  /* tx hash table: key bytes -> set index */
  uint32_t tx_cap, n_sets;
  uint32_t* tx_slot;    /* tx_cap entries, 0 = empty else set index + 1 */
  uint8_t** set_key; uint32_t* set_key_len;
  int64_t* set_sum; int32_t* set_maj23;
  uint32_t sets_alloc;
  /* accepted votes: (set, val) -> acc_sig, open addressing on 64-bit keys */
  uint64_t acc_cap, n_acc;
  uint64_t* acc_key;    /* 0 = empty, else ((set+1) << 32) | val */
  acc_sig* acc_val;
  uint64_t n_verifies;
};

static uint64_t hash_bytes(const uint8_t* p, uint32_t n) {
  uint64_t h = 1469598103934665603ULL;
  for (uint32_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ULL; }
  return h ^ (h >> 29);
}
static uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

static const uint8_t* g_addr_base;
static int cmp_addr_idx(const void* a, const void* b) {
  return memcmp(g_addr_base + 20 * (*(const uint32_t*)a), g_addr_base + 20 * (*(const uint32_t*)b), 20);
}

orc_flow* orc_flow_new(const uint8_t* pubs32, const int64_t* powers, uint32_t n_vals,
                       const uint8_t* chain_id, size_t chain_len) {
  orc_flow* f = (orc_flow*)calloc(1, sizeof *f);
  f->n_vals = n_vals;
  f->pubs = (uint8_t*)malloc((size_t)n_vals * 32 + 1);
  f->addrs = (uint8_t*)malloc((size_t)n_vals * 20 + 1);
  f->powers = (int64_t*)malloc((size_t)n_vals * 8 + 8);
  f->by_addr = (uint32_t*)malloc((size_t)n_vals * 4 + 4);
  memcpy(f->pubs, pubs32, (size_t)n_vals * 32);
  for (uint32_t i = 0; i < n_vals; ++i) {
    uint8_t h[32];
    orc_sha256(pubs32 + 32 * i, 32, h);
    memcpy(f->addrs + 20 * i, h, 20);
    f->powers[i] = powers[i];
    f->total += powers[i];
    f->by_addr[i] = i;
  }
  g_addr_base = f->addrs;
  qsort(f->by_addr, n_vals, sizeof(uint32_t), cmp_addr_idx);
  f->quorum = f->total * 2 / 3 + 1;
  f->chain_len = chain_len < sizeof f->chain ? chain_len : sizeof f->chain;
  memcpy(f->chain, chain_id, f->chain_len);
  f->tx_cap = 1024;
  f->tx_slot = (uint32_t*)calloc(f->tx_cap, 4);
  f->acc_cap = 4096;
  f->acc_key = (uint64_t*)calloc(f->acc_cap, 8);
  f->acc_val = (acc_sig*)calloc(f->acc_cap, sizeof(acc_sig));
  return f;
}

void orc_flow_free(orc_flow* f) {
  if (!f) return;
  for (uint32_t i = 0; i < f->n_sets; ++i) free(f->set_key[i]);
  free(f->set_key); free(f->set_key_len); free(f->set_sum); free(f->set_maj23);
  free(f->tx_slot); free(f->acc_key); free(f->acc_val);
  free(f->pubs); free(f->addrs); free(f->powers); free(f->by_addr);
  free(f);
}

/* exact-match lookup by address bytes; -1 when absent */
static int64_t val_by_addr(const orc_flow* f, const uint8_t* addr, uint32_t len) {
  if (len != 20) return -1;
  int64_t lo = 0, hi = (int64_t)f->n_vals - 1;
  while (lo <= hi) {
    int64_t mid = (lo + hi) / 2;
    int c = memcmp(f->addrs + 20 * f->by_addr[mid], addr, 20);
    if (c == 0) return f->by_addr[mid];
    if (c < 0) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}

static int64_t find_set(const orc_flow* f, const uint8_t* key, uint32_t len) {
  uint32_t mask = f->tx_cap - 1;
  uint32_t i = (uint32_t)hash_bytes(key, len) & mask;
  for (;;) {
    uint32_t s = f->tx_slot[i];
    if (!s) return -1;
    if (f->set_key_len[s - 1] == len && !memcmp(f->set_key[s - 1], key, len)) return s - 1;
    i = (i + 1) & mask;
  }
}

static void tx_rehash(orc_flow* f) {
  uint32_t ncap = f->tx_cap * 2;
  uint32_t* ns = (uint32_t*)calloc(ncap, 4);
  for (uint32_t s = 0; s < f->n_sets; ++s) {
    uint32_t i = (uint32_t)hash_bytes(f->set_key[s], f->set_key_len[s]) & (ncap - 1);
    while (ns[i]) i = (i + 1) & (ncap - 1);
    ns[i] = s + 1;
  }
  free(f->tx_slot); f->tx_slot = ns; f->tx_cap = ncap;
}

static uint32_t get_or_create_set(orc_flow* f, const uint8_t* key, uint32_t len) {
  int64_t s = find_set(f, key, len);
  if (s >= 0) return (uint32_t)s;
  if ((f->n_sets + 1) * 2 > f->tx_cap) tx_rehash(f);
  if (f->n_sets == f->sets_alloc) {
    uint32_t na = f->sets_alloc ? f->sets_alloc * 2 : 256;
    f->set_key = (uint8_t**)realloc(f->set_key, na * sizeof(uint8_t*));
    f->set_key_len = (uint32_t*)realloc(f->set_key_len, na * 4);
    f->set_sum = (int64_t*)realloc(f->set_sum, na * 8);
    f->set_maj23 = (int32_t*)realloc(f->set_maj23, na * 4);
    f->sets_alloc = na;
  }
  uint32_t id = f->n_sets++;
  f->set_key[id] = (uint8_t*)malloc(len + 1);
  memcpy(f->set_key[id], key, len);
  f->set_key_len[id] = len;
  f->set_sum[id] = 0; f->set_maj23[id] = 0;
  uint32_t mask = f->tx_cap - 1;
  uint32_t i = (uint32_t)hash_bytes(key, len) & mask;
  while (f->tx_slot[i]) i = (i + 1) & mask;
  f->tx_slot[i] = id + 1;
  return id;
}

static acc_sig* acc_find(const orc_flow* f, uint64_t key) {
  uint64_t mask = f->acc_cap - 1, i = mix64(key) & mask;
  for (;;) {
    if (!f->acc_key[i]) return 0;
    if (f->acc_key[i] == key) return &f->acc_val[i];
    i = (i + 1) & mask;
  }
}
static void acc_insert(orc_flow* f, uint64_t key, const uint8_t* sig, uint32_t len) {
  if ((f->n_acc + 1) * 2 > f->acc_cap) {
    uint64_t ncap = f->acc_cap * 2;
    uint64_t* nk = (uint64_t*)calloc(ncap, 8);
    acc_sig* nv = (acc_sig*)calloc(ncap, sizeof(acc_sig));
    for (uint64_t j = 0; j < f->acc_cap; ++j) {
      if (!f->acc_key[j]) continue;
      uint64_t i = mix64(f->acc_key[j]) & (ncap - 1);
      while (nk[i]) i = (i + 1) & (ncap - 1);
      nk[i] = f->acc_key[j]; nv[i] = f->acc_val[j];
    }
    free(f->acc_key); free(f->acc_val); f->acc_key = nk; f->acc_val = nv; f->acc_cap = ncap;
  }
  uint64_t mask = f->acc_cap - 1, i = mix64(key) & mask;
  while (f->acc_key[i]) i = (i + 1) & mask;
  f->acc_key[i] = key;
  memcpy(f->acc_val[i].sig, sig, len > 64 ? 64 : len);
  f->acc_val[i].len = len;
  f->n_acc++;
}

int orc_txvote_verify(const orc_vote* v, const uint8_t* chain_id, size_t chain_len,
                      const uint8_t pub[32]) {
  uint8_t h[32];
  orc_sha256(pub, 32, h);
  if (v->addr_len != 20 || memcmp(h, v->addr, 20)) return ORC_ERR_INVALID_VALIDATOR_ADDRESS;
  uint8_t sb[1024];
  int n = orc_signbytes(v->height, v->txhash, v->txhash_len, v->ts_sec, v->ts_nanos,
                        chain_id, chain_len, sb, sizeof sb);
  if (n < 0) return ORC_ERR_SIGNBYTES;
  if (!orc_ed25519_verify(pub, sb, (size_t)n, v->sig, v->sig_len)) return ORC_ERR_INVALID_SIGNATURE;
  return ORC_ADDED;
}

static int sig_equal(const acc_sig* a, const uint8_t* sig, uint32_t len) {
  if (a->len != len) return 0;
  if (len > 64) return 0;   /* accepted signatures are exactly 64 bytes */
  return memcmp(a->sig, sig, len) == 0;
}

/* One vote through TxFlow.addVote.  code >= 0: the Verify outcome is supplied (ORC_ADDED,
 * ORC_ERR_INVALID_SIGNATURE or ORC_ERR_SIGNBYTES); code < 0: verify here when reached. */
static uint8_t flow_add_one(orc_flow* f, const orc_vote* v, int code, int64_t* sum_after, uint8_t* fired) {
  if (fired) *fired = 0;
  if (v->is_nil) { if (sum_after) *sum_after = 0; return ORC_ERR_NIL; }
  uint32_t s = get_or_create_set(f, v->txhash, v->txhash_len);
  uint8_t st;
  int64_t vi = -1;
  if (v->addr_len == 0) st = ORC_ERR_EMPTY_ADDR;
  else if ((vi = val_by_addr(f, v->addr, v->addr_len)) < 0) st = ORC_ERR_UNKNOWN_VALIDATOR;
  else {
    uint64_t key = ((uint64_t)(s + 1) << 32) | (uint64_t)vi;
    acc_sig* ex = acc_find(f, key);
    if (ex) st = sig_equal(ex, v->sig, v->sig_len) ? ORC_DUPLICATE : ORC_ERR_NONDETERMINISTIC;
    else {
      int ok = code;
      if (ok < 0) { ok = orc_txvote_verify(v, f->chain, f->chain_len, f->pubs + 32 * vi); f->n_verifies++; }
      if (ok == ORC_ADDED) {
        acc_insert(f, key, v->sig, v->sig_len);
        f->set_sum[s] += f->powers[vi];
        if (f->quorum <= f->set_sum[s]) f->set_maj23[s] = 1;
        st = ORC_ADDED;
        if (fired && f->set_maj23[s]) *fired = 1;
      } else st = (uint8_t)ok;
    }
  }
  if (sum_after) *sum_after = f->set_sum[s];
  return st;
}

void orc_flow_add_votes(orc_flow* f, const orc_vote* votes, uint32_t n, const uint8_t* verdicts,
                        uint8_t* status, int64_t* sum_after, uint8_t* fired) {
  for (uint32_t i = 0; i < n; ++i) {
    int code = verdicts ? (verdicts[i] ? ORC_ADDED : ORC_ERR_INVALID_SIGNATURE) : -1;
    status[i] = flow_add_one(f, &votes[i], code, sum_after ? sum_after + i : 0, fired ? fired + i : 0);
  }
}

/* ---- SoA batches (the txv_votes layout): verify in parallel, then the sequential loop ---- */
typedef struct {
  const orc_flow* f;
  const orc_soa* b;
  uint8_t* code;
  uint32_t begin, end;
} soa_job;

static orc_vote soa_vote(const orc_soa* b, uint32_t i) {
  orc_vote v;
  v.is_nil = b->is_nil ? b->is_nil[i] : 0;
  v.height = b->height[i];
  v.txhash = b->txhash + b->txhash_off[i]; v.txhash_len = b->txhash_len[i];
  v.ts_sec = b->ts_sec[i]; v.ts_nanos = b->ts_nanos[i];
  v.addr = b->addr + 20 * (size_t)i; v.addr_len = b->addr_len[i];
  v.sig = b->sig + 64 * (size_t)i; v.sig_len = b->sig_len[i];
  return v;
}

static void* soa_verify(void* p) {
  soa_job* j = (soa_job*)p;
  for (uint32_t i = j->begin; i < j->end; ++i) {
    orc_vote v = soa_vote(j->b, i);
    int64_t vi = v.is_nil ? -1 : val_by_addr(j->f, v.addr, v.addr_len);
    /* votes that cannot reach Verify keep 0xFF; the sequential pass never reads their code */
    j->code[i] = vi < 0 ? 0xFF : (uint8_t)orc_txvote_verify(&v, j->f->chain, j->f->chain_len, j->f->pubs + 32 * vi);
  }
  return 0;
}

void orc_flow_add_votes_soa(orc_flow* f, const orc_soa* b, int threads, uint8_t* status, int64_t* sum_after,
                            uint8_t* fired) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  uint8_t* code = (uint8_t*)malloc(b->n ? b->n : 1);
  soa_job jobs[256];
  pthread_t th[256];
  int started[256];
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (soa_job){f, b, code, (uint32_t)((uint64_t)b->n * t / threads), (uint32_t)((uint64_t)b->n * (t + 1) / threads)};
    /* a thread that cannot be created runs its range inline: never a range left unverified */
    started[t] = threads > 1 && pthread_create(&th[t], 0, soa_verify, &jobs[t]) == 0;
    if (!started[t]) soa_verify(&jobs[t]);
  }
  for (int t = 0; t < threads; ++t)
    if (started[t]) pthread_join(th[t], 0);
  for (uint32_t i = 0; i < b->n; ++i) {
    orc_vote v = soa_vote(b, i);
    status[i] = flow_add_one(f, &v, code[i] == 0xFF ? -1 : code[i], sum_after ? sum_after + i : 0, fired ? fired + i : 0);
  }
  free(code);
}

typedef struct {
  const orc_soa* b;
  const uint8_t* pubs;
  const uint8_t* chain; size_t chain_len;
  uint8_t* out;
  uint32_t begin, end;
} verify_job;

static void* soa_txvote_verify(void* p) {
  verify_job* j = (verify_job*)p;
  for (uint32_t i = j->begin; i < j->end; ++i) {
    orc_vote v = soa_vote(j->b, i);
    j->out[i] = v.is_nil ? ORC_ERR_NIL : (uint8_t)orc_txvote_verify(&v, j->chain, j->chain_len, j->pubs + 32 * (size_t)i);
  }
  return 0;
}

void orc_txvote_verify_soa(const orc_soa* b, const uint8_t* pubs32, const uint8_t* chain_id, size_t chain_len,
                           int threads, uint8_t* out) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  verify_job jobs[256];
  pthread_t th[256];
  int started[256];
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (verify_job){b, pubs32, chain_id, chain_len, out, (uint32_t)((uint64_t)b->n * t / threads),
                           (uint32_t)((uint64_t)b->n * (t + 1) / threads)};
    started[t] = threads > 1 && pthread_create(&th[t], 0, soa_txvote_verify, &jobs[t]) == 0;
    if (!started[t]) soa_txvote_verify(&jobs[t]);
  }
  for (int t = 0; t < threads; ++t)
    if (started[t]) pthread_join(th[t], 0);
}

int orc_flow_query(orc_flow* f, const uint8_t* txhash, uint32_t len, int64_t* sum, int32_t* maj23) {
  int64_t s = find_set(f, txhash, len);
  if (s < 0) return 0;
  if (sum) *sum = f->set_sum[s];
  if (maj23) *maj23 = f->set_maj23[s];
  return 1;
}
uint32_t orc_flow_get_votes(orc_flow* f, const uint8_t* txhash, uint32_t len, uint32_t* val_out, uint8_t* sig_out,
                            uint32_t cap) {
  int64_t s = find_set(f, txhash, len);
  if (s < 0) return 0;
  uint32_t k = 0;
  for (uint32_t v = 0; v < f->n_vals; ++v) {
    acc_sig* a = acc_find(f, ((uint64_t)(s + 1) << 32) | v);
    if (!a) continue;
    if (k < cap) {
      if (val_out) val_out[k] = v;
      if (sig_out) memcpy(sig_out + 64 * (size_t)k, a->sig, 64);
    }
    ++k;
  }
  return k;
}

uint32_t orc_flow_num_sets(orc_flow* f) { return f->n_sets; }
uint64_t orc_flow_num_verifies(orc_flow* f) { return f->n_verifies; }
