/*
 * pool.c — sequential restatement of TxVotePool.CheckTxWithInfo / Update / ReapMaxTxs / Flush
 * and mapTxCache (txvotepool/txvotepool.go).  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 *   :187-261  CheckTxWithInfo: full (Size() >= config.Size || size + TxsBytes > MaxTxsBytes,
 *             size = TxVote.Size() = 0 when amino rejects the timestamp),
 *             too large (size > MaxMsgBytes - 8, reactor.go:27,379), cache.Push false ->
 *             ErrTxInCache, else addTx (:265-270)
 *   :416-438  mapTxCache.Push: present -> MoveToBack, false; full -> remove Front; PushBack
 *   :457-459  nopTxCache (CacheSize == 0 in the reference config; here cache_size == ~0u)
 *   :329-359  Update: cache.Push(tx); txsMap hit -> removeTx(tx, e, false) (:275-284, which
 *             subtracts the committed tx's Size())
 *   :310-324  ReapMaxTxs: loop while len(txs) <= max (max + 1 entries), max < 0 -> all
 *   :467-469  txVoteKey = sha256.Sum256(Signature)
 * Every list is a plain doubly linked list of heap nodes; lookups walk a chained hash.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

typedef struct pnode {
  uint8_t key[32];
  uint32_t size;
  int mapped;                   /* txs: this element is txsMap[key] (a later push of the key overwrites) */
  struct pnode *prev, *next;    /* list order */
  struct pnode *hnext;          /* hash chain */
} pnode;

typedef struct {
  pnode *head, *tail;
  size_t len;
  pnode** bucket;
  size_t nb;
} plist;

struct orc_pool {
  uint32_t size, cache_size, max_msg_bytes;
  uint64_t max_txs_bytes;
  int cache_on;
  int wal;                      /* InitWAL was called (node/node.go:805-807, config WalEnabled) */
  int64_t height, txs_bytes;
  plist cache, txs;
};

static size_t bidx(const plist* l, const uint8_t* k) {
  uint64_t h = 0;
  for (int i = 0; i < 8; ++i) h = (h << 8) | k[i];
  return (size_t)(h % l->nb);
}
static void pl_init(plist* l) { memset(l, 0, sizeof *l); l->nb = 65521; l->bucket = (pnode**)calloc(l->nb, sizeof(pnode*)); }
static pnode* pl_find(const plist* l, const uint8_t* k) {   /* the mapped node with key k */
  for (pnode* n = l->bucket[bidx(l, k)]; n; n = n->hnext)
    if (n->mapped && !memcmp(n->key, k, 32)) return n;
  return 0;
}
/* chains stay short: the bucket array doubles when the list outgrows it (the gate's pool holds
 * ~10^8 entries) */
static void pl_rehash(plist* l) {
  const size_t nb = l->nb * 2 + 1;
  pnode** b = (pnode**)calloc(nb, sizeof(pnode*));
  free(l->bucket);
  l->bucket = b;
  l->nb = nb;
  for (pnode* n = l->head; n; n = n->next) {
    const size_t i = bidx(l, n->key);
    n->hnext = b[i];
    b[i] = n;
  }
}
static pnode* pl_push_back(plist* l, const uint8_t* k, uint32_t size) {
  if (l->len >= 2 * l->nb) pl_rehash(l);
  pnode* old = pl_find(l, k);
  if (old) old->mapped = 0;     /* txsMap.Store / cache map assignment replaces the entry */
  pnode* n = (pnode*)calloc(1, sizeof *n);
  n->mapped = 1;
  memcpy(n->key, k, 32);
  n->size = size;
  n->prev = l->tail;
  if (l->tail) l->tail->next = n; else l->head = n;
  l->tail = n;
  size_t b = bidx(l, k);
  n->hnext = l->bucket[b];
  l->bucket[b] = n;
  l->len++;
  return n;
}
static void pl_remove(plist* l, pnode* n) {
  if (n->prev) n->prev->next = n->next; else l->head = n->next;
  if (n->next) n->next->prev = n->prev; else l->tail = n->prev;
  pnode** pp = &l->bucket[bidx(l, n->key)];
  while (*pp != n) pp = &(*pp)->hnext;
  *pp = n->hnext;
  l->len--;
  free(n);
}
static void pl_clear(plist* l) {
  while (l->head) pl_remove(l, l->head);
}
static void pl_free(plist* l) { pl_clear(l); free(l->bucket); }

orc_pool* orc_pool_new(uint32_t size, uint32_t cache_size, uint64_t max_txs_bytes, uint32_t max_msg_bytes,
                       int64_t height, int wal) {
  orc_pool* p = (orc_pool*)calloc(1, sizeof *p);
  p->wal = wal;
  p->size = size; p->cache_size = cache_size; p->max_txs_bytes = max_txs_bytes; p->max_msg_bytes = max_msg_bytes;
  p->cache_on = cache_size != 0xFFFFFFFFu;
  p->height = height;
  pl_init(&p->cache);
  pl_init(&p->txs);
  return p;
}
void orc_pool_free(orc_pool* p) {
  if (!p) return;
  pl_free(&p->cache); pl_free(&p->txs);
  free(p);
}

static int cache_push(orc_pool* p, const uint8_t* k) {
  if (!p->cache_on) return 1;
  pnode* n = pl_find(&p->cache, k);
  if (n) {   /* MoveToBack: re-append (the cache never holds a key twice) */
    pl_remove(&p->cache, n);
    pl_push_back(&p->cache, k, 0);
    return 0;
  }
  if (p->cache.len >= p->cache_size && p->cache.head) pl_remove(&p->cache, p->cache.head);
  pl_push_back(&p->cache, k, 0);
  return 1;
}

static void vote_key(const orc_vote* v, uint8_t key[32]) { orc_sha256(v->sig, v->sig_len, key); }

/* CheckTxWithInfo (txvotepool.go:187-261) for a vote whose txVoteKey k and Size() sz are known */
static int pool_check_key(orc_pool* p, const uint8_t* k, int sz) {
  if ((int64_t)p->txs.len >= (int64_t)p->size || (int64_t)sz + p->txs_bytes > (int64_t)p->max_txs_bytes) return 1;
  if ((int64_t)sz > (int64_t)p->max_msg_bytes - 8) return 2;
  if (!cache_push(p, k)) return 3;
  if (sz == 0 && p->wal) return 4;                        /* WAL MustMarshalBinaryBare panics */
  pl_push_back(&p->txs, k, (uint32_t)sz);
  p->txs_bytes += sz;
  return 0;
}

int orc_pool_check(orc_pool* p, const orc_vote* v) {
  /* TxVote.Size() returns 0 when amino rejects the timestamp (types/tx_vote.go:144-150): such a
   * vote passes the caps with size 0, is cached and admitted; only the WAL write
   * (MustMarshalBinaryBare, :231-242, after the cache push) panics, when a WAL is configured */
  const int sz = orc_txvote_size(v->height, v->txhash_len, v->ts_sec, v->ts_nanos, v->addr_len, v->sig_len);
  uint8_t k[32];
  vote_key(v, k);
  return pool_check_key(p, k, sz);
}

/* orc_pool_check over n votes given as (txVoteKey, Size()) pairs, in arrival order */
void orc_pool_check_keys(orc_pool* p, const uint8_t* keys32, const uint32_t* sizes, uint32_t n, uint8_t* out) {
  for (uint32_t i = 0; i < n; ++i) out[i] = (uint8_t)pool_check_key(p, keys32 + (size_t)i * 32, (int)sizes[i]);
}

/* orc_pool_check over an SoA batch in arrival order (the gate's pool stage).  Signatures longer
 * than 64 bytes are read from sig_full + sig_full_off[i] (NULL: none in the batch). */
void orc_pool_check_soa(orc_pool* p, const orc_soa* b, const uint8_t* sig_full, const uint64_t* sig_full_off,
                        uint8_t* out) {
  for (uint32_t i = 0; i < b->n; ++i) {
    orc_vote v;
    v.is_nil = b->is_nil ? b->is_nil[i] : 0;
    v.height = b->height[i];
    v.txhash = b->txhash + b->txhash_off[i];
    v.txhash_len = b->txhash_len[i];
    v.ts_sec = b->ts_sec[i];
    v.ts_nanos = b->ts_nanos[i];
    v.addr = b->addr + (size_t)i * 20;
    v.addr_len = b->addr_len[i];
    v.sig = (b->sig_len[i] > 64 && sig_full) ? sig_full + sig_full_off[i] : b->sig + (size_t)i * 64;
    v.sig_len = b->sig_len[i];
    out[i] = (uint8_t)orc_pool_check(p, &v);
  }
}

void orc_pool_update(orc_pool* p, int64_t height, const orc_vote* votes, uint32_t n) {
  p->height = height;
  for (uint32_t i = 0; i < n; ++i) {
    uint8_t k[32];
    vote_key(&votes[i], k);
    (void)cache_push(p, k);
    pnode* e = pl_find(&p->txs, k);
    if (e) {
      pl_remove(&p->txs, e);
      p->txs_bytes -= orc_txvote_size(votes[i].height, votes[i].txhash_len, votes[i].ts_sec, votes[i].ts_nanos,
                                      votes[i].addr_len, votes[i].sig_len);
    }
  }
}

/* orc_pool_update over (txVoteKey, Size()) pairs (txvotepool.go:329-359 with the keys given) */
void orc_pool_update_keys(orc_pool* p, int64_t height, const uint8_t* keys32, const uint32_t* sizes, uint32_t n) {
  p->height = height;
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t* k = keys32 + (size_t)i * 32;
    (void)cache_push(p, k);
    pnode* e = pl_find(&p->txs, k);
    if (e) {
      pl_remove(&p->txs, e);
      p->txs_bytes -= sizes[i];
    }
  }
}

/* orc_pool_update over an SoA batch (the committed votes of a TxVoteSet, txflow/service.go:224-227) */
void orc_pool_update_soa(orc_pool* p, int64_t height, const orc_soa* b, const uint8_t* sig_full,
                         const uint64_t* sig_full_off) {
  p->height = height;
  for (uint32_t i = 0; i < b->n; ++i) {
    orc_vote v;
    memset(&v, 0, sizeof v);
    v.height = b->height[i];
    v.txhash_len = b->txhash_len[i];
    v.ts_sec = b->ts_sec[i];
    v.ts_nanos = b->ts_nanos[i];
    v.addr_len = b->addr_len[i];
    v.sig = (b->sig_len[i] > 64 && sig_full) ? sig_full + sig_full_off[i] : b->sig + (size_t)i * 64;
    v.sig_len = b->sig_len[i];
    orc_pool_update(p, height, &v, 1);
  }
}

uint64_t orc_pool_reap(orc_pool* p, int64_t max, uint8_t* keys_out, uint32_t* sizes_out, uint64_t cap) {
  if (max < 0) max = (int64_t)p->txs.len;
  uint64_t n = 0;
  for (pnode* e = p->txs.head; e && (int64_t)n <= max; e = e->next, ++n)
    if (n < cap) { memcpy(keys_out + 32 * n, e->key, 32); if (sizes_out) sizes_out[n] = e->size; }
  return n;
}

void orc_pool_flush(orc_pool* p) { pl_clear(&p->cache); pl_clear(&p->txs); p->txs_bytes = 0; }
int64_t orc_pool_size(orc_pool* p) { return (int64_t)p->txs.len; }
int64_t orc_pool_txs_bytes(orc_pool* p) { return p->txs_bytes; }
uint64_t orc_pool_cache_keys(orc_pool* p, uint8_t* keys_out, uint64_t cap) {
  uint64_t n = 0;
  for (pnode* e = p->cache.head; e; e = e->next, ++n)
    if (n < cap) memcpy(keys_out + 32 * n, e->key, 32);
  return n;
}
