"""TxVotePool ingest (txvotepool/txvotepool.go): the oracle restatement (oracle/pool.c) against
the reference's own pool tests restated on the code semantics (several of them were written for
Tendermint's CListMempool and contradict this code, e.g. TestMempoolTxsBytes expects TxsBytes 1
for a vote whose TxVote.Size() is ~100), and libtxvote.so (txv_sig_keys on the GPU + the host
LRU / pool list) against the oracle on random streams.

Reference tests restated (Fantom-foundation/go-txflow):
  TestCacheRemove              txvotepool/cache_test.go:16-34   (pushes grow the cache list and map)
  TestCacheAfterUpdate         txvotepool/cache_test.go:36-99   (Update pushes to the cache; order)
  TestMempoolUpdateAddsTxsToCache txvotepool/txvotepool_test.go:110-120
  TestSerialReap               txvotepool/txvotepool_test.go:166-251 (dupes cached, Update, redeliver)
  TestMempoolMaxMsgSize        txvotepool/txvotepool_test.go:305-355 (ErrTxTooLarge boundary)
  TestMempoolTxsBytes          txvotepool/txvotepool_test.go:357-413 (TxsBytes, Update, Flush, full)
"""
import hashlib
import random

import numpy as np
import pytest

OK, FULL, TOO_LARGE, IN_CACHE, ENCODING = range(5)
ZERO_TIME = -62135596800          # Go time.Time{} in Unix seconds


def vote(sig, txhash=b"AB" * 32, height=1, ts=(1_700_000_000, 5), addr=b"\x01" * 20):
    return dict(height=height, txhash=txhash, ts_sec=ts[0], ts_nanos=ts[1], addr=addr, sig=sig)


def key(sig):
    return hashlib.sha256(sig).digest()


# ------------------------------------------------------------------ oracle vs reference tests
def test_cache_push_grows_list_and_map(oracle_lib):
    p = oracle_lib.Pool(cache_size=100)
    for i in range(10):
        assert p.check([vote(bytes([i]))])[0] == OK
        assert len(p.cache_keys()) == i + 1
    assert [bytes(k) for k in p.cache_keys()] == [key(bytes([i])) for i in range(10)]


def test_cache_after_update(oracle_lib):
    """cache_test.go:36-99 on the code: Update pushes committed keys to the back of the LRU
    (existing keys move), re-adding after Update is ErrTxInCache and makes no duplicate."""
    p = oracle_lib.Pool()
    assert list(p.check([vote(b"\x00"), vote(b"\x01")])) == [OK, OK]
    p.update(1, [vote(b"\x01")])
    assert [bytes(k) for k in p.cache_keys()] == [key(b"\x00"), key(b"\x01")]
    p.update(1, [vote(b"\x02")])
    assert [bytes(k) for k in p.cache_keys()] == [key(b"\x00"), key(b"\x01"), key(b"\x02")]
    p.update(1, [vote(b"\x00")])                       # moves 0 to the back
    assert [bytes(k) for k in p.cache_keys()] == [key(b"\x01"), key(b"\x02"), key(b"\x00")]
    assert list(p.check([vote(b"\x01")])) == [IN_CACHE]
    assert len(p.cache_keys()) == 3 and p.size() == 0   # both pooled votes were committed
    keys, _ = p.reap()
    assert len(keys) == 0


def test_update_adds_txs_to_cache(oracle_lib):
    """txvotepool_test.go:110-120: Update(0, [TxVote{}]) then CheckTx(TxVote{}) -> ErrTxInCache"""
    p = oracle_lib.Pool()
    empty = dict(height=0, txhash=b"", ts_sec=ZERO_TIME, ts_nanos=0, addr=b"", sig=b"")
    p.update(0, [empty])
    assert list(p.check([empty])) == [IN_CACHE]


def test_serial_reap(oracle_lib):
    """txvotepool_test.go:166-251 (code semantics): every first CheckTx of a new signature is
    added, every repeat is ErrTxInCache; after Update(0..500) those votes leave the pool but stay
    cached; redelivering 900..1100 adds only the 100 new ones."""
    p = oracle_lib.Pool()
    sig = lambda i: i.to_bytes(8, "big")
    st = p.check([vote(sig(i)) for i in range(100)] + [vote(sig(i)) for i in range(100)])
    assert list(st[:100]) == [OK] * 100 and list(st[100:]) == [IN_CACHE] * 100
    st = p.check([vote(sig(i)) for i in range(1000)])
    assert list(st[:100]) == [IN_CACHE] * 100 and list(st[100:]) == [OK] * 900
    assert p.size() == 1000
    p.update(3, [vote(sig(i)) for i in range(500)])
    assert p.size() == 500
    st = p.check([vote(sig(i)) for i in range(900, 1100)])
    assert list(st[:100]) == [IN_CACHE] * 100 and list(st[100:]) == [OK] * 100
    keys, _ = p.reap()
    assert [bytes(k) for k in keys] == [key(sig(i)) for i in list(range(500, 1000)) + list(range(1000, 1100))]
    keys, _ = p.reap(9)
    assert len(keys) == 10                      # ReapMaxTxs loop condition len(txs) <= max


def test_max_msg_size(oracle_lib):
    """txvotepool_test.go:305-355: ErrTxTooLarge exactly when Size() > MaxMsgBytes - 8."""
    max_msg = 400
    p = oracle_lib.Pool(max_msg_bytes=max_msg)
    base = oracle_lib.txvote_size(1, 64, 1_700_000_000, 5, 20, 0)
    for L in range(max_msg - 8 - base - 6, max_msg - 8 - base + 6):
        if L < 0:
            continue
        sg = bytes([L % 256]) * L + L.to_bytes(4, "little")
        sz = oracle_lib.txvote_size(1, 64, 1_700_000_000, 5, 20, len(sg))
        st = p.check([vote(sg)])[0]
        assert st == (TOO_LARGE if sz > max_msg - 8 else OK), (L, sz)


def test_txs_bytes(oracle_lib):
    """txvotepool_test.go:357-413 (code semantics): TxsBytes = sum of Size(); Update removes;
    Flush zeroes; ErrMempoolIsFull once MaxTxsBytes would be exceeded."""
    v1 = vote(b"\x01")
    sz = oracle_lib.txvote_size(1, 64, 1_700_000_000, 5, 20, 1)
    p = oracle_lib.Pool(max_txs_bytes=2 * sz + sz // 2)
    assert p.txs_bytes() == 0
    assert list(p.check([v1])) == [OK] and p.txs_bytes() == sz
    p.update(1, [v1])
    assert p.txs_bytes() == 0
    assert list(p.check([vote(b"\x02")])) == [OK] and p.txs_bytes() == sz
    p.flush()
    assert p.txs_bytes() == 0 and p.size() == 0
    assert list(p.check([vote(b"\x04"), vote(b"\x05"), vote(b"\x06")])) == [OK, OK, FULL]


def test_size_zero_vote_is_admitted(oracle_lib):
    """TxVote.Size() returns 0 when amino rejects the timestamp (types/tx_vote.go:144-150), it
    does not panic: CheckTxWithInfo (txvotepool.go:192-261) then passes the caps, caches
    SHA-256(sig) and admits the vote with 0 bytes.  Only a configured WAL panics (its
    MustMarshalBinaryBare, :231-242), after the cache push -- so a repeat is ErrTxInCache."""
    bad_ts = (10 ** 13, 1)                              # year > 9999: amino time error
    assert oracle_lib.txvote_size(1, 64, bad_ts[0], bad_ts[1], 20, 1) == 0
    p = oracle_lib.Pool(max_txs_bytes=100)
    st = p.check([vote(b"\x07", ts=bad_ts), vote(b"\x07", ts=bad_ts), vote(b"\x08")])
    assert list(st) == [OK, IN_CACHE, FULL]             # vote 3 (~100 B) exceeds MaxTxsBytes
    assert p.size() == 1 and p.txs_bytes() == 0
    keys, sizes = p.reap()
    assert [bytes(k) for k in keys] == [key(b"\x07")] and list(sizes) == [0]
    w = oracle_lib.Pool(wal=True)
    st = w.check([vote(b"\x07", ts=bad_ts), vote(b"\x07", ts=bad_ts), vote(b"\x08")])
    assert list(st) == [ENCODING, IN_CACHE, OK]
    assert w.size() == 1 and [bytes(k) for k in w.cache_keys()] == [key(b"\x07"), key(b"\x08")]


# ------------------------------------------------------------------ GPU parity
def _random_stream(rnd, n, n_sigs, long_frac=0.02):
    votes = []
    pool_of = [bytes(rnd.getrandbits(8) for _ in range(rnd.choice([0, 1, 55, 56, 63, 64, 64, 64, 64, 65, 119, 120, 200])))
               for _ in range(n_sigs)]
    for i in range(n):
        s = rnd.choice(pool_of)
        votes.append(vote(s, txhash=bytes(rnd.choice(b"0123456789ABCDEF") for _ in range(rnd.choice([0, 64, 64, 300]))),
                          height=rnd.choice([0, 1, 7]),
                          ts=rnd.choice([(1_700_000_000, i % 1000 + 1), (ZERO_TIME, 0), (0, 0), (10 ** 13, 1)]),
                          addr=bytes(rnd.getrandbits(8) for _ in range(rnd.choice([0, 20, 20, 33])))))
    return votes


def _batch(T, votes):
    vs = [T.TxVote(Height=v["height"], TxHash=v["txhash"], Timestamp=(v["ts_sec"], v["ts_nanos"]),
                   ValidatorAddress=v["addr"], Signature=v["sig"]) for v in votes]
    b = T.VoteBatch.from_votes(vs)
    long_sigs = {i: v["sig"] for i, v in enumerate(votes) if len(v["sig"]) > 64}
    return b, long_sigs


@pytest.mark.gpu
def test_sig_keys_match_sha256(gpu_ctx):
    import txflow_amd as T
    rnd = random.Random(5)
    votes = [vote(bytes(rnd.getrandbits(8) for _ in range(L))) for L in list(range(0, 131)) * 3]
    b, long_sigs = _batch(T, votes)
    keys = gpu_ctx.sig_keys(b, long_sigs)
    for v, k in zip(votes, keys):
        assert bytes(k) == key(v["sig"]), len(v["sig"])


@pytest.mark.gpu
@pytest.mark.parametrize("device_cache", [False, True], ids=["host-cache", "device-cache"])
@pytest.mark.parametrize("cfg", [dict(size=700, cache_size=300), dict(size=2000, cache_size=0xFFFFFFFF),
                                 dict(size=100000, cache_size=50, max_txs_bytes=60000, max_msg_bytes=300),
                                 dict(size=2000, cache_size=300, wal=True), dict(size=100000, cache_size=300, wal=True)],
                         ids=["small-cache", "no-cache", "byte-limits", "wal", "wal-roomy"])
def test_pool_matches_oracle(gpu_ctx, oracle_lib, cfg, device_cache):
    """Random streams with repeated / empty / long (> 64 B) signatures, zero and out-of-range
    timestamps, long TxHashes: per-vote CheckTx results, Update, ReapMaxTxs order + sizes,
    TxsBytes, Size and the LRU order equal the oracle's, across several batches.  device-cache:
    TXV_POOL_DEVICE_CACHE (batches whose caps cannot bind and without long signatures are decided
    on the GPU, the others on the host, the cache list moving between the two copies)."""
    import txflow_amd as T
    rnd = random.Random(hash(tuple(sorted(cfg.items()))) & 0xFFFF)
    pool = T.TxVotePool(gpu_ctx, **cfg, device_cache=device_cache)
    ref = oracle_lib.Pool(**{k: v for k, v in cfg.items()})
    try:
        seen = set()
        for rnd_batch in range(4):
            votes = _random_stream(rnd, 1500, 900)
            b, long_sigs = _batch(T, votes)
            st = pool.check_batch(b, long_sigs)
            exp = ref.check(votes)
            assert np.array_equal(st, exp), np.nonzero(st != exp)[0][:10]
            committed = rnd.sample(votes, 200)
            cb, clong = _batch(T, committed)
            pool.update(rnd_batch + 1, cb, clong)
            ref.update(rnd_batch + 1, committed)
            assert pool.Size() == ref.size() and pool.TxsBytes() == ref.txs_bytes()
            for m in (-1, 0, 17):
                gk, gs = pool.reap(m)
                ok, os_ = ref.reap(m)
                assert np.array_equal(gk, ok) and np.array_equal(gs, os_)
            assert np.array_equal(pool.cache_keys(), ref.cache_keys())
            seen |= set(int(x) for x in np.unique(exp))
        want = {OK} | ({FULL} if cfg["size"] < 6000 else set()) | ({IN_CACHE} if cfg["cache_size"] != 0xFFFFFFFF else set()) | \
            ({TOO_LARGE} if "max_msg_bytes" in cfg else set()) | ({ENCODING} if cfg.get("wal") else set())
        assert cfg.get("wal") or ENCODING not in seen      # without a WAL Size() == 0 votes are admitted
        assert seen >= want, (seen, want)
        pool.flush(); ref.flush()
        assert pool.Size() == 0 and pool.TxsBytes() == 0 and len(pool.cache_keys()) == 0
    finally:
        pool.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["check", "prepare", "device", "device-prepare"])
def test_pool_batch_admit_matches_oracle(oracle_lib, mode):
    """Batches of >= 4096 votes take txv_pool_check's batch path (pool.cpp batch_check: LRU
    decisions by stack distance, state written once): all-new keys, a key already cached, a key
    repeated inside the batch, a batch that evicts from the cache.  Every outcome, Size, TxsBytes,
    ReapMaxTxs order and the LRU order equal the oracle's, including node reuse after Update.
    mode "prepare": the same CheckTx in its two halves, txv_pool_prepare (keys on the GPU + Size)
    then txv_pool_check_keys (the order-dependent admission), as bench.py's C5 leg pipelines them.
    mode "device" / "device-prepare": the same two with TXV_POOL_DEVICE_CACHE (decided on the GPU)."""
    import txflow_amd as T
    rnd = random.Random(77)
    ctx = T.Context(max_batch=1 << 14, max_txs=1024, max_validators=8)
    cfg = dict(size=100000, cache_size=30000)
    pool = T.TxVotePool(ctx, **cfg, device_cache=mode.startswith("device"))
    ref = oracle_lib.Pool(**cfg)

    def fresh(n):
        return [vote(bytes(rnd.getrandbits(8) for _ in range(64)), ts=(1_700_000_000, 1 + i)) for i in range(n)]

    def check(votes):
        b, long_sigs = _batch(T, votes)
        if mode in ("check", "device"):
            st = pool.check_batch(b, long_sigs)
        else:
            keys, sizes = pool.prepare(b, long_sigs)
            assert keys.shape == (b.n, 32) and sizes.shape == (b.n,)
            st = pool.check_keys(keys, sizes)
        exp = ref.check(votes)
        assert np.array_equal(st, exp), np.nonzero(st != exp)[0][:10]
        assert pool.Size() == ref.size() and pool.TxsBytes() == ref.txs_bytes()
        for m in (-1, 0, 33):
            gk, gs = pool.reap(m)
            ok, os_ = ref.reap(m)
            assert np.array_equal(gk, ok) and np.array_equal(gs, os_)
        assert np.array_equal(pool.cache_keys(), ref.cache_keys())
        return st

    try:
        first = fresh(6000)
        assert (check(first) == OK).all()                       # batch-admit
        committed = rnd.sample(first, 1500)                      # Update: pool nodes to the free list
        cb, clong = _batch(T, committed)
        pool.update(1, cb, clong)
        ref.update(1, committed)
        assert (check(fresh(5000)) == OK).all()                  # batch-admit reusing freed nodes
        again = fresh(5000)
        again[2500] = dict(first[10])                            # an already cached key
        st = check(again)
        assert st[2500] == IN_CACHE and (np.delete(st, 2500) == OK).all()
        dup = fresh(5000)
        dup[4000] = dict(dup[7])                                 # a key repeated inside the batch
        st = check(dup)
        assert st[4000] == IN_CACHE and (np.delete(st, 4000) == OK).all()
        st = check(fresh(12000))                                 # the cache (30000) would evict
        assert (st == OK).all() and len(pool.cache_keys()) == 30000
    finally:
        pool.close()
        ctx.close()


@pytest.mark.gpu
def test_pool_batch_admit_no_cache_and_caps(oracle_lib):
    """The batch path without a cache (a key repeated inside the batch is admitted twice,
    txsMap.Store keeping the later node), a batch the Size cap cuts (ErrMempoolIsFull from the
    cut on) and one the byte cap could cut (sequential loop): outcomes, Size, TxsBytes and
    ReapMaxTxs equal the oracle's."""
    import txflow_amd as T
    rnd = random.Random(78)
    ctx = T.Context(max_batch=1 << 14, max_txs=1024, max_validators=8)

    def fresh(n):
        return [vote(bytes(rnd.getrandbits(8) for _ in range(64)), ts=(1_700_000_000, 1 + i)) for i in range(n)]

    for cfg, dev in [(c, d) for d in (False, True) for c in (
            dict(size=20000, cache_size=0xFFFFFFFF), dict(size=9000, cache_size=50000),
            dict(size=100000, cache_size=50000, max_txs_bytes=1_000_000))]:
        pool = T.TxVotePool(ctx, **cfg, device_cache=dev)
        ref = oracle_lib.Pool(**cfg)
        try:
            for votes in (fresh(6000), fresh(6000), fresh(5000)):
                if cfg["cache_size"] == 0xFFFFFFFF:
                    votes[3000] = dict(votes[11])
                b, long_sigs = _batch(T, votes)
                st = pool.check_batch(b, long_sigs)
                exp = ref.check(votes)
                assert np.array_equal(st, exp), (cfg, dev, np.nonzero(st != exp)[0][:10])
                assert pool.Size() == ref.size() and pool.TxsBytes() == ref.txs_bytes()
                gk, gs = pool.reap(-1)
                ok, os_ = ref.reap(-1)
                assert np.array_equal(gk, ok) and np.array_equal(gs, os_)
            assert pool.Size() < 17000 or cfg["cache_size"] == 0xFFFFFFFF   # the caps were reached
        finally:
            pool.close()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("device_cache", [False, True], ids=["host-cache", "device-cache"])
def test_pool_replay_stream_bounded_cache(oracle_lib, device_cache):
    """Appendix C's exact replays (near: within the last 4096 votes; far: any earlier vote) in
    32k-vote batches through txv_pool_check with tendermint's default CacheSize (10000): replays
    still cached -> ErrTxInCache, replays of evicted keys admitted again (second pool element);
    every outcome, the LRU order and the pool order equal the oracle's after each batch."""
    import txflow_amd as T
    rnd = random.Random(79)
    ctx = T.Context(max_batch=1 << 16, max_txs=1024, max_validators=8)
    pool = T.TxVotePool(ctx, size=1 << 20, cache_size=0, device_cache=device_cache)
    ref = oracle_lib.Pool(size=1 << 20, cache_size=10000)
    hist = []
    try:
        for b in range(4):
            votes = []
            for i in range(32768):
                if hist and rnd.random() < 0.05:
                    j = rnd.randrange(len(hist)) if rnd.random() < 0.5 else max(0, len(hist) - 1 - rnd.randrange(4096))
                    votes.append(dict(hist[j]))
                else:
                    votes.append(vote(rnd.randbytes(64), ts=(1_700_000_000, 1 + len(hist))))
                hist.append(votes[-1])
            bt, long_sigs = _batch(T, votes)
            st = pool.check_batch(bt, long_sigs)
            exp = ref.check(votes)
            assert np.array_equal(st, exp), (b, np.nonzero(st != exp)[0][:10])
            assert pool.Size() == ref.size() and pool.TxsBytes() == ref.txs_bytes()
            assert np.array_equal(pool.cache_keys(), ref.cache_keys())
            gk, gs = pool.reap(-1)
            ok, os_ = ref.reap(-1)
            assert np.array_equal(gk, ok) and np.array_equal(gs, os_)
            if b:
                assert (st == IN_CACHE).any() and (st == OK).sum() > 30000
    finally:
        pool.close()
        ctx.close()
