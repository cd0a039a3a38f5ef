"""The device cache's batch algorithm (kernels_pool.hip pd_init .. pd_index, TXV_POOL_DEVICE_CACHE)
restated step by step in numpy and run on the CPU against the sequential oracle pool over
test_pool_batch.py's streams: the same sort by a 32-bit key slice, previous / next occurrence by
a scan inside each run, stack-distance decisions with the nested-pair count for far repeats, and
the new cache built from the surviving old entries and the batch's last pushes.  It checks the
formulation the kernels implement; tests/test_pool_device.py checks the kernels themselves on the
GPU.  Reference: txvotepool/txvotepool.go:187-261, :416-438."""
import zlib

import numpy as np
import pytest

import oracle as O
from test_pool_batch import CASES, _stream

OK, FULL, TOO_LARGE, IN_CACHE, ENCODING = range(5)


def device_batch(cache, C, keys, sizes, max_tx, wal):
    """one batch as the kernels decide it; cache = list of 32-byte keys front to back (L0 <= C);
    C = 0 for nopTxCache.  Returns (statuses, new cache)."""
    n = len(sizes)
    kb = [bytes(k) for k in keys]
    push = sizes.astype(np.int64) <= max_tx                                   # pd_init
    aidx = np.concatenate([[0], np.cumsum(push)[:-1]]).astype(np.int64)       # exclusive scan
    na = int(push.sum())
    h = np.where(push, keys[:, 8:12].copy().view("<u4").ravel(), 0xFFFFFFFF)
    order = np.argsort(h, kind="stable")                                      # the pair sort
    prev = np.full(n, -1, np.int64)
    crank = np.full(n, -1, np.int64)
    last = push.copy()
    L0 = len(cache) if C else 0
    where = {k: r for r, k in enumerate(cache)} if C else {}
    detached = np.zeros(max(C, 1), bool)
    for j in range(n):                                                        # pd_link
        i = order[j]
        if not push[i]:
            continue
        jj = j - 1
        found = False
        while jj >= 0 and h[order[jj]] == h[i]:
            k = order[jj]
            if push[k] and kb[k] == kb[i]:
                prev[i] = k
                last[k] = False
                found = True
                break
            jj -= 1
        if not found and C and L0:
            r = where.get(kb[i], -1)
            crank[i] = r
            if r >= 0:
                detached[r] = True
    evict = C != 0 and L0 + na > C                                            # pd_decide
    F = min(L0, na)
    dec = np.zeros(n, np.int64)
    pst = np.full(n, -1, np.int64)
    pend = np.full(n, -1, np.int64)
    for i in range(n):
        if not push[i]:
            continue
        e2 = 2 * (L0 + aidx[i])
        d = 1
        if prev[i] >= 0:
            pj = prev[i]
            d = 1 if not C else (2 if (not evict or aidx[i] - aidx[pj] - 1 < C) else 3)
            if evict:
                pst[i], pend[i] = 2 * (L0 + aidx[pj]), e2
        elif crank[i] >= 0:
            r = crank[i]
            front = evict and r < F
            d = 2 if (not front or L0 + aidx[i] - r - 1 < C) else 3
            if evict:
                pst[i], pend[i] = (2 * r if front else 2 * L0 - 1), e2
        dec[i] = d
    has = pst >= 0
    for i in np.flatnonzero(dec == 3):                                         # pd_far
        nested = int(np.count_nonzero(has & (pst > pst[i]) & (pend < pend[i])))
        window = (pend[i] - pst[i]) // 2 - 1
        dec[i] = 2 if window - nested < C else 1
    st = np.where(dec == 0, TOO_LARGE, np.where(dec == 2, IN_CACHE,            # pd_status
                  np.where((sizes == 0) & wal, ENCODING, OK))).astype(np.uint8)
    if not C:
        return st, cache
    surv = [r for r in range(L0) if not detached[r]]                           # pd_newcache
    lasts = [i for i in range(n) if last[i]]
    keepU = min(len(lasts), C)
    keep_old = min(len(surv), C - keepU)
    new = [cache[r] for r in surv[len(surv) - keep_old:]] + [kb[i] for i in lasts[len(lasts) - keepU:]]
    return st, new


NO_CUT = [c for c in CASES if c[2] >= (1 << 20) and c[3] >= (1 << 40) and c[9] * c[10] <= 30000]


@pytest.mark.parametrize("case", NO_CUT, ids=[c[0] for c in NO_CUT])
def test_device_formulation_matches_oracle(case):
    name, cache_size, size, max_bytes, wal, replay, far, big, zero, nb, batch = case
    O.build()
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    opool = O.Pool(size=size, cache_size=cache_size, max_txs_bytes=max_bytes, wal=wal)
    C = 0 if cache_size == 0xFFFFFFFF else cache_size
    max_tx = (1 << 20) - 8
    cache = []
    for b, (keys, sizes) in enumerate(_stream(rng, nb, batch, replay, far, big, zero)):
        st, cache = device_batch(cache, C, keys, sizes, max_tx, wal)
        ost = opool.check_keys(keys, sizes)
        assert np.array_equal(st, ost), f"{name} batch {b}: {int(np.count_nonzero(st != ost))} mismatches"
        if C:
            ock = opool.cache_keys()
            assert [bytes(k) for k in ock] == cache, f"{name} batch {b}: LRU differs"


def test_device_formulation_tiny_caches():
    """caches of 1..5 entries with dense repeats: every far-repeat corner of the stack distance"""
    O.build()
    rng = np.random.default_rng(3)
    for C in (1, 2, 3, 5):
        opool = O.Pool(size=1 << 20, cache_size=C, max_txs_bytes=1 << 40)
        cache = []
        for b in range(6):
            keys = rng.integers(0, 4, size=(300, 32), dtype=np.uint8)          # few distinct keys
            keys[:, 1:] = keys[:, :1]
            sizes = np.full(300, 150, np.uint32)
            st, cache = device_batch(cache, C, keys, sizes, (1 << 20) - 8, False)
            ost = opool.check_keys(keys, sizes)
            assert np.array_equal(st, ost), (C, b)
            assert [bytes(k) for k in opool.cache_keys()] == cache, (C, b)
