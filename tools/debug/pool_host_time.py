"""TxVotePool.CheckTx batch path on the host (txv_pool_check_keys, no context: the pool's own
worker threads), C5-shaped: 64k-key batches with Appendix C's 5 % replays, CacheSize 10000.
python tools/debug/pool_host_time.py [batches] [rounds]; TXV_PROFILE_HOST=1 for the phases."""
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "go-txflow_amd"))
import txflow_amd as T  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 32
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
B = 65536
rng = np.random.default_rng(5)
uniq = rng.integers(0, 256, size=(nb * B, 32), dtype=np.uint8)
batches, hist = [], 0
for b in range(nb):
    keys = uniq[b * B:(b + 1) * B].copy()
    rep = np.flatnonzero(rng.random(B) < 0.05)
    for i in rep:                       # exact replays of an earlier vote: near or anywhere before
        tot = b * B + int(i)
        if tot == 0:
            continue
        j = tot - 1 - int(rng.integers(0, min(tot, 4096))) if rng.random() < 0.5 else int(rng.integers(0, tot))
        keys[i] = uniq[j] if j < b * B else keys[j - b * B]
    batches.append(keys)
sizes = np.full(B, 150, np.uint32)
res = []
pool = T.TxVotePool(None, size=nb * B + 1, cache_size=10000, max_txs_bytes=1 << 40)
for r in range(rounds + 1):             # as bench.py's C5: a warm-up pass first, flushed between
    t = []
    for keys in batches:
        t0 = time.perf_counter()
        pool.check_keys(keys, sizes)
        t.append((time.perf_counter() - t0) * 1e3)
    pool.flush()
    if r:
        res.append(statistics.median(t))
pool.close()
print(os.environ.get("TXV_LIB_PATH", "in-tree"), "p50 ms per 64k batch", [round(x, 3) for x in res])
