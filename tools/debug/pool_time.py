"""TxVotePool.CheckTx cost per 64k-vote batch (C5 votes, 1000 validators) for the in-tree build
or TXV_LIB_PATH: python tools/debug/pool_time.py [rounds]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "go-txflow_amd"))
import txflow_amd as T  # noqa: E402
from txflow_amd.workload import StreamWorkload, SEEDS  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
ctx = T.Context(max_batch=65536, max_txs=2048 + 64, max_validators=1000)
wl = StreamWorkload(ctx, 1000, 2048, SEEDS["c5"], 65536)
pool = T.TxVotePool(ctx, size=wl.n + 1, cache_size=wl.n + 1, max_txs_bytes=1 << 40)
res = []
for r in range(rounds):
    pool.flush()
    t = []
    for b in wl.batches:
        t0 = time.perf_counter()
        st = pool.check_batch(b)
        t.append((time.perf_counter() - t0) * 1e3)
        assert (st == T.POOL_OK).all()
    if r:
        res.append(statistics.median(t))
print(os.environ.get("TXV_LIB_PATH", "in-tree"), "median ms per 64k batch", round(statistics.median(res), 3),
      [round(x, 3) for x in res])
