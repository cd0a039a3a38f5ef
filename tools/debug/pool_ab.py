"""TxVotePool.CheckTx cost per 64k-vote batch, two-thread vs one-thread loop, alternated in one
process (C5 votes, 1000 validators): python tools/debug/pool_ab.py [rounds]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "go-txflow_amd"))
import txflow_amd as T  # noqa: E402
from txflow_amd.workload import StreamWorkload, SEEDS  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
ctx = T.Context(max_batch=65536, max_txs=2048 + 64, max_validators=1000)
wl = StreamWorkload(ctx, 1000, 1024, SEEDS["c5"], 65536)
pool = T.TxVotePool(ctx, size=wl.n + 1, cache_size=wl.n + 1, max_txs_bytes=1 << 40)
res = {"two": [], "one": []}
for r in range(rounds):
    for mode in ("two", "one"):
        if mode == "one":
            os.environ["TXV_POOL_ONE_THREAD"] = "1"
        else:
            os.environ.pop("TXV_POOL_ONE_THREAD", None)
        pool.flush()
        t = []
        for b in wl.batches:
            t0 = time.perf_counter()
            st = pool.check_batch(b)
            t.append((time.perf_counter() - t0) * 1e3)
            assert (st == T.POOL_OK).all()
        if r:
            res[mode].append(statistics.median(t))
for m, v in res.items():
    print(m, "median ms per 64k batch", round(statistics.median(v), 3), [round(x, 3) for x in v])
