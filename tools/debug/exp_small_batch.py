"""Verify time of small batches (C5's 64k votes, 1000 validators) for each K1b lane_votes mode,
against the in-tree build or an experiment build (TXV_LIB_PATH).  Statuses are checked (all
ADDED): python tools/debug/exp_small_batch.py [n_votes] [n_vals] [V,V,...]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "go-txflow_amd"))
import numpy as np  # noqa: E402
import txflow_amd as T  # noqa: E402
from txflow_amd.workload import Workload, SEEDS  # noqa: E402

n_votes = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
n_vals = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
lvs = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 4, 8]
for lv in lvs:
    ctx = T.Context(max_batch=n_votes, max_txs=n_votes // n_vals + 64, max_validators=n_vals, lane_votes=lv)
    wl = Workload(ctx, n_vals, n_votes // n_vals, SEEDS["c5"])
    ctx.stage(0, wl.batch)
    v, t, tot = [], [], []
    for rep in range(8):
        ctx.reset_flow()
        ms = ctx.run_staged(0, timed=True)
        st, _ = ctx.fetch_staged(0, wl.n, ev_cap=wl.n_txs + 1)
        assert int(np.count_nonzero((st & 0x7F) == T.ADDED)) == wl.n
        if rep:
            v.append(ms[1]); t.append(ms[2]); tot.append(ms[3])
    print(f"n={wl.n} vals={n_vals} W={ctx.table_w}/{ctx.base_w} V={lv}: verify {statistics.median(v):.3f} ms "
          f"tally {statistics.median(t):.3f} total {statistics.median(tot):.3f}", flush=True)
    ctx.close()
