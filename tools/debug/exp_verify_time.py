"""Time K1 (verify) and K2 (tally) of the C2 workload against an alternative libtxvote build
(experiments: python tools/debug/exp_verify_time.py build_exp/libX.so ...).  Statuses are
not checked: experiment builds may compute wrong verdicts on purpose."""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "go-txflow_amd"))
import txflow_amd as T  # noqa: E402
from txflow_amd.workload import Workload, SEEDS  # noqa: E402

for arg in sys.argv[1:]:
    path, _, wv = arg.partition("@")         # lib.so@W[:V]: that validator-table window / lane_votes
    w, _, v = wv.partition(":")
    T._lib = None
    T.LIB_PATH = os.path.abspath(path)
    ctx = T.Context(max_batch=2 * 1_000_000, max_txs=10_064, max_validators=100, table_w=int(w) if w else None,
                    lane_votes=int(v) if v else 0)
    wl = Workload(ctx, 100, 10_000, SEEDS["c2"])
    ctx.stage(0, wl.batch)
    v, t = [], []
    for rep in range(6):
        ctx.reset_flow()
        ms = ctx.run_staged(0, timed=True)          # route, verify, tally, total (ms)
        ctx.fetch_staged(0, wl.n, ev_cap=wl.n_txs + 1)
        if rep:
            v.append(ms[1]); t.append(ms[2])
    print(f"{arg} (W={ctx.table_w}/{ctx.base_w}): verify {statistics.median(v):.3f} ms  tally {statistics.median(t):.3f} ms", flush=True)
    ctx.close()
