"""Per-phase timing of one C5 batch (1000 validators, 64k votes): stage (host pack + H2D),
run (verify + tally kernels, HIP events), fetch (D2H + events), pool check."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "go-txflow_amd"))
import numpy as np
import txflow_amd as T
from txflow_amd.workload import StreamWorkload, SEEDS

n_vals = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
n_txs = 1024 * 1000 // n_vals
ctx = T.Context(device=0, max_batch=batch, max_txs=n_txs + 64, max_validators=n_vals, max_accepted=1 << 26)
wl = StreamWorkload(ctx, n_vals, n_txs, SEEDS["c5"], batch)
pool = T.TxVotePool(ctx, size=1 << 24, cache_size=1 << 24, max_txs_bytes=1 << 40)
res = {"stage": [], "run_host": [], "verify_ms": [], "tally_ms": [], "fetch": [], "pool": [], "add_votes": []}
for rep in range(3):
    ctx.reset_flow()
    pool.flush()
    for b in wl.batches:
        t0 = time.perf_counter(); pool.check_batch(b); t1 = time.perf_counter()
        ctx.stage(0, b); t2 = time.perf_counter()
        ms = ctx.run_staged(0, timed=True); t3 = time.perf_counter()
        ctx.fetch_staged(0, b.n); t4 = time.perf_counter()
        if rep:
            res["pool"].append((t1 - t0) * 1e3); res["stage"].append((t2 - t1) * 1e3)
            res["run_host"].append((t3 - t2) * 1e3); res["verify_ms"].append(ms[0]); res["tally_ms"].append(ms[1])
            res["fetch"].append((t4 - t3) * 1e3)
ctx.reset_flow()
for b in wl.batches:
    t0 = time.perf_counter(); ctx.add_votes(b, ev_cap=b.n); res["add_votes"].append((time.perf_counter() - t0) * 1e3)
print({k: round(float(np.median(v)), 3) for k, v in res.items()}, "table_w", ctx.table_w, "base_w", ctx.base_w)
