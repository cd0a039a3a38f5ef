import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "go-txflow_amd"))
import numpy as np
import txflow_amd as T
from txflow_amd.workload import Workload
ctx = T.Context(max_batch=1 << 16, max_txs=200)
wl = Workload(ctx, 10, 100, 5)
st, ev = ctx.add_votes(wl.batch)
print("add_votes: events", len(ev), "fired", int(np.count_nonzero(st & 0x80)))
ctx.reset_tally()
ctx.stage(0, wl.batch)
ctx.run_staged(0, timed=True)
st, ev = ctx.fetch_staged(0, wl.n, ev_cap=wl.n_txs + 1)
print("staged: events", len(ev), "fired", int(np.count_nonzero(st & 0x80)))
ctx.reset_tally()
ctx.run_staged(0, timed=True)
st, ev = ctx.fetch_staged(0, wl.n, ev_cap=wl.n_txs + 1)
print("staged after reset: events", len(ev), "fired", int(np.count_nonzero(st & 0x80)))
