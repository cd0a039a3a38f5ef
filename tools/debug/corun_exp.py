#!/usr/bin/env python3
"""Co-running attribution (experiment build with -DTXV_EXP_SKIP, TXV_LIB_PATH pointing at it):
the C2 pipelined step with the flow kernels of TXV_EXP_SKIP's mask left out; prints the
in-pipeline and standalone stage times (slot_kernel_ms: prep, verify = K1a + K1b, tally).
Only masks that leave no kernel reading unwritten indices are safe: 4, 8, 16, 32 and their sums,
and 255 (no flow kernel at all: the verify chain alone, pipelined)."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "go-txflow_amd"))
import txflow_amd as T  # noqa: E402
from txflow_amd.pipeline import PipelinedSteps  # noqa: E402
from txflow_amd.workload import Workload, SEEDS  # noqa: E402

mask = int(os.environ.get("TXV_EXP_SKIP", "0"), 0)
lib = os.path.basename(os.path.dirname(os.environ.get("TXV_LIB_PATH", "in-tree/x")))
assert mask & ~60 == 0 or mask == 255, "unsafe mask"
ctx = T.Context(max_batch=1_000_000, max_txs=10_064, max_validators=100)
wl = Workload(ctx, 100, 10_000, SEEDS["c2"])
ps = PipelinedSteps(ctx, [wl.batch], depth=3, fresh_flow=True, ev_cap=wl.n_txs + 1)
ms = []
ps.run(3)
ctx.sync()
t0 = time.perf_counter()
ps.run(30, lambda k, st, ev: ms.append(ctx.slot_kernel_ms(k % 3)))
ctx.sync()
el = (time.perf_counter() - t0) / 30 * 1e3
solo = []
for _ in range(3):
    ctx.reset_flow()
    solo.append(ctx.run_staged(0, timed=True))
    ps.finish(0)
print(json.dumps({"lib": lib, "mask": mask, "ms_per_step": round(el, 3),
                  "pipe": [round(statistics.median(x[j] for x in ms), 3) for j in range(3)],
                  "solo": [round(statistics.median(x[j] for x in solo), 3) for j in range(4)]}), flush=True)
ctx.close()
