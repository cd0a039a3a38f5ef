"""Run the library's VALU issue-rate probe (txv_k_valu_probe: 8 independent v_add_u32 or
v_mad_u64_u32 per loop iteration, 2048 x 256 threads x 16384 iterations per launch, 4 launches
each) so a PMC pass sees kernels of known instruction counts (the profiling run scripts)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "go-txflow_amd"))
import txflow_amd as T  # noqa: E402

ctx = T.Context(max_batch=1024, max_txs=64, max_validators=4)
add, mad = ctx.valu_probe()
print(f"v_add_u32 {add:.4e} lane-ops/s, v_mad_u64_u32 {mad:.4e} lane-ops/s")
ctx.close()
