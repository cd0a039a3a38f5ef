"""Times txv_k_decode_msgs on n C2-shaped TxVoteMessages (random signatures: decode only).
TXV_LIB_PATH selects an experiment build.  Usage: python tools/debug/wire_time.py [n] [reps]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "go-txflow_amd"))
import numpy as np
import txflow_amd as T

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rng = np.random.default_rng(1)
hexd = np.frombuffer(b"0123456789ABCDEF", np.uint8)
arena = hexd[rng.integers(0, 16, size=64 * n)]
b = T.VoteBatch(n, height=np.ones(n, np.int64), txhash_arena=arena, txhash_off=np.arange(n, dtype=np.uint32) * 64,
                txhash_len=np.full(n, 64, np.uint32), ts_sec=np.full(n, 1_700_000_000, np.int64),
                ts_nanos=(np.arange(n) + 1).astype(np.int32), addr=rng.integers(0, 256, size=20 * n, dtype=np.uint8),
                addr_len=np.full(n, 20, np.uint32), sig=rng.integers(0, 256, size=64 * n, dtype=np.uint8),
                sig_len=np.full(n, 64, np.uint32))
wb = T.encode_msgs(b)
ctx = T.Context(max_batch=1 << 16, max_txs=1 << 12, max_validators=16, table_w=4)
ctx.decode_stage(wb)
ctx.decode_run(reps=3)
best = min(ctx.decode_run(reps=reps) for _ in range(3))
d = ctx.decode_fetch(wb)
ok = bool((d.status[:n] == 0).all() and (d.sig[:n].reshape(-1) == b.sig).all() and (d.height[:n] == 1).all())
alg = wb.nbytes + n * (12 + 160)
print(f"{os.environ.get('TXV_LIB_PATH', 'default')}: n={n} {wb.nbytes / n:.1f} B/msg  kernel {best:.4f} ms  "
      f"{n / best / 1e6:.2f} G msgs/s  {alg / best / 1e6:.0f} GB/s  ok={ok}", flush=True)
