#!/usr/bin/env python3
"""C4 bit-exact gate (BASELINE.json config 4): stream N adversarial TxVotes
through libtxvote.so on cuda:0 and through the sequential CPU oracle; every per-vote status,
commit-fire bit, commit event, direct-Verify verdict (slice) and per-tx (sum, maj23) must agree.  By default every
batch first passes TxVotePool.CheckTx (device txv_pool_check vs the oracle pool, outcomes compared
per vote; replays still cached -> ErrTxInCache) and only the admitted votes reach TxFlow.

    python tools/gate/c4_gate.py --votes 100000000 --out gpurun_out/c4/gate.json

Prints one progress line per batch; writes the final stats as JSON."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "go-txflow_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--votes", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--batches-per-epoch", type=int, default=4)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default="")
    ap.add_argument("--lane-votes", type=int, default=0, choices=(0, 1, 2, 4, 8))
    ap.add_argument("--no-pool", action="store_true", help="feed txv_add_votes directly (no TxVotePool stage)")
    ap.add_argument("--pool-cache", type=int, default=1 << 20, help="TxVotePool CacheSize (LRU entries)")
    ap.add_argument("--pool-device", action="store_true", help="the pool's cache in HBM (TXV_POOL_DEVICE_CACHE)")
    ap.add_argument("--table-w", type=int, default=0, choices=(0, 12, 16, 18, 20, 21),
                    help="validator table window (0 = the library's automatic one; 21 = bench.py's C2 context)")
    ap.add_argument("--base-w", type=int, default=0, choices=(0, 24, 26),
                    help="base-point table window (0 = automatic; 26 = bench.py's C2 context)")
    args = ap.parse_args()
    import oracle
    oracle.build()
    import txflow_amd as T
    import adversarial as A
    ctx = T.Context(device=0, max_batch=args.batch + args.batch // 4, max_txs=1 << 17, max_validators=256,
                    lane_votes=args.lane_votes, table_w=args.table_w or None, base_w=args.base_w)
    t0 = time.time()
    st = A.run_gate(ctx, args.votes, batch=args.batch, batches_per_epoch=args.batches_per_epoch,
                    threads=args.threads, log=lambda s: print(s, flush=True), pool_stage=not args.no_pool,
                    pool_cache=args.pool_cache, pool_device=args.pool_device)
    import subprocess
    try:
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
    except Exception:
        head = ""
    st.update(head=head or os.environ.get("TXV_HEAD", ""), device=ctx.device_name(), table_window=ctx.table_w, base_window=ctx.base_w,
              validators=len(A.crafted_keys()) + A.N_HONEST, wall_s=round(time.time() - t0, 1),
              oracle_threads=args.threads, batch=args.batch, batches_per_epoch=args.batches_per_epoch)
    print(json.dumps(st), flush=True)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(st, f, indent=1)
    ctx.close()
    sys.exit(0 if st["mismatches"] == 0 else 1)


if __name__ == "__main__":
    main()
