#!/bin/bash
# C5 leg with the two-thread and the one-thread pool CheckTx loop (same box)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2_pool_ab
mkdir -p $O
for e in "TXV_NONE=0" "TXV_POOL_ONE_THREAD=1" "TXV_NONE=0"; do
  env $e timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c1 --no-wire --no-e2e --steps 5 > $O/c5.json 2> $O/c5.err || { echo C5FAIL; tail $O/c5.err; exit 2; }
  python3 -c "import json,sys;b=json.load(open('$O/c5.json'))['c5_streaming'];print(sys.argv[1], b['votes_per_s'], b['p50_pool_check_ms'], b['p50_commit_latency_ms'])" "$e"
done
