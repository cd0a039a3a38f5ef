#!/bin/bash
# r3_c5b.sh TAG: pool GPU tests, then bench.py's C5 legs with the worker pool spinning before it
# sleeps (TXV_HOST_SPIN_US=200, default) and sleeping at once (0); host pool phases in *.err
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_c5b}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_pool.py tests/test_wire.py \
  > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for spin in 200 0; do
    TXV_HOST_SPIN_US=$spin TXV_PROFILE_HOST=1 timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-c1 --no-wire --no-e2e --no-cpu-baseline \
      > $O/bench_s${spin}_$rep.json 2> $O/bench_s${spin}_$rep.err || { echo BENCHFAIL; tail $O/bench_s${spin}_$rep.err; exit 3; }
    python3 -c "
import json,sys;b=json.load(open('$O/bench_s${spin}_$rep.json'));c=b['c5_streaming'];w=b['c5_wire']
print('spin $spin rep $rep', b['value'], b['ms_per_step'], 'c5', c['votes_per_s'], c['p50_pool_check_ms'], c['p50_commit_latency_ms'], c['correct'], 'wire', w.get('votes_per_s'), w.get('p50_pool_check_ms'))"
  done
done
