#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r2_pool5}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_pool.py tests/test_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "pool or c5" > $O/pool_tests.log 2>&1 || { echo POOLTESTFAIL; tail -40 $O/pool_tests.log; exit 1; }
tail -1 $O/pool_tests.log
TXV_PROFILE_HOST=1 timeout -k 10 120 python3 -u tools/debug/pool_time.py 4 > $O/pool_prof.log 2>&1 || { echo POOLFAIL; tail $O/pool_prof.log; exit 3; }
grep -v "^\[txv pool\]" $O/pool_prof.log | tail -2; grep "txv pool" $O/pool_prof.log | tail -2
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c1 --no-wire --no-e2e --steps 10 > $O/c5.json 2> $O/c5.err || { echo C5FAIL; tail $O/c5.err; exit 4; }
python3 -c "import json;b=json.load(open('$O/c5.json'));c=b['c5_streaming'];print(b['value'], c.get('votes_per_s_passes'), c['votes_per_s'], c['p50_pool_check_ms'], c['p50_commit_latency_ms'], c['p99_commit_latency_ms'])"
