#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2_pool4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_pool.py -m gpu -x -q --timeout 200 --timeout-method thread -k "batch_admit or matches_oracle" > $O/pool_tests.log 2>&1 || { echo POOLTESTFAIL; tail -40 $O/pool_tests.log; exit 1; }
tail -1 $O/pool_tests.log
TXV_PROFILE_HOST=1 timeout -k 10 120 python3 -u tools/debug/pool_time.py 4 > $O/pool_prof.log 2>&1 || { echo POOLFAIL; tail $O/pool_prof.log; exit 3; }
grep -v "^\[txv pool\]" $O/pool_prof.log | tail -2
