#!/bin/bash
# walk microbench (incl. 40 back-to-back launches), pool/ingest GPU tests, default bench with the
# host pool phase timings (bench.err)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_batch5}
mkdir -p $O
timeout -k 10 120 tools/microbench/walk_rate > $O/walk_rate.json 2>&1 || { echo WALKFAIL; exit 1; }
timeout -k 10 120 tools/microbench/walk_rate_sgpr > $O/walk_rate_sgpr.json 2>&1 || { echo WALKFAIL; exit 1; }
cat $O/walk_rate_sgpr.json | tr "\n" " "; echo
cat $O/walk_rate.json | tr '\n' ' '; echo
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_pool.py tests/test_wire.py \
  > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 2; }
tail -1 $O/tests.log
TXV_PROFILE_HOST=1 timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'],b['ms_per_step'],b['device_ms_p50'],b['device_ms_standalone']);c=b['c5_streaming'];print({k:c[k] for k in c if k!='workload'});print(b['c5_wire']['votes_per_s'], b['c5_wire']['p50_commit_latency_ms'])"
grep "batch:" $O/bench.err | tail -3
grep "keys+sizes" $O/bench.err | tail -2
