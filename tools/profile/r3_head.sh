#!/bin/bash
# r3_head.sh TAG: whole -m gpu suite, smoke, default bench, kernel trace of the bench workload
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_head}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail $O/smoke.log; exit 2; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'],b['ms_per_step'],b['device_ms_standalone'],b['end_to_end']['registered']['votes_per_s'],b['c5_streaming']['votes_per_s'],b['c5_streaming']['p50_commit_latency_ms'],b['c5_wire']['votes_per_s'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e --steps 5 --warmup 1 > $O/kt_bench.json 2> $O/kt_bench.err || { echo KTFAIL; exit 4; }
echo ALLDONE
