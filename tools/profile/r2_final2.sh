#!/bin/bash
# r2_final2.sh TAG: -m gpu suite, smoke, default bench, kernel trace of the C2 leg
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2_final2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail $O/smoke.log; exit 2; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'],b['ms_per_step'],b['device_ms_p50']['verify'],b['roofline']['frac'],b['roofline']['standalone'],b['end_to_end']['registered']['votes_per_s'],b['c5_streaming']['votes_per_s'],b['c5_streaming']['p50_commit_latency_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e --steps 8 --warmup 2 > $O/kt_bench.json 2> $O/kt_bench.err || { echo KTFAIL; exit 4; }
echo ALLDONE
