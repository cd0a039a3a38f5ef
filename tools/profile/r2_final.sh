#!/bin/bash
# r2_final.sh TAG: -m gpu suite, smoke, default bench, rocprofv3 kernel trace + PMC passes
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2_final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail $O/smoke.log; exit 2; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'],b['ms_per_step'],b['device_ms_standalone'],b['end_to_end']['registered']['votes_per_s'],b['c5_streaming']['votes_per_s'],b['c5_streaming']['p50_commit_latency_ms'],b['cpu_baseline']['value'])"
bash tools/profile/run_profiles.sh $TAG || { echo PROFFAIL; exit 4; }
echo ALLDONE
