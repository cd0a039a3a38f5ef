#!/bin/bash
# whole -m gpu suite, smoke, default bench (C5 pool phases in bench.err), co-running / K1b attribution
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_batch3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail $O/smoke.log; exit 2; }
TXV_PROFILE_HOST=1 timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'],b['ms_per_step'],b['device_ms_p50'],b['device_ms_standalone']);print(b['c5_streaming']);print(b['c5_wire'])"
grep "batch:" $O/bench.err | tail -3
bash tools/profile/r3_corun.sh ${1:-r3_batch3}/corun 255 0 || exit 4
CORUN_LIB=build_exp/notail CORUN_TAG=notail bash tools/profile/r3_corun.sh ${1:-r3_batch3}/corun 0 || exit 5
CORUN_LIB=build_exp/nowalk CORUN_TAG=nowalk bash tools/profile/r3_corun.sh ${1:-r3_batch3}/corun 0 || exit 6
echo ALLDONE
