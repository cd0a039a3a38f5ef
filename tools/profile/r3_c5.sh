#!/bin/bash
# r3_c5.sh TAG: pool GPU tests, then bench.py's C5 legs (host pool phase timings in bench.err)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_c5}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_pool.py tests/test_wire.py \
  > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
TXV_PROFILE_HOST=1 timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-c1 --no-wire --no-e2e --no-cpu-baseline \
  > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['c5_streaming']);print(b['c5_wire'])"
grep "batch:" $O/bench.err | tail -4
bash tools/profile/r3_corun.sh ${1:-r3_c5}/corun 255 0 255 || exit 4
CORUN_LIB=build_exp/notail CORUN_TAG=notail bash tools/profile/r3_corun.sh ${1:-r3_c5}/corun 0 || exit 5
CORUN_LIB=build_exp/nowalk CORUN_TAG=nowalk bash tools/profile/r3_corun.sh ${1:-r3_c5}/corun 0 || exit 6
