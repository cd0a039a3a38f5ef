#!/bin/bash
# pool / ingest GPU tests, co-running attribution (build_exp/skip), one default bench run
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_batch2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_pool.py tests/test_wire.py \
  > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/profile/r3_corun.sh ${1:-r3_batch2}/corun 0 16 32 48 4 60 || exit 2
TXV_PROFILE_HOST=1 timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'],b['ms_per_step'],b['device_ms_p50'],b['device_ms_standalone']);print(b['c5_streaming']);print(b['c5_wire'])"
