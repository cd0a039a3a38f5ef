#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_ingest}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_wire.py tests/test_pool.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -50 $O/tests.log; exit 1; }
tail -3 $O/tests.log
