#!/bin/bash
# full -m gpu suite without -x (every failure reported)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r2_nox}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" $O/gpu_tests.log | tail -30
exit $rc
