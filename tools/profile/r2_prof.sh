#!/bin/bash
# r2_prof.sh TAG: -m gpu suite, pool A/B, then rocprofv3 kernel trace + PMC passes of bench.py
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2_prof}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u tools/debug/pool_ab.py 6 > $O/pool_ab.log 2>&1 || { echo POOLFAIL; tail $O/pool_ab.log; exit 2; }
cat $O/pool_ab.log
bash tools/profile/run_profiles.sh $TAG || { echo PROFFAIL; exit 3; }
echo ALLDONE
