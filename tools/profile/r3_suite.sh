#!/bin/bash
# r3_suite.sh TAG: the whole -m gpu suite + smoke on this tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
echo ALLDONE
