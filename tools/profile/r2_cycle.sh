#!/bin/bash
# r2_cycle.sh TAG [variants...]: -m gpu suite, then bench.py's C2 leg for the in-tree build and each
# build_exp/<variant> (A/B on one box), then a kernel trace of the in-tree build
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-cycle}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/profile/ab.sh $TAG cur "$@" || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e --steps 5 --warmup 1 > $O/kt_bench.json 2> $O/kt_bench.err || { echo KTFAIL; exit 4; }
echo ALLDONE
