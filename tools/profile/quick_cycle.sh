#!/bin/bash
# usage: prof_run.sh TAG  -- GPU tests, kernel trace, bench
set -o pipefail
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/$TAG/gpu.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e --steps 5 --warmup 1 > gpurun_out/$TAG/kt_bench.json 2> gpurun_out/$TAG/kt_bench.err || { echo KTFAIL; grep -v "^[EW]20" gpurun_out/$TAG/kt_bench.err | tail; exit 2; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-c5 --no-c1 --no-wire --no-cpu-baseline > gpurun_out/$TAG/bench.log 2>&1 || { echo BENCHFAIL; tail gpurun_out/$TAG/bench.log; exit 3; }
tail -2 gpurun_out/$TAG/gpu.log
