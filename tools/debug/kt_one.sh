#!/bin/bash
# kernel-trace stats of the experiment timer for one library build: tools/debug/kt_one.sh <lib.so> <tag>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/$2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$2 -o kt --output-format csv -- python3 tools/debug/exp_verify_time.py $1 > gpurun_out/$2/log 2>&1
