#!/bin/bash
# the C4 bit-exact gate at 10^8 adversarial votes on the current kernels (pipelined submit/wait)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
timeout -k 10 1080 python -u tools/gate/c4_gate.py --votes 100000000 --threads 16 --out gpurun_out/c4/gate_1e8_r2final.json > gpurun_out/c4/gate_1e8_r2final.log 2>&1
rc=$?
tail -3 gpurun_out/c4/gate_1e8_r2final.log
exit $rc
