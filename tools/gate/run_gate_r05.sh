#!/bin/bash
# run_gate_r05.sh SHA: the C4 gate at 1e8 adversarial votes with the device-cache TxVotePool stage
# in front (tools/gate/c4_gate.py --pool-device), progress lines straight to a file under
# gpurun_out/r5_gate/ (and every 10th batch on stdout), the record as JSON
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_gate
TXV_HEAD=$1 timeout -k 10 1150 python -u tools/gate/c4_gate.py --votes 100000000 --threads 16 --pool-device \
  --out gpurun_out/r5_gate/gate_1e8_dev_$1.json > gpurun_out/r5_gate/gate_1e8_dev_$1.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do
  sleep 30
  tail -1 gpurun_out/r5_gate/gate_1e8_dev_$1.log | cut -c1-200
done
wait $pid
