#!/bin/bash
# run_gate_1e8.sh SHA: the C4 gate at 1e8 adversarial votes with the TxVotePool stage in front
# (tools/gate/c4_gate.py), progress on stdout, record under gpurun_out/r3_gate/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3_gate
TXV_HEAD=$1 timeout -k 10 1150 python -u tools/gate/c4_gate.py --votes 100000000 --threads 16 \
  --out gpurun_out/r3_gate/gate_1e8_$1.json 2>&1 | tee gpurun_out/r3_gate/gate_1e8_$1.log | grep -E "batch [0-9]*0 |mismatches\": " 
