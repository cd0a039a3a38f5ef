#!/bin/bash
# run_gate.sh DIR SHA [c4_gate.py args...]: the C4 gate at 1e8 adversarial votes
# (tools/gate/c4_gate.py) with the device-cache TxVotePool stage in front, at the windows the
# arguments give (bench.py's C2 context: --table-w 21 --base-w 26); progress lines to
# gpurun_out/DIR/gate.log (every 30 s the last one on stdout), the record to gpurun_out/DIR/gate.json
set -o pipefail
DIR=$1; SHA=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out/$DIR
TXV_HEAD=$SHA timeout -k 10 1150 python -u tools/gate/c4_gate.py --votes 100000000 --threads 16 --pool-device "$@" \
  --out gpurun_out/$DIR/gate.json > gpurun_out/$DIR/gate.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do
  sleep 30
  tail -1 gpurun_out/$DIR/gate.log | cut -c1-200
done
wait $pid
