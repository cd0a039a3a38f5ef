#!/bin/bash
# c5_trace.sh TAG: kernel trace (per dispatch + stats) of bench.py's C5 legs (SoA and wire, the
# pool engine's pd_* kernels and the 64k TxFlow chains in the pipeline), then the C5 legs alone
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-c5trace}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --c5-only > $O/c5_kt.json 2> $O/c5_kt.err || { echo KTFAIL; tail -5 $O/c5_kt.err; exit 4; }
timeout -k 10 300 python3 bench.py --c5-only > $O/c5.json 2> $O/c5.err || { echo C5FAIL; tail -5 $O/c5.err; exit 5; }
python3 -c "
import json
d=json.load(open('$O/c5.json'))
c=d['c5_streaming']; w=d.get('c5_wire',{})
print('c5', c['votes_per_s'], c['correct'], c['p50_commit_latency_ms'], c['device_ms_batch'])
print('wire', w.get('votes_per_s'), w.get('correct'), w.get('p50_commit_latency_ms'))"
echo ALLDONE
