#!/bin/bash
# microbench (pure-ALU walk ceiling) then the -m gpu suite + smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_mb}
mkdir -p $O
timeout -k 10 120 ./tools/microbench/fe10_rate > $O/fe10_rate.json 2> $O/fe10_rate.err || { echo MBFAIL; cat $O/fe10_rate.err; exit 1; }
cat $O/fe10_rate.json
bash tools/profile/r3_suite.sh ${1:-r3_mb}
