#!/bin/bash
# r3_corun.sh TAG MASK...: co-running attribution, one process per TXV_EXP_SKIP mask (build_exp/skip)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for m in "$@"; do
  TXV_LIB_PATH=$PWD/${CORUN_LIB:-build_exp/skip}/libtxvote.so TXV_EXP_SKIP=$m timeout -k 10 200 python3 -u tools/debug/corun_exp.py \
    >> $O/corun.jsonl 2> $O/corun_${CORUN_TAG:-}$m.err || { echo "FAIL $m"; tail -5 $O/corun_$m.err; exit 1; }
  tail -1 $O/corun.jsonl
done
