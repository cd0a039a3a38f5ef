#!/bin/bash
# r2_cycle2.sh TAG: r2_cycle.sh (tests, A/B, kernel trace) + small-batch lane_votes sweep per build
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-cycle}; shift
bash tools/profile/r2_cycle.sh $TAG "$@" || exit 1
O=gpurun_out/$TAG
unset TXV_LIB_PATH
timeout -k 10 240 python -u tools/debug/exp_small_batch.py 65536 1000 > $O/small_cur.log 2>&1 || { echo SMALLFAIL; tail $O/small_cur.log; exit 5; }
cat $O/small_cur.log
for v in "$@"; do
  TXV_LIB_PATH=$PWD/build_exp/$v/libtxvote.so timeout -k 10 240 python -u tools/debug/exp_small_batch.py 65536 1000 > $O/small_$v.log 2>&1 || { echo SMALLFAIL $v; tail $O/small_$v.log; exit 6; }
  echo "== $v"; cat $O/small_$v.log
done
