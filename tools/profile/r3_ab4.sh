#!/bin/bash
# 3-wave work-stealing K1b at partial occupancy: blocks per CU x 100 swept, beside the in-tree kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_ab4}
mkdir -p $O
for rep in 1 2; do
  TXV_EXP_SKIP=0 timeout -k 10 200 python3 -u tools/debug/corun_exp.py >> $O/corun.jsonl 2> $O/corun_cur.err || { echo "FAIL cur"; exit 3; }
  tail -1 $O/corun.jsonl
  for b in 200 225 250 275; do
    TXV_K1B_DYN_BLOCKS=$b TXV_LIB_PATH=$PWD/build_exp/dyn3/libtxvote.so TXV_EXP_SKIP=0 timeout -k 10 200 python3 -u tools/debug/corun_exp.py >> $O/corun.jsonl 2> $O/corun_$b.err || { echo "FAIL $b"; tail -3 $O/corun_$b.err; exit 3; }
    echo "blocks $b: $(tail -1 $O/corun.jsonl)"
  done
done
