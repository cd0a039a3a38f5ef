#!/bin/bash
# does the out-of-order-fetch test catch the round-2 runtime (build_exp/oldrt)?  Expected: FAIL there.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_oldrt}
mkdir -p $O
TXV_LIB_PATH=$PWD/build_exp/oldrt/libtxvote.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu \
  tests/test_configs.py::test_fetch_out_of_run_order_keeps_every_set_tallied > $O/oldrt.log 2>&1
echo "old runtime rc=$?"
tail -5 $O/oldrt.log
