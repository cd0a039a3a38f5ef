#!/bin/bash
# 3-waves/SIMD work-stealing K1b (build_exp/dyn3): parity, same-box A/B vs the in-tree 2-wave
# kernel; then the base-window A/B (radix 2^24 vs 2^26) on the in-tree build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_ab3}
mkdir -p $O
TXV_LIB_PATH=$PWD/build_exp/dyn3/libtxvote.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_configs.py::test_c2_full_size_matches_oracle tests/test_configs.py::test_c4_adversarial_1m_gate > $O/tests.log 2>&1 \
  || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in dyn3 cur; do
    if [ $v = cur ]; then
      TXV_EXP_SKIP=0 timeout -k 10 200 python3 -u tools/debug/corun_exp.py >> $O/corun.jsonl 2> $O/corun_cur.err || { echo "FAIL cur"; tail -3 $O/corun_cur.err; exit 3; }
    else
      TXV_LIB_PATH=$PWD/build_exp/$v/libtxvote.so TXV_EXP_SKIP=0 timeout -k 10 200 python3 -u tools/debug/corun_exp.py >> $O/corun.jsonl 2> $O/corun_$v.err || { echo "FAIL $v"; tail -3 $O/corun_$v.err; exit 3; }
    fi
    tail -1 $O/corun.jsonl
  done
done
bash tools/profile/r3_wb.sh ${1:-r3_ab3}/wb || exit 4
