#!/bin/bash
# same-box A/B: walk microbench variants, then the C2 pipeline with the old tally chain
# (build_exp/oldchain = e4108e3), the new chain without wave priority (prio0) and the in-tree build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_ab2}
mkdir -p $O
for w in walk_rate walk_rate_nofence walk_rate_noregstage; do
  timeout -k 10 120 tools/microbench/$w > $O/$w.json 2>&1 || { echo "WALKFAIL $w"; exit 1; }
  echo "$w: $(grep -o '"mode": "[a-z_0-9]*", "ms": [0-9.]*' $O/$w.json | tr '\n' ' ')"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_configs.py::test_c2_full_size_matches_oracle \
  tests/test_configs.py::test_c4_adversarial_1m_gate > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in oldchain prio0 cur; do
    if [ $v = cur ]; then unset CORUN_LIB; CL=""; else CL=build_exp/$v; fi
    if [ -z "$CL" ]; then
      TXV_EXP_SKIP=0 timeout -k 10 200 python3 -u tools/debug/corun_exp.py >> $O/corun.jsonl 2> $O/corun_cur.err || { echo "FAIL cur"; exit 3; }
    else
      TXV_LIB_PATH=$PWD/$CL/libtxvote.so TXV_EXP_SKIP=0 timeout -k 10 200 python3 -u tools/debug/corun_exp.py >> $O/corun.jsonl 2> $O/corun_$v.err || { echo "FAIL $v"; tail -3 $O/corun_$v.err; exit 3; }
    fi
    tail -1 $O/corun.jsonl
  done
done
