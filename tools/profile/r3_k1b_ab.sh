#!/bin/bash
# r3_k1b_ab.sh TAG VARIANTS...: walk microbenches, then K1b parity tests on the in-tree build,
# then bench.py's device-resident leg per build (cur = in-tree, else build_exp/NAME)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for w in tools/microbench/walk_rate*; do
  case $w in *.hip) continue;; esac
  timeout -k 10 120 $w > $O/$(basename $w).json 2>&1 || { echo "WALKFAIL $w"; exit 1; }
  echo "$(basename $w): $(grep -o '"mode": "[a-z_0-9]*", "ms": [0-9.]*' $O/$(basename $w).json | tr '\n' ' ')"
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_configs.py::test_c2_full_size_matches_oracle tests/test_configs.py::test_c4_adversarial_1m_gate > $O/tests.log 2>&1 \
  || { echo TESTFAIL; tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
bash tools/profile/ab.sh $TAG "$@"
