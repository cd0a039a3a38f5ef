#!/bin/bash
# r3_fused_ab.sh TAG VARIANTS...: K1 parity tests on the in-tree build (V = 8 paths included),
# then bench.py's device-resident leg per build (cur = in-tree, else build_exp/NAME)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_configs.py::test_c2_full_size_matches_oracle tests/test_configs.py::test_c3_one_rank_full_shard_matches_oracle \
  tests/test_configs.py::test_lane_votes_8_without_the_wide_base_table > $O/tests.log 2>&1 \
  || { echo TESTFAIL; tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
bash tools/profile/ab.sh $TAG "$@"
for v in "$@"; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['device_ms_standalone'])" $O/$v.json $v; done
