#!/bin/bash
# r3_newtests.sh TAG: the round-3 GPU tests (out-of-order fetch, C1, C3 full shard, multi-rank step path)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r3_newtests}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_configs.py::test_fetch_out_of_run_order_keeps_every_set_tallied \
  tests/test_configs.py::test_c1_full_config_matches_oracle \
  tests/test_dist_gpu.py \
  tests/test_configs.py::test_c3_one_rank_full_shard_matches_oracle > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -8 $O/tests.log
echo ALLDONE
