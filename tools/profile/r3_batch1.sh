#!/bin/bash
# ingest + wire/pool GPU tests, C2 parity, K1a grid A/B (env), then one default bench run
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_batch1}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_wire.py tests/test_pool.py \
  tests/test_configs.py::test_c2_full_size_matches_oracle tests/test_gpu_parity.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -50 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/profile/env_ab.sh ${1:-r3_batch1}/k1a "TXV_K1A_BLOCKS_PER_CU=0" "TXV_K1A_BLOCKS_PER_CU=4" "TXV_K1A_BLOCKS_PER_CU=5" "TXV_K1A_BLOCKS_PER_CU=0" "TXV_K1A_BLOCKS_PER_CU=4" || exit 2
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'],b['ms_per_step'],b['device_ms_standalone']['verify'],b['end_to_end']['registered'],b['c5_streaming']['votes_per_s'],b['c5_streaming']['p50_commit_latency_ms'],b['c5_wire'])"
