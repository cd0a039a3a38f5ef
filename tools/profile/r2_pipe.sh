#!/bin/bash
# GPU check of the two-stream (verify / TxFlow) pipeline: -m gpu suite, bench (C2 only) under a
# kernel trace, plain bench, and the N=2 gloo rehearsal (two ranks on one GPU)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r2_pipe}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'],b['ms_per_step'],b['p50_batch_ms'],b['device_ms_p50'],b['end_to_end']['registered']['votes_per_s'],b['end_to_end']['pageable']['votes_per_s'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e --steps 5 --warmup 1 > $O/kt_bench.json 2> $O/kt_bench.err || { echo KTFAIL; exit 4; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --same-gpu > $O/n2.json 2> $O/n2.err || { echo N2FAIL; tail $O/n2.err; exit 5; }
tail -c 400 $O/n2.json
echo ALLDONE
