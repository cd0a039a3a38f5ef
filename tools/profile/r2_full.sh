#!/bin/bash
# r2_full.sh TAG: -m gpu suite, smoke, the default bench (every leg), a kernel trace of the C2
# leg, the small-batch lane_votes sweep and the N=2 gloo rehearsal (two ranks on one GPU)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r2_full}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail $O/smoke.log; exit 2; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'],b['ms_per_step'],b['p50_batch_ms'],b['device_ms_p50']['verify'],b['device_ms_p50']['tally_after_verify'],b['device_ms_standalone'],b['end_to_end']['registered']['votes_per_s'],b['c5_streaming']['votes_per_s'],b['c5_streaming']['p50_commit_latency_ms'],b['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e --steps 8 --warmup 2 > $O/kt_bench.json 2> $O/kt_bench.err || { echo KTFAIL; exit 4; }
timeout -k 10 240 python -u tools/debug/exp_small_batch.py 65536 1000 > $O/small.log 2>&1 || { echo SMALLFAIL; tail $O/small.log; exit 5; }
cat $O/small.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 --dist-backend gloo --same-gpu > $O/n2.json 2> $O/n2.err || { echo N2FAIL; tail $O/n2.err; exit 6; }
grep -o '"value": [0-9.]*' $O/n2.json
echo ALLDONE
