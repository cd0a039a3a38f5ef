#!/bin/bash
# r3_tally.sh TAG: the whole -m gpu suite (tally parity: duplicates, conflicts, invalid, replays,
# C4-shaped streams), a bench run, then FETCH_SIZE / WRITE_SIZE passes of the C2 bench workload
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_tally}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
B="python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e"
timeout -k 10 300 $B --steps 30 --warmup 3 > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 2; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'],b['ms_per_step'],b['device_ms_p50'],b['device_ms_standalone'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $B --steps 5 --warmup 1 > $O/bench_kt.json 2> $O/bench_kt.err || { echo KTFAIL; exit 3; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_b -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_b.err || { echo PMCB; exit 4; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_c.err || { echo PMCC; exit 5; }
echo ALLDONE
