# whole -m gpu suite; C2 bench legs (base 26) and their kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_step5}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
B="python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e"
timeout -k 10 300 $B > $O/c2.json 2> $O/c2.err || { echo C2FAIL; tail $O/c2.err; exit 2; }
python3 -c "import json;b=json.load(open('$O/c2.json'));print('c2',b['value'],b['ms_per_step'],b['device_ms_p50'],b['device_ms_standalone'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $B --steps 5 --warmup 1 > $O/bench_kt.json 2> $O/bench_kt.err || { echo KTFAIL; exit 4; }
echo ALLDONE
