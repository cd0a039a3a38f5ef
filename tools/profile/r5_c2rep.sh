# flow parity tests, then the C2 bench legs three times
set -o pipefail
O=gpurun_out/${1:-r5_c2rep}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_tally_cross.py tests/test_gpu_parity.py tests/test_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 4; }
tail -1 $O/tests.log
B="python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e"
for rep in 1 2 3; do
  timeout -k 10 300 $B > $O/c2_$rep.json 2> $O/c2_$rep.err || { echo "FAIL $rep"; tail -3 $O/c2_$rep.err; exit 2; }
  python3 -c "import json;b=json.load(open('$O/c2_$rep.json'));print('rep $rep',b['value'],b['ms_per_step'],b['device_ms_p50']['verify'],b['device_ms_p50']['tally_after_verify'])"
done
echo ALLDONE
