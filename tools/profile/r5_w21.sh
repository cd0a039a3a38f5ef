# radix-2^21 validator tables: the window parity tests, then C2 A/B (table window 20 vs 21)
set -o pipefail
O=gpurun_out/${1:-r5_w21}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "wide_base or window_policy" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 4; }
tail -1 $O/tests.log
B="python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e"
for rep in 1 2; do
  for tw in 20 21; do
    timeout -k 10 300 $B --table-w $tw > $O/c2_${tw}_$rep.json 2> $O/c2_${tw}_$rep.err || { echo "FAIL $tw $rep"; tail -5 $O/c2_${tw}_$rep.err; exit 2; }
    python3 -c "import json;b=json.load(open('$O/c2_${tw}_$rep.json'));r=b['roofline'];print('w $tw rep $rep',b['value'],b['ms_per_step'],b['device_ms_p50']['verify'],r['frac'],r['standalone'])"
  done
done
echo ALLDONE
