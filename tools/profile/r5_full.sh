# the whole -m gpu suite, then the C5 SoA leg (device pass) with the pool phase timers
set -o pipefail
O=gpurun_out/${1:-r5_full}
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 4; }
tail -3 $O/tests.log
TXV_C5_DEVICE_ONLY=1 TXV_BENCH_WATCHDOG=100 timeout -k 10 300 python3 -u bench.py --c5-only --no-wire > $O/c5.json 2> $O/c5.err || { echo C5FAIL; grep "^\[c5" $O/c5.err; tail -5 $O/c5.err; exit 5; }
grep "^\[c5" $O/c5.err
echo ALLDONE
