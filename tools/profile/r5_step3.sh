# pool + C4 pool-stage tests on the GPU, then the C5 SoA device pass with and without Update
set -o pipefail
O=gpurun_out/${1:-r5_step3}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_pool_device.py tests/test_pool.py tests/test_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 4; }
tail -2 $O/tests.log
run() {
  local tag=$1; shift
  env "$@" TXV_C5_DEVICE_ONLY=1 TXV_BENCH_WATCHDOG=100 timeout -k 10 200 python3 -u bench.py --c5-only --no-wire > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAIL"; tail -3 $O/$tag.err; return 1; }
  echo "== $tag $*"; grep "cache pass" $O/$tag.err | sed 's/correct.*p50 ms/ p50 ms/'
}
run upd X=0 && run noupd TXV_C5_NO_UPDATE=1 && run upd2 X=0
echo ALLDONE
