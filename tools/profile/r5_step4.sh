# pool tests, then the C5 SoA device pass: signature uploads on the copy stream (default) vs the engine's stream
set -o pipefail
O=gpurun_out/${1:-r5_step4}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_pool_device.py tests/test_pool.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 4; }
tail -2 $O/tests.log
run() {
  local tag=$1; shift
  env "$@" TXV_C5_DEVICE_ONLY=1 TXV_BENCH_WATCHDOG=100 timeout -k 10 200 python3 -u bench.py --c5-only --no-wire > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAIL"; tail -3 $O/$tag.err; return 1; }
  echo "== $tag $*"; grep "cache pass" $O/$tag.err | sed 's/correct.*p50 ms/ p50 ms/'
}
run up1 X=0 && run up0 TXV_POOL_UPLOAD_STREAM=0 && run up1b X=0 && run noupd TXV_C5_NO_UPDATE=1
echo ALLDONE
