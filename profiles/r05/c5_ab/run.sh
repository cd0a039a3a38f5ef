# C5 SoA leg (device pass only) under engine / stream placement variants: one line per pass
set -o pipefail
O=gpurun_out/${1:-r5_ab}
mkdir -p $O
run() {
  local tag=$1; shift
  env "$@" TXV_C5_DEVICE_ONLY=1 TXV_BENCH_WATCHDOG=100 timeout -k 10 200 python3 -u bench.py --c5-only --no-wire > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAIL"; tail -3 $O/$tag.err; return 1; }
  echo "== $tag $*"; grep "cache pass" $O/$tag.err | sed 's/correct.*p50 ms/ p50 ms/'
}
run base X=0 && run vcoff16 TXV_VERIFY_CUS_OFF=16 && run vcoff32 TXV_VERIFY_CUS_OFF=32 && run poolkey TXV_POOL_STREAM=2 && run poolnorm TXV_POOL_STREAM=1 && run infl3 TXV_C5_INFLIGHT=3
echo ALLDONE
