# C5: both legs; the SoA device pass without Update and with three TxFlow batches in flight; a
# kernel trace of the SoA device pass
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_c5ab2}
mkdir -p $O
TXV_BENCH_WATCHDOG=100 timeout -k 10 400 python3 -u bench.py --c5-only > $O/c5.json 2> $O/c5.err || { echo C5FAIL; grep "^\[c5" $O/c5.err; tail -5 $O/c5.err; exit 5; }
grep "^\[c5" $O/c5.err | grep -v "host cache"
run() {
  local tag=$1; shift
  env "$@" TXV_C5_DEVICE_ONLY=1 TXV_BENCH_WATCHDOG=100 timeout -k 10 200 python3 -u bench.py --c5-only --no-wire > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAIL"; tail -3 $O/$tag.err; return 1; }
  echo "== $tag $*"; grep "cache pass" $O/$tag.err | sed 's/correct.*p50 ms/ p50 ms/'
}
run noupd TXV_C5_NO_UPDATE=1 && run infl3 TXV_C5_INFLIGHT=3 &&
TXV_C5_DEVICE_ONLY=1 TXV_BENCH_WATCHDOG=100 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 -u bench.py --c5-only --no-wire > $O/kt.json 2> $O/kt.err || { echo KTFAIL; exit 6; }
grep "cache pass" $O/kt.err
find $O/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
find $O/kt -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $O/kernel_trace.csv
rm -rf $O/kt
echo ALLDONE
