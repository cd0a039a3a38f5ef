# kernel trace of the C5 SoA leg (device pass only) with the pool list in HBM
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_trace_pl
mkdir -p $O
TXV_C5_DEVICE_ONLY=1 TXV_BENCH_WATCHDOG=100 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 -u bench.py --c5-only --no-wire > $O/c5_kt.json 2> $O/c5_kt.err || { echo KTFAIL; tail -5 $O/c5_kt.err; exit 4; }
grep "^\[c5" $O/c5_kt.err
find $O/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
find $O/kt -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $O/kernel_trace.csv
ls -la $O
echo ALLDONE
