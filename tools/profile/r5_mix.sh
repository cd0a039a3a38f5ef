# the interleaved wire / SoA device-pool test and the device pool suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_mix}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_pool_device.py -x -v -k "interleaved or update_submit or compaction" -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo ALLDONE
