# pool + C4 pool-stage tests on the GPU, then r5_c5ab2.sh
set -o pipefail
O=gpurun_out/${1:-r5_step}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_pool_device.py tests/test_pool.py tests/test_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 4; }
tail -2 $O/tests.log
bash tools/profile/r5_c5ab2.sh ${1:-r5_step}
