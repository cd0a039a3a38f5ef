#!/bin/bash
# validate.sh TAG: whole -m gpu suite, smoke, default bench, then the kernel trace and the four PMC
# passes of the bench workload (one --pmc pass per counter group, never with traces); summarise
# with tools/profile/summarize.py gpurun_out/TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-validate}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail $O/smoke.log; exit 2; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'],b['ms_per_step'],b['device_ms_p50']['verify'],b['device_ms_standalone'])"
B="python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e"
SQA="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
SQD="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $B --steps 5 --warmup 1 > $O/bench_kt.json 2> $O/bench_kt.err || { echo KTFAIL; exit 4; }
timeout -s KILL 200 rocprofv3 --pmc $SQA -d $O/pmc_a -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_a.err || { echo PMCA; exit 5; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_b -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_b.err || { echo PMCB; exit 6; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_c.err || { echo PMCC; exit 7; }
timeout -s KILL 200 rocprofv3 --pmc $SQD -d $O/pmc_d -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_d.err || { echo PMCD; exit 8; }
echo ALLDONE
