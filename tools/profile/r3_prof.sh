#!/bin/bash
# r3_prof.sh TAG: kernel trace + PMC passes of the bench workload on this build, plus the same
# PMC passes over the VALU issue-rate probe (calibrates what the cycle counters count).
# One --pmc pass per counter group, never combined with traces.  Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r3_prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e"
P="python3 tools/profile/valu_probe_run.py"
SQA="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
SQD="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $B --steps 5 --warmup 1 > $OUT/bench_kt.json 2> $OUT/bench_kt.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc $SQA -d $OUT/pmc_a -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $OUT/pmc_a.err || exit 2
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_b -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $OUT/pmc_b.err || exit 3
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_c -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $OUT/pmc_c.err || exit 4
timeout -s KILL 200 rocprofv3 --pmc $SQD -d $OUT/pmc_d -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $OUT/pmc_d.err || exit 5
timeout -s KILL 120 rocprofv3 --pmc $SQA -d $OUT/probe_a -o pmc --output-format csv -- $P > $OUT/probe.log 2> $OUT/probe_a.err || exit 6
timeout -s KILL 120 rocprofv3 --pmc $SQD -d $OUT/probe_d -o pmc --output-format csv -- $P >> $OUT/probe.log 2> $OUT/probe_d.err || exit 7
echo profiles done
