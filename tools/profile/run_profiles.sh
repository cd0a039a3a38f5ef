#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root).
# Kernel trace + stats first, then one PMC pass per counter group (never combined with
# runtime/sys traces).  Outputs under gpurun_out/$TAG/.
set -o pipefail
TAG=${1:-prof}
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e"
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $B --steps 5 --warmup 1 > $OUT/bench_kt.json 2> $OUT/bench_kt.err || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc_a -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $OUT/pmc_a.err || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_b -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $OUT/pmc_b.err || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_c -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $OUT/pmc_c.err || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_d -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $OUT/pmc_d.err || exit 5
echo profiles done
