# round-5 validation, part 2: kernel trace of the default bench's C2 leg and the four PMC passes
# (one --pmc pass per counter group, never with traces); summarise with tools/profile/summarize.py
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_val2}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e"
SQA="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
SQD="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $B --steps 5 --warmup 1 > $O/bench_kt.json 2> $O/bench_kt.err || { echo KTFAIL; exit 4; }
timeout -s KILL 200 rocprofv3 --pmc $SQA -d $O/pmc_a -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_a.err || { echo PMCA; exit 5; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_b -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_b.err || { echo PMCB; exit 6; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_c.err || { echo PMCC; exit 7; }
timeout -s KILL 200 rocprofv3 --pmc $SQD -d $O/pmc_d -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_d.err || { echo PMCD; exit 8; }
echo ALLDONE
