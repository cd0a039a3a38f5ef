# round-5 final validation in one call: the whole -m gpu suite, smoke, the default bench, the C2
# legs twice more, then the kernel trace and the four PMC passes of the C2 legs (one --pmc pass per
# counter group, never with traces); summarise with tools/profile/summarize.py
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_val6}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "
import json;b=json.load(open('$O/bench.json'))
print('value',b['value'],'ms',b['ms_per_step'],'roof',b['roofline']['frac'],b['device_ms_standalone'])
c=b.get('c5_streaming',{}); w=b.get('c5_wire',{})
print('c5',c.get('votes_per_s'),c.get('votes_per_s_passes'),c.get('correct'),c.get('pool_matches_oracle'),c.get('p50_commit_latency_ms'))
print('wire',w.get('votes_per_s'),w.get('correct'),w.get('p50_commit_latency_ms'))
"
B="python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e"
for rep in 1 2; do
  timeout -k 10 300 $B > $O/c2_$rep.json 2> $O/c2_$rep.err || { echo "C2FAIL $rep"; tail -3 $O/c2_$rep.err; exit 4; }
  python3 -c "import json;b=json.load(open('$O/c2_$rep.json'));print('rep $rep',b['value'],b['ms_per_step'],b['device_ms_standalone']['k1b'])"
done
SQA="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
SQD="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $B --steps 5 --warmup 1 > $O/bench_kt.json 2> $O/bench_kt.err || { echo KTFAIL; exit 5; }
timeout -s KILL 200 rocprofv3 --pmc $SQA -d $O/pmc_a -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_a.err || { echo PMCA; exit 6; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_b -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_b.err || { echo PMCB; exit 7; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_c.err || { echo PMCC; exit 8; }
timeout -s KILL 200 rocprofv3 --pmc $SQD -d $O/pmc_d -o pmc --output-format csv -- $B --steps 2 --warmup 0 > /dev/null 2> $O/pmc_d.err || { echo PMCD; exit 9; }
echo ALLDONE
