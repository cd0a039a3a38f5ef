# round-5 final validation of the last tree: the whole -m gpu suite, smoke, the default bench, the
# C2 legs twice more
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_val7}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "
import json;b=json.load(open('$O/bench.json'))
r=b['roofline'];print('value',b['value'],'ms',b['ms_per_step'],'roof',r['frac'],'traffic',r['traffic'],b['device_ms_standalone'])
c=b.get('c5_streaming',{}); w=b.get('c5_wire',{}); e=b.get('end_to_end',{})
print('c5',c.get('votes_per_s'),c.get('votes_per_s_passes'),c.get('correct'),c.get('pool_matches_oracle'),c.get('p50_commit_latency_ms'),c.get('p99_commit_latency_ms'))
print('wire',w.get('votes_per_s'),w.get('votes_per_s_passes'),w.get('correct'),w.get('p50_commit_latency_ms'))
print('e2e',{k:(v.get('votes_per_s') if isinstance(v,dict) else v) for k,v in e.items() if k!='note'})
print('cpu',b['cpu_baseline'].get('value'),b['cpu_baseline'].get('cores'),'c1',b.get('c1',{}).get('votes_per_s'))
"
B="python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e"
for rep in 1 2; do
  timeout -k 10 300 $B > $O/c2_$rep.json 2> $O/c2_$rep.err || { echo "C2FAIL $rep"; tail -3 $O/c2_$rep.err; exit 4; }
  python3 -c "import json;b=json.load(open('$O/c2_$rep.json'));print('rep $rep',b['value'],b['ms_per_step'],b['device_ms_standalone']['k1b'])"
done
echo ALLDONE
