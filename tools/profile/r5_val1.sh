# round-5 validation, part 1: the whole -m gpu suite, smoke, the default bench, and the bench
# with the radix-2^26 base table (C2 legs only) for the default decision
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_val1}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "
import json;b=json.load(open('$O/bench.json'))
print('value',b['value'],'ms',b['ms_per_step'],'roof',b['roofline']['frac'])
c=b.get('c5_streaming',{}); w=b.get('c5_wire',{})
print('c5',c.get('votes_per_s'),c.get('votes_per_s_passes'),c.get('correct'),c.get('pool_matches_oracle'),c.get('p50_commit_latency_ms'))
print('wire',w.get('votes_per_s'),w.get('correct'),w.get('p50_commit_latency_ms'))
print('e2e',b.get('end_to_end',{}).get('value') if isinstance(b.get('end_to_end'),dict) else b.get('end_to_end'))
"
timeout -k 10 400 python -u bench.py --base-w 26 --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e > $O/bench26.json 2> $O/bench26.err || { echo B26FAIL; tail $O/bench26.err; exit 4; }
python3 -c "import json;b=json.load(open('$O/bench26.json'));print('b26 value',b['value'],'ms',b['ms_per_step'])"
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e > $O/bench24.json 2> $O/bench24.err || { echo B24FAIL; tail $O/bench24.err; exit 5; }
python3 -c "import json;b=json.load(open('$O/bench24.json'));print('b24 value',b['value'],'ms',b['ms_per_step'])"
echo ALLDONE
