# fused status + event compaction kernel: the whole -m gpu suite, then the C5 legs and the C2 legs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_ev}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python3 bench.py --c5-only > $O/c5.json 2> $O/c5.err || { echo "C5FAIL"; tail -5 $O/c5.err; exit 2; }
python3 -c "
import json;b=json.load(open('$O/c5.json'));c=b['c5_streaming'];w=b['c5_wire']
print('c5', c['votes_per_s'], c['votes_per_s_passes'], c['correct'], c['pool_matches_oracle'], c['p50_commit_latency_ms'], c['device_ms_batch']['standalone'], c['device_ms_batch']['in_pipeline_p50'])
print('wire', w['votes_per_s'], w.get('correct'))"
B="python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e"
for rep in 1 2; do
  timeout -k 10 300 $B > $O/c2_$rep.json 2> $O/c2_$rep.err || { echo "C2FAIL $rep"; tail -3 $O/c2_$rep.err; exit 4; }
  python3 -c "import json;b=json.load(open('$O/c2_$rep.json'));print('rep $rep',b['value'],b['ms_per_step'],b['device_ms_standalone'],b['device_ms_p50']['tally_after_verify'],b['roofline']['traffic'])"
done
echo ALLDONE
