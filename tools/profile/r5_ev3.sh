# the whole -m gpu suite, then the C5 legs twice
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_ev3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for rep in 1 2; do
  timeout -k 10 400 python3 bench.py --c5-only > $O/c5_$rep.json 2> $O/c5_$rep.err || { echo "C5FAIL"; tail -5 $O/c5_$rep.err; exit 2; }
  python3 -c "
import json;b=json.load(open('$O/c5_$rep.json'));c=b['c5_streaming'];w=b['c5_wire']
print('c5', c['votes_per_s'], c['votes_per_s_passes'], c['correct'], c['pool_matches_oracle'], c['p50_commit_latency_ms'])
print('wire', w['votes_per_s'], w['votes_per_s_passes'], w['correct'], w['pool_matches_oracle'], w['p50_admit_ms'], w['p50_commit_latency_ms'], w['unloaded']['p50_commit_latency_ms'])"
done
echo ALLDONE
