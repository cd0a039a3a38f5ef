set -o pipefail
O=gpurun_out/r5_ab5
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "^E  " $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for m in 0:2 2:2 2:3; do
  ps=${m%:*}; fl=${m#*:}
  TXV_POOL_STREAM=$ps TXV_C5_INFLIGHT=$fl timeout -k 10 300 python3 bench.py --c5-only > $O/c5_m$ps$fl.json 2> $O/c5_m$ps$fl.err || { echo C5FAIL $m; tail -5 $O/c5_m$ps$fl.err; exit 5; }
  python3 -c "
import json
d=json.load(open('$O/c5_m$ps$fl.json'))
c=d['c5_streaming']; w=d.get('c5_wire',{})
print('mode $m c5', c['votes_per_s'], c['votes_per_s_passes'], c['correct'], c['pool_matches_oracle'], c['p50_commit_latency_ms'], 'maxsize', c['pool_size_max'], 'host', c['host_cache']['votes_per_s'], 'unl', c['unloaded']['correct'], 'standalone', c['device_ms_batch']['standalone'])
print('mode $m wire', w.get('votes_per_s'), w.get('votes_per_s_passes'), w.get('correct'), w.get('p50_commit_latency_ms'), w['unloaded']['correct'])"
done
echo ALLDONE
