set -o pipefail
O=gpurun_out/r5_ab2
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_pool_device.py tests/test_tally_cross.py tests/test_pool.py tests/test_configs.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for m in 0 1 2; do
  TXV_POOL_STREAM=$m timeout -k 10 300 python3 bench.py --c5-only > $O/c5_m$m.json 2> $O/c5_m$m.err || { echo C5FAIL $m; tail -5 $O/c5_m$m.err; exit 5; }
  python3 -c "
import json
d=json.load(open('$O/c5_m$m.json'))
c=d['c5_streaming']; w=d.get('c5_wire',{})
print('mode $m c5', c['votes_per_s'], c['votes_per_s_passes'], c['correct'], c['pool_matches_oracle'], c['p50_commit_latency_ms'], 'maxsize', c['pool_size_max'], 'host', c['host_cache']['votes_per_s'], 'unl', c['unloaded']['correct'], 'standalone', c['device_ms_batch']['standalone'])
print('mode $m wire', w.get('votes_per_s'), w.get('votes_per_s_passes'), w.get('correct'), w.get('p50_commit_latency_ms'), w['unloaded']['correct'])"
done
echo ALLDONE
