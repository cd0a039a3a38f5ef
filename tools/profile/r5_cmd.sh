set -o pipefail
O=gpurun_out/r5_ab6
mkdir -p $O
for m in 0:2 2:2 2:3; do
  ps=${m%:*}; fl=${m#*:}
  TXV_BENCH_WATCHDOG=100 TXV_POOL_STREAM=$ps TXV_C5_INFLIGHT=$fl timeout -k 10 330 python3 -u bench.py --c5-only > $O/c5_m$ps$fl.json 2> >(tee $O/c5_m$ps$fl.err >&2) || { echo C5FAIL $m; tail -30 $O/c5_m$ps$fl.err; exit 5; }
  python3 -c "
import json
d=json.load(open('$O/c5_m$ps$fl.json'))
c=d['c5_streaming']; w=d.get('c5_wire',{})
print('mode $m c5', c['votes_per_s'], c['votes_per_s_passes'], c['correct'], c['pool_matches_oracle'], c['p50_commit_latency_ms'], 'maxsize', c['pool_size_max'], 'host', c['host_cache']['votes_per_s'], 'unl', c['unloaded']['correct'], 'standalone', c['device_ms_batch']['standalone'])
print('mode $m wire', w.get('votes_per_s'), w.get('votes_per_s_passes'), w.get('correct'), w.get('p50_commit_latency_ms'), w['unloaded']['correct'])"
done
echo ALLDONE
