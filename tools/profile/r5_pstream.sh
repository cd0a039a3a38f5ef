# pool engine on the copy stream (TXV_POOL_STREAM=3) vs the key stream (default), C5 legs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_pstream}
mkdir -p $O
for m in 3 2 3; do
  TXV_POOL_STREAM=$m timeout -k 10 400 python3 bench.py --c5-only > $O/c5_$m.json 2> $O/c5_$m.err || { echo "C5FAIL $m"; tail -5 $O/c5_$m.err; exit 2; }
  python3 -c "
import json;b=json.load(open('$O/c5_$m.json'));c=b['c5_streaming'];w=b['c5_wire']
print('mode $m c5', c['votes_per_s'], c['votes_per_s_passes'], c['correct'], c['pool_matches_oracle'], c['p50_commit_latency_ms'])
print('mode $m wire', w['votes_per_s'], w['votes_per_s_passes'], w['correct'], w['p50_admit_ms'], w['p50_commit_latency_ms'])"
done
echo ALLDONE
