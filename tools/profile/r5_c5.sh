# bench.py --c5-only (SoA leg: host- and device-cache passes; wire leg)
set -o pipefail
O=gpurun_out/${1:-r5_c5}
mkdir -p $O
TXV_BENCH_WATCHDOG=100 timeout -k 10 400 python3 -u bench.py --c5-only > $O/c5.json 2> $O/c5.err || { echo C5FAIL; grep "^\[c5" $O/c5.err; tail -5 $O/c5.err; exit 5; }
grep "^\[c5" $O/c5.err
python3 -c "
import json; d=json.load(open('$O/c5.json'))
for k in ('c5_streaming','c5_wire'):
    c=d.get(k,{}); print(k, c.get('votes_per_s'), c.get('votes_per_s_passes'), c.get('correct'), c.get('pool_matches_oracle'), c.get('p50_commit_latency_ms'), c.get('p99_commit_latency_ms'))
"
echo ALLDONE
