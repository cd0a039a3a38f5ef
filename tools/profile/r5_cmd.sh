set -o pipefail
O=gpurun_out/r5_prof2
mkdir -p $O
TXV_PROFILE_HOST=1 TXV_C5_DEVICE_ONLY=1 TXV_BENCH_WATCHDOG=100 timeout -k 10 300 python3 -u bench.py --c5-only --no-wire > $O/c5.json 2> $O/c5.err || { echo C5FAIL; grep "^\[c5" $O/c5.err; tail -5 $O/c5.err; exit 5; }
grep "^\[c5" $O/c5.err
python3 - <<'PY'
import re, collections, statistics
d = collections.defaultdict(lambda: collections.defaultdict(list))
for line in open("gpurun_out/r5_prof2/c5.err"):
    if not line.startswith("[txv pool]"):
        continue
    body = line[len("[txv pool] "):].strip()
    m = re.match(r"([a-z_ ]+?)((?: \w[\w+]*=[0-9.]+)+)$", body)
    if not m:
        continue
    for k, v in re.findall(r"(\w[\w+]*)=([0-9.]+)", m.group(2)):
        d[m.group(1).strip()][k].append(float(v))
for what, kv in d.items():
    print(what, {k: (len(v), round(statistics.median(v), 3), round(sum(v), 1)) for k, v in kv.items()})
PY
echo ALLDONE
