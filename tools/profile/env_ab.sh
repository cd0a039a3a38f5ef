#!/bin/bash
# env_ab.sh TAG "ENV1" "ENV2" ...: bench.py's C2 leg once per environment setting (same box)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 240 python3 -u bench.py --steps 20 --warmup 3 --no-c5 --no-c1 --no-wire --no-cpu-baseline --no-e2e \
    > gpurun_out/$TAG/v$i.json 2> gpurun_out/$TAG/v$i.err || { echo "FAIL $e"; tail -5 gpurun_out/$TAG/v$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,1), 'M/s', d['device_ms_p50']['verify'], d['device_ms_standalone'])" gpurun_out/$TAG/v$i.json "$e"
done
