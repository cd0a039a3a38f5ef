#!/bin/bash
# ab.sh TAG V1 V2 ... — bench.py's device-resident leg for each experiment build (build_exp/V or
# "cur" = the in-tree build), one after the other on the same box; one JSON line per variant
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for v in "$@"; do
  if [ "$v" = cur ]; then unset TXV_LIB_PATH; else export TXV_LIB_PATH=$PWD/build_exp/$v/libtxvote.so; fi
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-c5 --no-c1 --no-wire --no-cpu-baseline --no-e2e \
    > gpurun_out/$TAG/$v.json 2> gpurun_out/$TAG/$v.err || { echo "FAIL $v"; tail -5 gpurun_out/$TAG/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,1), 'M/s', d['device_ms_p50'])" gpurun_out/$TAG/$v.json $v
done
