set -o pipefail
bash tools/profile/env_ab.sh r2_envab "TXV_NONE=0" "TXV_VSTREAM_PRIO=1" "TXV_FLOW_CUS=64" "TXV_FLOW_CUS=128" "TXV_FLOW_CUS=32" || exit 1
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c1 --no-wire --no-e2e --steps 10 > gpurun_out/r2_envab/c5.json 2> gpurun_out/r2_envab/c5.err || { echo C5FAIL; tail gpurun_out/r2_envab/c5.err; exit 2; }
python3 -c "import json;b=json.load(open('gpurun_out/r2_envab/c5.json'));print(b['c5_streaming'])"
