#!/bin/bash
# r3_probe.sh TAG: list the PMC counters this box's rocprofv3 offers (gfx950), then one default
# bench run on HEAD.  Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r3_probe}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1 || { echo LISTFAIL; tail $O/counters_list.txt; }
grep -n -i -E "VALU|WAVE_CYCLES|BUSY|WAIT" $O/counters_list.txt > $O/counters_valu.txt || true
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 3; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'],b['ms_per_step'],b['device_ms_standalone'],b['end_to_end']['registered']['votes_per_s'],b['c5_streaming']['votes_per_s'],b['c5_streaming']['p50_commit_latency_ms'],b['cpu_baseline']['value'])"
echo ALLDONE
