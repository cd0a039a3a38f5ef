#!/bin/bash
# same-box A/B of the base-point window: radix-2^24 (11.8 GB, default) vs radix-2^26 (43 GB, one
# addition fewer per vote) through bench.py's C2 leg, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_wb}
mkdir -p $O
for rep in 1 2; do
  for bw in 24 26; do
    timeout -k 10 240 python3 -u bench.py --steps 20 --warmup 3 --base-w $bw --no-c5 --no-c1 --no-wire --no-cpu-baseline --no-e2e \
      > $O/bw${bw}_$rep.json 2> $O/bw${bw}_$rep.err || { echo "FAIL $bw"; tail -5 $O/bw${bw}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,1), 'M/s', d['ms_per_step'], d['device_ms_p50']['verify'], d['device_ms_standalone']['verify'])" $O/bw${bw}_$rep.json bw$bw
  done
done
