# C2 bench legs: tally_cross block cap 4096 (default) / 1024 / 256, twice each, alternating
set -o pipefail
O=gpurun_out/${1:-r5_cross}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-c5 --no-c1 --no-wire --no-e2e"
for rep in 1 2; do
  for cap in 4096 1024 256; do
    TXV_CROSS_BLOCKS=$cap timeout -k 10 300 $B > $O/c2_${cap}_$rep.json 2> $O/c2_${cap}_$rep.err || { echo "FAIL $cap"; tail -3 $O/c2_${cap}_$rep.err; exit 2; }
    python3 -c "import json;b=json.load(open('$O/c2_${cap}_$rep.json'));print('cap $cap rep $rep',b['value'],b['ms_per_step'],b['device_ms_p50']['verify'],b['device_ms_p50']['tally_after_verify'])"
  done
done
echo ALLDONE
