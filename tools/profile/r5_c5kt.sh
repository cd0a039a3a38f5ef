# kernel trace of the C5 legs (SoA with Update, wire) on the last tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_c5kt}
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --c5-only > $O/c5_kt.json 2> $O/c5_kt.err || { echo KTFAIL; tail -5 $O/c5_kt.err; exit 3; }
python3 -c "
import json;b=json.load(open('$O/c5_kt.json'));c=b['c5_streaming'];w=b['c5_wire'];print('c5',c['votes_per_s'],c['correct'],c['pool_matches_oracle'],'wire',w['votes_per_s'],w['correct'])"
echo ALLDONE
