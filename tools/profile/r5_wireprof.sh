# host-side phase times of the C5 wire leg (TXV_PROFILE_HOST) and its kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_wireprof}
mkdir -p $O
TXV_PROFILE_HOST=1 timeout -k 10 400 python3 bench.py --c5-only > $O/c5.json 2> $O/c5.err || { echo "C5FAIL"; tail -5 $O/c5.err; exit 2; }
python3 -c "
import json;b=json.load(open('$O/c5.json'));w=b['c5_wire'];print('wire', w['votes_per_s'], w['p50_admit_ms'], w['p50_decode_ms'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --c5-only > $O/c5_kt.json 2> $O/c5_kt.err || { echo KTFAIL; exit 3; }
echo ALLDONE
