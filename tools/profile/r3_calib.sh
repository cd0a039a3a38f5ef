#!/bin/bash
# r3_calib.sh TAG: FETCH_SIZE / WRITE_SIZE of the tally's access shapes (tools/microbench/tally_calib),
# one --pmc pass per counter, never with traces
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_calib}
mkdir -p $O
timeout -k 10 60 tools/microbench/tally_calib > $O/calib.json 2> $O/calib.err || { echo RUNFAIL; cat $O/calib.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_f -o pmc --output-format csv -- tools/microbench/tally_calib > /dev/null 2> $O/pmc_f.err || { echo PMCF; exit 2; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_w -o pmc --output-format csv -- tools/microbench/tally_calib > /dev/null 2> $O/pmc_w.err || { echo PMCW; exit 3; }
timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- tools/microbench/tally_calib > /dev/null 2> $O/kt.err || { echo KT; exit 4; }
cat $O/calib.json
echo ALLDONE
