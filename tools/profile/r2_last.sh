#!/bin/bash
# r2_last.sh: bench depth A/B, then the final -m gpu suite, smoke, default bench and kernel trace
set -o pipefail
export TMPDIR=/tmp
bash tools/profile/env_ab.sh r2_depth "TXV_BENCH_DEPTH=3" "TXV_BENCH_DEPTH=4" "TXV_BENCH_DEPTH=2" "TXV_BENCH_DEPTH=4" "TXV_BENCH_DEPTH=3" || exit 1
bash tools/profile/r2_final2.sh r2_last || exit 2
