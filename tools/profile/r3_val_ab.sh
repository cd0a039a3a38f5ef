#!/bin/bash
# r3_val_ab.sh TAG VARIANTS...: the whole validation + profile pass of r3_final.sh on the in-tree
# build, then bench.py's device-resident leg per experiment build (ab.sh), same box
set -o pipefail
bash tools/profile/r3_final.sh "$1" || exit $?
TAG=$1; shift
bash tools/profile/ab.sh "${TAG}_ab" "$@"
