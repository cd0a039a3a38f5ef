#!/bin/bash
# build_variant_flow.sh NAME "EXTRA HIPFLAGS" — an experiment build of libtxvote.so with
# kernels_flow.hip compiled under extra defines, into build_exp/NAME/libtxvote.so
set -e
cd "$(dirname "$0")/../../go-txflow_amd"
make -s ARCH=gfx950 >/dev/null
OUT=../build_exp/$1
mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $2 -c csrc/kernels_flow.hip -o $OUT/kernels_flow.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o $OUT/libtxvote.so $OUT/kernels_flow.o $(ls build/*.o | grep -v kernels_flow)
rm $OUT/kernels_flow.o
echo built $OUT/libtxvote.so
