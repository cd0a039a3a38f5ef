#!/bin/bash
# build_variant.sh NAME "EXTRA HIPFLAGS" — an experiment build of libtxvote.so with kernels_verify.hip
# compiled under extra defines, into build_exp/NAME/libtxvote.so (run with TXV_LIB_PATH=...)
set -e
cd "$(dirname "$0")/../../go-txflow_amd"
make -s ARCH=gfx950 >/dev/null
OUT=../build_exp/$1
mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $2 -c csrc/kernels_verify.hip -o $OUT/kernels_verify.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o $OUT/libtxvote.so $OUT/kernels_verify.o $(ls build/*.o | grep -v kernels_verify)
rm $OUT/kernels_verify.o
echo built $OUT/libtxvote.so
