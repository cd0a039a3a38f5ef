#!/bin/bash
# build_variant_all.sh NAME "EXTRA HIPFLAGS": every object of libtxvote.so compiled with the extra
# defines, into build_exp/NAME/libtxvote.so (run with TXV_LIB_PATH=...)
set -e
cd "$(dirname "$0")/../../go-txflow_amd"
OUT=../build_exp/$1
mkdir -p $OUT
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $2"
for k in kernels_verify kernels_flow kernels_pool kernels_signbytes kernels_wire; do
  /opt/rocm/bin/hipcc $F -c csrc/$k.hip -o $OUT/$k.o &
done
/opt/rocm/bin/hipcc $F -x hip -c csrc/runtime.cpp -o $OUT/runtime.o &
/opt/rocm/bin/hipcc $F -x hip -c csrc/pool.cpp -o $OUT/pool.o &
wait
/opt/rocm/bin/hipcc $F -shared -o $OUT/libtxvote.so $OUT/*.o
rm $OUT/*.o
echo built $OUT/libtxvote.so
