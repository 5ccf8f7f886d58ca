#!/bin/bash
# A/B builds of libzdl with -D overrides: tools/ab_build.sh NAME "-DLK_DEPTH=2 -DLK_WAVES=14" ...
# (pairs of arguments); each lands in ab/NAME/libzdl.so (ZDL_LIB_PATH selects it). One object per
# source, compiled in parallel (as __graft_entry__.build does), then one link per variant.
cd "$(dirname "$0")/.."
C=${ZDL_AB_SRC:-zipkin_amd/csrc}
SRCS="zdl zdl_group zdl_sparse zdl_proto3 zdl_rows zdl_store"
while [ $# -ge 2 ]; do
  n=$1; d=$2; shift 2
  mkdir -p ab/$n/obj
  (
    for s in $SRCS; do
      hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -w $d -c $C/$s.hip -o ab/$n/obj/$s.o &
    done
    wait
    hipcc --offload-arch=gfx950 -shared ab/$n/obj/*.o -o ab/$n/libzdl.so -L/opt/rocm/lib -lrccl -lhsa-runtime64 \
      -Wl,-rpath,/opt/rocm/lib && rm -rf ab/$n/obj
  ) &
done
wait
