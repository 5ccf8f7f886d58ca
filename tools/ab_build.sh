#!/bin/bash
# A/B builds of libzdl with -D overrides: tools/ab_build.sh NAME "-DLK_DEPTH=2 -DLK_WAVES=14" ...
# (pairs of arguments); each lands in ab/NAME/libzdl.so (ZDL_LIB_PATH selects it).
cd "$(dirname "$0")/.."
C=zipkin_amd/csrc
while [ $# -ge 2 ]; do
  n=$1; d=$2; shift 2
  mkdir -p ab/$n
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -w $d $C/zdl.hip $C/zdl_group.hip $C/zdl_sparse.hip $C/zdl_proto3.hip $C/zdl_rows.hip $C/zdl_store.hip -o ab/$n/libzdl.so -L/opt/rocm/lib -lrccl -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib &
done
wait
