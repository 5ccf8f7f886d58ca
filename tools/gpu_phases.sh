#!/bin/bash
# k_link's cycle stamps per phase (ZDL_PROF=1: the PROF == 1 instantiation) at C2, serial, for
# this tree's libzdl and every ab/*/libzdl.so: phase 0 = plan + load issue, 3..11 = lk_window's
# steps, 2 = the rest of the iteration (the wait for the next window's loads).
#   tools/gpu_phases.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
TAG=${1:-ph}
B="bench.py --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity --no-c5 --no-traffic --no-put-trace"
for d in zipkin_amd ab/*; do
  v=$(basename $d)
  ZDL_PROF=1 ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 120 python -u $B > $O/ph_${TAG}_$v.log 2>&1 || exit $?
  echo "$v: $(grep -h 'zdl prof' $O/ph_${TAG}_$v.log | tail -2 | tr '\n' ' ')"
done
