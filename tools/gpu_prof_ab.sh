#!/bin/bash
# Per-kernel durations of every A/B variant in ab/*/ (tools/ab_build.sh), one step at a time
# (--inflight 1: a kernel's duration is its own, not time spent queued behind the other step's):
#   tools/gpu_prof_ab.sh c2|c3 TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
CFG=${1:-c3}; TAG=${2:-pab}
B="bench.py --config $CFG --steps 10 --warmup 3 --inflight 1 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity --no-c5 --no-traffic --no-put-trace"
for d in ab/*/; do
  v=$(basename $d)
  ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/${TAG}_$v -o run --output-format csv -- python3 $B > $O/${TAG}_$v.log 2>&1 || exit $?
  echo "== $v"; python3 tools/kstats.py $(find $O/${TAG}_$v -name 'run_kernel_stats.csv' | head -1) | head -16
done
exit 0
