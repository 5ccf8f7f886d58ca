#!/bin/bash
# k_link A/B: the serial C2 bench line for every ab/*/libzdl.so (tools/ab_build.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
CFG=${CFG:-c2}
for d in ab/*/; do
  n=$(basename $d)
  ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 120 python -u bench.py --config $CFG --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity > $O/ab_${CFG}_$n.log 2>&1 || exit $?
  echo "$n $(tail -1 $O/ab_${CFG}_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["kernel_ms"], d["ms_per_step"])')"
done
