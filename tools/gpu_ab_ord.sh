#!/bin/bash
# Insertion-order A/B: the bench insertion_order leg for every ab/*/libzdl.so (tools/ab_build.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for d in ab/*/; do
  n=$(basename $d)
  ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-parity --no-c5 --no-put-trace > $O/abo_$n.log 2>&1 || exit $?
  echo "$n $(tail -1 $O/abo_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["insertion_order"])')"
done
