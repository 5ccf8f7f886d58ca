#!/bin/bash
# Insertion-order leg at C2 for each libzdl variant in ab/*/ (tools/ab_build.sh), alternating, one GPU call.
#   tools/ord_ab.sh [ROUNDS]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="bench.py --steps 20 --no-cpu-baseline --no-traffic --no-c5 --no-c3-job --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-put-trace"
for r in $(seq ${1:-2}); do
  for d in ab/*/; do
    v=$(basename $d)
    ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 300 python3 $B > gpurun_out/ord_ab_${v}_$r.log 2>&1 || exit $?
    python3 - gpurun_out/ord_ab_${v}_$r.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); o = d["config"]["insertion_order"]
        print(sys.argv[2], "inflight", round(o["ms_per_step"], 4), "serial", round(o["ms_per_step_serial"], 4), o["parity"], "| c2", round(d["ms_per_step"], 4))
PY
  done
done
