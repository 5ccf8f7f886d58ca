#!/bin/bash
# C2 bench line at several puts in flight and k_link timing strides (value, ms/step, roofline
# fraction):  INFL="1 2 3" STRIDES="1 8" tools/gpu_inflight.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="--steps 20 --warmup 3 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity"
for s in ${STRIDES:-8}; do
  for f in ${INFL:-1 2 3 4}; do
    timeout -k 10 120 python -u bench.py $B --inflight $f --timing-stride $s > gpurun_out/infl_${f}_$s.log 2>&1 || exit $?
    echo "inflight $f stride $s $(tail -1 gpurun_out/infl_${f}_$s.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')"
  done
done
