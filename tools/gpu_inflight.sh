#!/bin/bash
# C2 step with 1-4 puts in flight (distinct input copies), twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
B="bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-h2d --no-c5 --no-traffic --no-put-trace --no-parity"
for rep in 1 2; do for k in 2 3 4; do
  timeout -k 10 120 python -u $B --inflight $k > $O/infl_$k.log 2>&1 || exit $?
  echo "inflight $k $(tail -1 $O/infl_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["config"]["kernel_ms"]["k_link"])')"
done; done
