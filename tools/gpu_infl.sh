#!/bin/bash
# C2 headline only, steps in flight 2 vs 3 (alternating, twice)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
B="bench.py --steps 60 --warmup 5 --no-parity --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-h2d --no-c5 --no-traffic --no-cpu-baseline"
for i in 2 3 2 3; do
  timeout -k 10 200 python -u $B --inflight $i > $O/infl_$i.log 2>&1 || exit $?
  tail -1 $O/infl_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("inflight '$i'", d["ms_per_step"]*1e3, d["value"], d["config"]["step_roofline_frac"])' | tee -a $O/infl_sum.log
done
exit 0
