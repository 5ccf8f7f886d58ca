#!/bin/bash
# r03m: the default bench line (all legs, live PMC traffic), then C2 at 2 / 3 / 4 puts in flight
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-r03m}
timeout -k 10 400 python -u bench.py > $O/bench_$T.log 2>&1 || exit $?
tail -1 $O/bench_$T.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("C2", d["value"], d["ms_per_step"], c["ms_per_step_serial"], c["step_roofline_frac"], d["roofline"]["frac"], d["roofline"]["traffic"]); print("C5", c["c5"]["ms_per_step"], c["c5"]["parity"])'
B="bench.py --steps 40 --warmup 5 --no-parity --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-c5 --no-traffic"
for n in 2 3 4 2 3 4; do
  timeout -k 10 120 python -u $B --inflight $n > $O/infl_$T.log 2>&1 || exit $?
  tail -1 $O/infl_$T.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("inflight '$n'", round(d["ms_per_step"]*1e3,1), d["value"])'
done
exit 0
