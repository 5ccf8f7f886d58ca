#!/bin/bash
# C5 leg: one host thread per context vs one thread alternating both (A/B, parity on)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-c5t}
B="bench.py --steps 3 --warmup 1 --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-h2d --no-traffic --no-cpu-baseline"
for h in 2 1 2; do
  timeout -k 10 300 python -u $B --c5-host-threads $h > $O/c5t_${T}_$h.log 2>&1 || exit $?
  tail -1 $O/c5t_${T}_$h.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]["c5"]; print("host threads '$h'", c["ms_per_step"], c["ms_per_step_serial"], c["parity"])'
done
exit 0
