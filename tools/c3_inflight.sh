#!/bin/bash
# C3 shard step at 1..4 steps in flight (bench.py --config c3 --inflight N), one GPU call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
B="bench.py --config c3 --no-c3-job --steps 16 --warmup 3 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity --no-c5 --no-traffic --no-put-trace"
for n in ${*:-2 3 4 2}; do
  timeout -k 10 200 python -u $B --inflight $n > $O/c3inf_$n.log 2>&1 || exit $?
  tail -1 $O/c3inf_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("inflight", c["inflight"], "step", round(d["ms_per_step"],4), "legs", [round(g["ms_per_step"],4) for g in c["interleaved_legs"] or []], "k_link", round(c["kernel_ms"]["k_link"],4))'
done
exit 0
