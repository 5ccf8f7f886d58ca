#!/bin/bash
# C2 headline step at 1, 2, 3 and 4 steps in flight (bench.py --inflight N), side legs off, one GPU call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="bench.py --steps 40 --no-cpu-baseline --no-traffic --no-c5 --no-c3-job --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-put-trace --no-insertion-order"
for r in 1 2; do for n in 2 3 4; do
  timeout -k 10 300 python3 $B --inflight $n > gpurun_out/infl_${n}_$r.log 2>&1 || exit $?
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('inflight', sys.argv[2], round(d['ms_per_step'],4), [round(g['ms_per_step'],4) for g in d['config']['interleaved_legs']])" gpurun_out/infl_${n}_$r.log $n
done; done
