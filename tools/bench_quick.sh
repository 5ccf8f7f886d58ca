#!/bin/bash
# Quick bench lines without the slow side legs: C2 (default warm-up and --warmup 3) and the C3 shard.
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
B="--no-cpu-baseline --no-traffic --no-c5 --no-c3-job --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-put-trace"
timeout -k 10 300 python3 bench.py $B > gpurun_out/w_c2.log 2>&1 && timeout -k 10 300 python3 bench.py $B --warmup 3 > gpurun_out/w_c2_w3.log 2>&1 && timeout -k 10 400 python3 bench.py $B --config c3 > gpurun_out/w_c3.log 2>&1 || exit $?
for f in w_c2 w_c2_w3 w_c3; do python3 - gpurun_out/$f.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); c = d["config"]
        print(sys.argv[1], "value %.3e" % d["value"], "head", round(d["ms_per_step"], 4), "warm", c["warm_up"], "legs", [round(g["ms_per_step"], 4) for g in c["interleaved_legs"]], "frac", round(d["roofline"]["frac"], 3), "ins", c["insertion_order"] and round(c["insertion_order"]["ms_per_step"], 4))
PY
done
