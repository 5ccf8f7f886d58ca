#!/bin/bash
# C2 headline against the warm-up length (--warmup W steps, no time floor): profiles/r06i_warm_probe.txt
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
B="bench.py --steps 20 --no-cpu-baseline --no-traffic --no-c5 --no-c3-job --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-put-trace --no-insertion-order"
for w in 20 500 2000 20; do
  timeout -k 10 300 python3 $B --warmup $w --warm-ms 0 > gpurun_out/warm_$w.log 2>&1 || exit $?
  python3 - gpurun_out/warm_$w.log $w <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); c = d["config"]
        print("warmup", sys.argv[2], "head", round(d["ms_per_step"], 4), "legs", [round(g["ms_per_step"], 4) for g in c["interleaved_legs"]], "serial", round(c["ms_per_step_serial"], 4), "k_link", round(c["kernel_ms"]["k_link"], 4))
PY
done
