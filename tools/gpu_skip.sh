#!/bin/bash
# k_link ablations at C2 (ZDL_SKIP, the PROF == 2 instantiation; 1 = no effect): serial k_link
# time (HIP events) and the in-flight step, one bench run per value.
#   SKIPS="1 32 64 4096 8192" tools/gpu_skip.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity --no-c5 --no-traffic --no-put-trace"
for sk in ${SKIPS:-1 32 64 4096 8192}; do
  ZDL_SKIP=$sk timeout -k 10 120 python -u $B > $O/skip_$sk.log 2>&1 || exit $?
  echo "skip $sk: $(tail -1 $O/skip_$sk.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("k_link us", round(c["kernel_ms"]["k_link"]*1e3,1), "step us", round(d["ms_per_step"]*1e3,1))')"
done
