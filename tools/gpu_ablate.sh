#!/bin/bash
# Timing-only ablation of k_link phases (results are wrong by design under ZDL_SKIP).
#   SKIPS="0 32 4096 4128" tools/gpu_ablate.sh TAG
# 32: no lk_window (the stream alone); 4096: every window re-reads the chunk's first 128
# positions (cache-resident: compute without HBM stalls); 64/128/256/512/2048: cut after a phase.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-x}
B="bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline --no-parity --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order"
for sk in ${SKIPS:-0 32 64 128 256 512 2048}; do
  ZDL_SKIP=$sk timeout -k 10 100 python -u $B > gpurun_out/abl_${TAG}_$sk.log 2>&1 || exit $?
done
for sk in ${SKIPS:-0 32 64 128 256 512 2048}; do echo "$sk $(tail -1 gpurun_out/abl_${TAG}_$sk.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["kernel_ms"], d["ms_per_step"])')"; done
