#!/bin/bash
# Timing-only ablation of k_link phases (results are wrong by design under ZDL_SKIP).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-x}
for sk in ${SKIPS:-0 32 64 128 256 512 2048}; do
  ZDL_SKIP=$sk timeout -k 10 100 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/abl_${TAG}_$sk.log 2>&1 || exit $?
done
for sk in ${SKIPS:-0 32 64 128 256 512 2048}; do echo "$sk $(tail -1 gpurun_out/abl_${TAG}_$sk.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["kernel_ms"])')"; done
