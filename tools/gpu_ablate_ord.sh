#!/bin/bash
# Timing-only ablation of the insertion-order path (k_tail ORD): 8192 no BFS ranks, 16384 no ord_min.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for sk in 0 8192 16384 24576; do
  ZDL_SKIP=$sk timeout -k 10 100 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/ablord_$sk.log 2>&1 || exit $?
  echo "$sk $(grep -o '"insertion_order": {"ms_per_step": [0-9.]*' gpurun_out/ablord_$sk.log)"
done
