#!/bin/bash
# Instruction mix of k_link per ablation level (ZDL_SKIP), one rocprofv3 pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-i}
O=gpurun_out
mkdir -p $O
B="bench.py --steps 2 --warmup 1 --no-parity --no-cpu-baseline"
for sk in ${SKIPS:-0 32 64 128 256 512 2048}; do
  ZDL_SKIP=$sk timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY -d $O/pmc_ins_${TAG}_$sk -o run --output-format csv -- python3 $B > $O/pmc_ins_${TAG}_$sk.log 2>&1 || exit $?
done
