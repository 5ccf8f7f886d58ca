#!/bin/bash
# Issue/stall picture of k_link: instruction counts and wave-state cycles (two passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-j}
O=gpurun_out
mkdir -p $O
B="bench.py --steps 2 --warmup 1 --no-parity --no-cpu-baseline"
for sk in ${SKIPS:-0}; do
  ZDL_SKIP=$sk timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_SMEM -d $O/pmc_ja_${TAG}_$sk -o run --output-format csv -- python3 $B > $O/pmc_ja_${TAG}_$sk.log 2>&1 || exit $?
  ZDL_SKIP=$sk timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU -d $O/pmc_jb_${TAG}_$sk -o run --output-format csv -- python3 $B > $O/pmc_jb_${TAG}_$sk.log 2>&1 || exit $?
  ZDL_SKIP=$sk timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE -d $O/pmc_jc_${TAG}_$sk -o run --output-format csv -- python3 $B > $O/pmc_jc_${TAG}_$sk.log 2>&1 || exit $?
done
