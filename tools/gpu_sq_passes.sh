#!/bin/bash
# SQ counter passes over a short bench run (k_link issue / wait breakdown). One pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-sq}
B="bench.py --steps 2 --warmup 1 --no-parity --no-cpu-baseline --no-insertion-order"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM -d gpurun_out/pmc_sqa_$TAG -o run --output-format csv -- python3 $B > gpurun_out/pmc_sqa_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE -d gpurun_out/pmc_sqb_$TAG -o run --output-format csv -- python3 $B > gpurun_out/pmc_sqb_$TAG.log 2>&1 || exit $?
