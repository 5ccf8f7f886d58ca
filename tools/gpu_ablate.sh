#!/bin/bash
# Timing-only ablation of k_wave phases (results are wrong by design under ZDL_SKIP).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sk in 0 16 1 2 4 8 32 64 127; do
  ZDL_SKIP=$sk timeout -k 10 100 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/abl_$sk.log 2>&1 || exit $?
done
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_sq_w -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-parity --no-cpu-baseline > gpurun_out/pmc_sq_w.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq2_w -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-parity --no-cpu-baseline > gpurun_out/pmc_sq2_w.log 2>&1
exit 0
