#!/bin/bash
# rocprofv3 session: kernel-trace stats + separate PMC passes over a short bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
B="bench.py --steps 10 --warmup 2 --no-parity --no-cpu-baseline --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 $B > gpurun_out/prof_${TAG}_bench.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-parity --no-cpu-baseline --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order > gpurun_out/pmc_fetch_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-parity --no-cpu-baseline --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order > gpurun_out/pmc_write_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_sq_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-parity --no-cpu-baseline --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order > gpurun_out/pmc_sq_$TAG.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq2_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-parity --no-cpu-baseline --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order > gpurun_out/pmc_sq2_$TAG.log 2>&1
exit 0
