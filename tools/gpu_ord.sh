#!/bin/bash
# Insertion-order check: parity tests, the bench insertion_order leg, kernel stats.  tools/gpu_ord.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_insertion_order.py tests/test_gpu_store.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${1:-ord}.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-proto3 --no-json --no-store --no-mysql-rows --no-h2d > gpurun_out/${1:-ord}_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${1:-ord} -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-parity --no-cpu-baseline --no-proto3 --no-json --no-store --no-mysql-rows --no-h2d > gpurun_out/prof_${1:-ord}.log 2>&1
