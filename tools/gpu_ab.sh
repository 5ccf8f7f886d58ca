#!/bin/bash
# GPU session: parity tests, then bench with the wave kernel and the block kernel (A/B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/gpu_tests.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_wave.log 2>&1 || exit $?
ZDL_KERNEL=block timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/bench_block.log 2>&1
