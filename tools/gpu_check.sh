#!/bin/bash
# GPU session script: gpu tests, smoke, short bench (each step time-limited).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -v --maxfail=30 --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/gpu_tests.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
