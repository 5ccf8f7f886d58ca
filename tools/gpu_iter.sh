#!/bin/bash
# One optimisation iteration: GPU parity tests, then a short bench (k_link time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-it}
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/gpu_tests_$TAG.log; tail -2 gpurun_out/gpu_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-insertion-order > gpurun_out/bench_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("k_link ms", d["config"]["kernel_ms"]["k_link"], "step ms", d["ms_per_step"], "parity", d["config"]["parity"], "frac", d["roofline"]["frac"])'
