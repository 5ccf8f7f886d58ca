#!/bin/bash
# Quick GPU check: parity tests (stop at first failure), the k_link ablation, one profiled run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/gpu_tests_$TAG.log; tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ablate.sh $TAG || exit $?
ZDL_PROF=1 timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-parity --no-cpu-baseline 2>&1 | grep 'zdl prof'
