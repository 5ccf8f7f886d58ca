#!/bin/bash
# Quick GPU check: the whole -m gpu suite, then a serial C2 bench line (k_link HIP events).
#   tools/gpu_quick.sh TAG [extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-q}; shift
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests_$TAG.log; tail -3 $O/gpu_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order "$@" > $O/bench_$TAG.log 2>&1 || exit $?
tail -1 $O/bench_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["kernel_ms"], d["roofline"]["frac"], d["config"]["parity"])'
