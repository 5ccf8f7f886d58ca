#!/bin/bash
# One GPU session: parity tests, smoke, the bench line (with CPU baseline), then
# rocprofv3 kernel-trace stats and separate FETCH_SIZE / WRITE_SIZE passes.
# Every GPU step has its own time limit and the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}
O=gpurun_out
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench_$TAG.log 2>&1 || exit $?
B="bench.py --steps 10 --warmup 2 --no-parity --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- python3 $B > $O/prof_${TAG}_bench.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$TAG -o run --output-format csv -- python3 $B > $O/pmc_fetch_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$TAG -o run --output-format csv -- python3 $B > $O/pmc_write_$TAG.log 2>&1 || exit $?
exit 0
