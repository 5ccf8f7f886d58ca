#!/bin/bash
# One GPU check: the whole -m gpu suite, smoke(), then the default bench line.
#   tools/gpu_check.sh TAG [nobench]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-chk}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests_$TAG.log; tail -3 $O/gpu_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$TAG.log 2>&1 || exit $?
[ "$2" = "nobench" ] && exit 0
timeout -k 10 400 python -u bench.py > $O/bench_$TAG.log 2>&1 || exit $?
grep -v '^{' $O/bench_$TAG.log | tail -12
