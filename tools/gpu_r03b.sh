#!/bin/bash
# r03b: full GPU suite, C5 at two giant-tier thresholds (parity), rocprof of the C5 step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${1:-r03b}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/${T}_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/${T}_tests.log; tail -5 $O/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/c5_run.py --giant-min 2048 > $O/${T}_c5_2048.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/c5_run.py --giant-min 192 > $O/${T}_c5_192.log 2>&1 || exit $?
tail -c 1500 $O/${T}_c5_2048.log; tail -c 1500 $O/${T}_c5_192.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c5_$T -o run --output-format csv -- python3 tools/c5_run.py --giant-min 192 --no-parity > $O/${T}_c5prof.log 2>&1 || exit $?

# k_link wave timing (ZDL_PROF=1: per-wave start/end stamps of the last put, printed at close)
ZDL_PROF=1 timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --inflight 1 --no-parity --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-c5 --no-traffic > $O/${T}_prof_waves.log 2>&1 || exit $?
grep "zdl prof" $O/${T}_prof_waves.log

exit 0
