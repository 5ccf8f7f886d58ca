#!/bin/bash
# r03c: giant-tier tests, C5 at two thresholds (parity), rocprof of the C5 step, C2 k_link wave timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${1:-r03c}
timeout -k 10 600 python -u -m pytest tests/test_gpu_giant.py tests/test_gpu_tree_stream.py tests/test_gpu_scale.py -k "giant or c5 or sparse or mid_size or stream" -x -q --timeout 400 --timeout-method thread > $O/${T}_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/${T}_tests.log; tail -3 $O/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/c5_run.py --giant-min 2048 > $O/${T}_c5_2048.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/c5_run.py --giant-min 192 > $O/${T}_c5_192.log 2>&1 || exit $?
tail -c 1300 $O/${T}_c5_2048.log; tail -c 1300 $O/${T}_c5_192.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c5_$T -o run --output-format csv -- python3 tools/c5_run.py --giant-min 2048 --no-parity > $O/${T}_c5prof.log 2>&1 || exit $?
ZDL_PROF=1 timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --inflight 1 --no-parity --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-c5 --no-traffic > $O/${T}_prof_waves.log 2>&1 || exit $?
grep "zdl prof" $O/${T}_prof_waves.log
exit 0
