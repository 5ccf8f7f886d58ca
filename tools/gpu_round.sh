#!/bin/bash
# One GPU session: parity tests, smoke, the C2 bench line (with CPU baseline), the C3
# per-GPU-shard line, rocprofv3 kernel-trace stats of both, separate FETCH_SIZE /
# WRITE_SIZE passes on C2 and the FETCH_SIZE calibration for 4/8/16-B lanes.
# Every GPU step has its own time limit and the chain stops at the first failure.
#   tools/gpu_round.sh TAG [quick]   (quick: tests + smoke + C2 bench only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r02}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench_$TAG.log 2>&1 || exit $?
[ "$2" = "quick" ] && exit 0
timeout -k 10 300 python -u bench.py --config c3 > $O/bench_c3_$TAG.log 2>&1 || exit $?
B="bench.py --steps 10 --warmup 2 --inflight 1 --no-parity --no-cpu-baseline --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-h2d --no-c5 --no-traffic --no-put-trace"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- python3 $B > $O/prof_${TAG}_bench.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c3_$TAG -o run --output-format csv -- python3 $B --config c3 > $O/prof_c3_${TAG}_bench.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$TAG -o run --output-format csv -- python3 $B > $O/pmc_fetch_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$TAG -o run --output-format csv -- python3 $B > $O/pmc_write_$TAG.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/calib_$TAG -o run --output-format csv -- tools/calib_fetch > $O/calib_$TAG.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_json_$TAG -o run --output-format csv -- python3 tools/json_decode_run.py > $O/prof_json_${TAG}.log 2>&1 || exit $?
exit 0
