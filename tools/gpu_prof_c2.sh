#!/bin/bash
# rocprofv3 kernel-trace stats and the FETCH_SIZE / WRITE_SIZE passes of the C2 headline put
# alone (the bench line's serial steps; no side legs), for tools/prof_summary.py TAG.
#   tools/gpu_prof_c2.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-c2}
O=gpurun_out; mkdir -p $O
B="bench.py --steps 10 --warmup 2 --inflight 1 --no-parity --no-cpu-baseline --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-h2d --no-c5 --no-traffic --no-put-trace"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- python3 $B > $O/prof_${TAG}_bench.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$TAG -o run --output-format csv -- python3 $B > $O/pmc_fetch_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$TAG -o run --output-format csv -- python3 $B > $O/pmc_write_$TAG.log 2>&1 || exit $?
tail -1 $O/prof_${TAG}_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench under rocprof:", d["ms_per_step"], d["config"]["kernel_ms"]["k_link"])'
