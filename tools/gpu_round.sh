#!/bin/bash
# The round's record on one box: the -m gpu suite, smoke(), the default bench line, the C3 shard
# bench (with parity) and a rocprofv3 kernel-stats run of the C2 headline.
#   tools/gpu_round.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06}
O=gpurun_out; mkdir -p $O
bash tools/gpu_check.sh $TAG || exit $?
timeout -k 10 400 python -u bench.py --config c3 > $O/bench_c3_$TAG.log 2>&1 || exit $?
grep -v '^{' $O/bench_c3_$TAG.log | tail -4
B="bench.py --steps 20 --warmup 5 --inflight 1 --no-parity --no-cpu-baseline --no-traffic --no-c5 --no-c3-job --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-put-trace --no-insertion-order"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kst_c2_$TAG -o run --output-format csv -- python3 $B > $O/kst_c2_$TAG.log 2>&1 || exit $?
exit 0
