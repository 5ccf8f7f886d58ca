#!/bin/bash
# Kernel timeline of the insertion-order side leg (two contexts in flight) at C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
B="bench.py --steps 20 --warmup 3 --warm-ms 0 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-parity --no-c5 --no-traffic --no-put-trace --no-c3-job"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ordtl -o run --output-format csv -- python3 $B > $O/ordtl_bench.log 2>&1 || exit $?
f=$(find $O/ordtl -name '*kernel_trace.csv' | head -1); d=$(dirname $f)
python3 tools/timeline.py $d --min-us 0 --marker "k_link<1, 0, 6>" --from 12 --to 16 > $O/ordtl_timeline.txt 2>&1
exit 0
