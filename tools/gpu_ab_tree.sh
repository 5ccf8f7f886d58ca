#!/bin/bash
# A/B of the default bench's C2 legs between this tree and an older tree extracted under abx/NAME
# (built there beforehand): the same flags in both, results in gpurun_out/ab_<NAME>_*.log.
#   tools/gpu_ab_tree.sh NAME [extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
N=$1; shift
O=$PWD/gpurun_out; mkdir -p $O
B="bench.py --steps 20 --warmup 3 --no-proto3 --no-json --no-store --no-mysql-rows --no-h2d --no-c5 --no-traffic --no-cpu-baseline $*"
for rep in 1 2; do
  (cd abx/$N && timeout -k 10 200 python -u $B > $O/ab_${N}_old_$rep.log 2>&1) || exit $?
  timeout -k 10 200 python -u $B --no-put-trace > $O/ab_${N}_new_$rep.log 2>&1 || exit $?
done
for f in $O/ab_${N}_*.log; do
  echo "$(basename $f) $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["ms_per_step"], c.get("ms_per_step_serial"), c["kernel_ms"], (c["insertion_order"] or {}).get("ms_per_step"))')"
done
