#!/bin/bash
# C3 A/B over ab/*/libzdl.so (tools/ab_build.sh): k_link and step, serial and two in flight, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
B="bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity --no-c5 --no-traffic --no-put-trace"
j() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["config"]["kernel_ms"]; print(round(k["k_link"]*1e3,1), round(d["ms_per_step"]*1e3,1))'; }
for rep in 1 2 3; do
for d in ab/*/; do
  v=$(basename $d)
  ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 200 python -u $B --inflight 1 > $O/ab3s_$v.log 2>&1 || exit $?
  ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 200 python -u $B > $O/ab3i_$v.log 2>&1 || exit $?
  echo "$v c3 serial(us k_link, step) $(j $O/ab3s_$v.log)  inflight2 $(j $O/ab3i_$v.log)"
done
done
exit 0
