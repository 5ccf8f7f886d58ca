#!/bin/bash
# k_link A/B over ab/*/libzdl.so (tools/ab_build.sh): C2 k_link time and step (inflight 1 and 2)
# for every variant whose name does not start with "w"; per-wave finish distribution
# (ZDL_PROF=1, build with -DLK_PROF_PHASES=0) for the "w*" ones; C3 for the variants in $C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity --no-c5 --no-traffic"
j() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["config"]["kernel_ms"]["k_link"]*1e3,1), round(d["ms_per_step"]*1e3,1))'; }
for rep in 1 2; do
for d in ab/*/; do
  v=$(basename $d); case $v in w*) continue;; esac
  ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 120 python -u $B --inflight 1 > $O/abk1_$v.log 2>&1 || exit $?
  ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 120 python -u $B > $O/abk2_$v.log 2>&1 || exit $?
  echo "$v serial(us k_link, step) $(j $O/abk1_$v.log)  inflight2 $(j $O/abk2_$v.log)"
done
done
for d in $(ls -d ab/w*/ 2>/dev/null); do
  v=$(basename $d)
  ZDL_PROF=1 ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 120 python -u $B --inflight 1 --steps 3 > $O/abkw_$v.log 2>&1 || exit $?
  echo "$v $(grep 'k_link waves' $O/abkw_$v.log)"
done
for v in $C3; do
  ZDL_LIB_PATH=$PWD/ab/$v/libzdl.so timeout -k 10 200 python -u $B --config c3 --inflight 1 --steps 10 > $O/abk3_$v.log 2>&1 || exit $?
  echo "$v c3 serial $(j $O/abk3_$v.log)"
done
exit 0
