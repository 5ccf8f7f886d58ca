#!/bin/bash
# k_link issue-priority A/B (tools/ab_build.sh base/prio/waves/prio_w): C2 kernel time of each
# production variant (inflight 1 and 2), and the per-wave finish distribution (ZDL_PROF=1) of
# the stamp-only variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity --no-c5 --no-traffic"
for v in base prio base prio; do
  ZDL_LIB_PATH=$PWD/ab/$v/libzdl.so timeout -k 10 120 python -u $B --inflight 1 > $O/abp_$v.log 2>&1 || exit $?
  echo "$v inflight1 $(tail -1 $O/abp_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["kernel_ms"], d["ms_per_step"])')"
  ZDL_LIB_PATH=$PWD/ab/$v/libzdl.so timeout -k 10 120 python -u $B > $O/abp2_$v.log 2>&1 || exit $?
  echo "$v inflight2 $(tail -1 $O/abp2_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["kernel_ms"], d["ms_per_step"])')"
done
for v in waves prio_w; do
  ZDL_PROF=1 ZDL_LIB_PATH=$PWD/ab/$v/libzdl.so timeout -k 10 120 python -u $B --inflight 1 --steps 3 > $O/abw_$v.log 2>&1 || exit $?
  echo "$v $(grep 'k_link waves' $O/abw_$v.log)"
done
for v in base prio; do
  ZDL_LIB_PATH=$PWD/ab/$v/libzdl.so timeout -k 10 200 python -u $B --config c3 --inflight 1 --steps 10 > $O/abp3_$v.log 2>&1 || exit $?
  echo "$v c3 $(tail -1 $O/abp3_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["kernel_ms"], d["ms_per_step"])')"
done
exit 0
