#!/bin/bash
# r03d: the whole GPU suite; C2 with the lazy tail vs ZDL_NOLAZY=1 (serial and two in flight)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${1:-r03d}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/${T}_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/${T}_tests.log; tail -3 $O/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-c5 --no-traffic"
j() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["config"]["kernel_ms"]["k_link"]*1e3,1), round(d["ms_per_step"]*1e3,1), d["config"]["parity"])'; }
for rep in 1 2; do
  timeout -k 10 120 python -u $B --inflight 1 > $O/${T}_l1.log 2>&1 || exit $?
  timeout -k 10 120 python -u $B > $O/${T}_l2.log 2>&1 || exit $?
  ZDL_NOLAZY=1 timeout -k 10 120 python -u $B --inflight 1 > $O/${T}_n1.log 2>&1 || exit $?
  ZDL_NOLAZY=1 timeout -k 10 120 python -u $B > $O/${T}_n2.log 2>&1 || exit $?
  echo "lazy serial $(j $O/${T}_l1.log) inflight2 $(j $O/${T}_l2.log) | nolazy serial $(j $O/${T}_n1.log) inflight2 $(j $O/${T}_n2.log)"
done
for n in 3 4; do
  timeout -k 10 120 python -u $B --inflight $n > $O/${T}_l$n.log 2>&1 || exit $?
  echo "lazy inflight$n $(j $O/${T}_l$n.log)"
done
exit 0
