#!/bin/bash
# C2 A/B: the lazy tail vs ZDL_NOLAZY=1, serial and two puts in flight (k_link by HIP events, step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${1:-lazy}
B="bench.py --steps 20 --warmup 3 --no-parity --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-c5 --no-traffic"
j() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["config"]["kernel_ms"]["k_link"]*1e3,1), round(d["ms_per_step"]*1e3,1))'; }
for rep in 1 2; do
  timeout -k 10 120 python -u $B --inflight 1 > $O/${T}_l1.log 2>&1 || exit $?
  timeout -k 10 120 python -u $B > $O/${T}_l2.log 2>&1 || exit $?
  ZDL_NOLAZY=1 timeout -k 10 120 python -u $B --inflight 1 > $O/${T}_n1.log 2>&1 || exit $?
  ZDL_NOLAZY=1 timeout -k 10 120 python -u $B > $O/${T}_n2.log 2>&1 || exit $?
  echo "lazy serial $(j $O/${T}_l1.log) inflight2 $(j $O/${T}_l2.log) | nolazy serial $(j $O/${T}_n1.log) inflight2 $(j $O/${T}_n2.log)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_${T}_l -o run --output-format csv -- python3 $B --inflight 1 > $O/prof_${T}_l.log 2>&1 || exit $?
ZDL_NOLAZY=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_${T}_n -o run --output-format csv -- python3 $B --inflight 1 > $O/prof_${T}_n.log 2>&1 || exit $?
python3 tools/kstats.py $O/prof_${T}_l/run_kernel_stats.csv | head -5
python3 tools/kstats.py $O/prof_${T}_n/run_kernel_stats.csv | head -5
exit 0
