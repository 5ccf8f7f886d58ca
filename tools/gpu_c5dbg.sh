#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for v in "ZDL_KB_SMALL=0" "ZDL_KB_SMALL=471" "ZDL_KB_SMALL=300" "ZDL_KB_SMALL=471 ZDL_GIANT_MIN=0"; do
  env $v timeout -k 10 200 python -u tools/c5_run.py --steps 2 > $O/c5dbg.log 2>&1
  echo "$v rc=$? $(tail -1 $O/c5dbg.log | cut -c1-200)"
done
exit 0
