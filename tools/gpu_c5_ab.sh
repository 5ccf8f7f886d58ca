#!/bin/bash
# C5 leg A/B over environment variants (one process each, 8 steps, the first with parity).
#   tools/gpu_c5_ab.sh TAG "VAR=1 VAR2=x" "VAR=2" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out; mkdir -p $O
i=0
for v in "$@"; do
  i=$((i+1))
  P=--no-parity; [ $i -eq 1 ] && P=
  env $v timeout -k 10 200 python -u tools/c5_run.py --steps 8 $P > $O/c5ab_${TAG}_$i.log 2>&1 || exit $?
  echo "[$v] $(tail -1 $O/c5ab_${TAG}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["ms_per_step_serial"],3), d["parity"], {k: round(v["ms"],3) for k,v in d["phases"].items()})')"
done
