#!/bin/bash
# r03i: C5 two in flight with the non-temporal PCIe copy at 4 / 8 / 16 workgroups
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-r03i}
for w in 8 16 32; do
  ZDL_PCIE_WGS=$w timeout -k 10 200 python -u tools/c5_run.py --no-parity --steps 4 > $O/c5_${T}_$w.log 2>&1 || exit $?
  tail -1 $O/c5_${T}_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("wgs '$w'", round(d["ms_per_step"],3), round(d["ms_per_step_serial"],3), {k: round(v["ms"],3) for k, v in d["phases"].items()})'
done
exit 0
