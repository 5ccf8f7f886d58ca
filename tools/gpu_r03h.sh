#!/bin/bash
# r03h: sparse/large-table GPU tests, then C5 with the narrow PCIe copy at 8 / 32 / 64 workgroups
# and a timeline of the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-r03h}
timeout -k 10 400 python -u -m pytest tests/test_gpu_giant.py tests/test_gpu_scale.py tests/test_gpu_store.py -q -x --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests_$T.log; tail -2 $O/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
for w in 8 32 64; do
  ZDL_PCIE_WGS=$w timeout -k 10 200 python -u tools/c5_run.py --no-parity --steps 4 > $O/c5_${T}_$w.log 2>&1 || exit $?
  tail -1 $O/c5_${T}_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("wgs '$w'", round(d["ms_per_step"],3), round(d["ms_per_step_serial"],3), {k: round(v["ms"],3) for k, v in d["phases"].items()})'
done
bash tools/gpu_c5_trace.sh c5tl_$T || exit $?
exit 0
