#!/bin/bash
# r03o: C5 link-record transfer A/B (narrow copy kernel vs hipMemcpyAsync into coarse-grained
# pinned memory), the bench's C5 leg alone, and a memory-copy timeline of the DMA variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-r03o}
for v in "ZDL_REC_DMA=0" "ZDL_REC_DMA=1" "ZDL_REC_DMA=0 ZDL_PCIE_WGS=16"; do
  env $v timeout -k 10 200 python -u tools/c5_run.py --no-parity --steps 8 > $O/c5_$T.log 2>&1 || exit $?
  tail -1 $O/c5_$T.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"$v"'", round(d["ms_per_step"],3), round(d["ms_per_step_serial"],3))'
done
B="bench.py --steps 5 --warmup 2 --no-parity --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-traffic"
timeout -k 10 300 python -u $B > $O/benchc5_$T.log 2>&1 || exit $?
tail -1 $O/benchc5_$T.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench c5 leg", d["config"]["c5"]["ms_per_step"], d["config"]["c5"]["ms_per_step_serial"])'
ZDL_REC_DMA=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/c5dma_$T -o run --output-format csv -- python3 tools/c5_run.py --no-parity --steps 4 > $O/c5dma_$T.log 2>&1 || exit $?
exit 0
