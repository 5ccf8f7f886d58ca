#!/bin/bash
# SQ / TCC counters of k_link at C2, one rocprofv3 pass per counter set, for ZDL_SKIP values
# (0 = the production kernel; other values the PROF == 2 ablation instantiation).
#   SKIPS="0 64" tools/gpu_sq.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
TAG=${1:-sq}
B="bench.py --pmc-probe --config c2"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_INT64 SQ_INSTS_LDS_ATOMIC GRBM_GUI_ACTIVE GRBM_COUNT"
P4="TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum"
for sk in ${SKIPS:-0}; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    ZDL_SKIP=$sk timeout -s KILL 90 rocprofv3 --pmc $P -d $O/sq_${TAG}_${sk}_$i -o run --output-format csv -- python3 $B > $O/sq_${TAG}_${sk}_$i.log 2>&1 || exit $?
  done
  ZDL_SKIP=$sk timeout -k 10 90 rocprofv3 --kernel-trace --stats -d $O/sq_${TAG}_${sk}_t -o run --output-format csv -- python3 $B > $O/sq_${TAG}_${sk}_t.log 2>&1 || exit $?
done
