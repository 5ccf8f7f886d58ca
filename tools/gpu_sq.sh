#!/bin/bash
# SQ counters of k_link at C2, one rocprofv3 pass per counter set, for ZDL_SKIP values
#   SKIPS="0 8224" tools/gpu_sq.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
TAG=${1:-sq}
B="bench.py --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH"
for sk in ${SKIPS:-0}; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    ZDL_SKIP=$sk timeout -s KILL 90 rocprofv3 --pmc $P -d $O/sq_${TAG}_${sk}_$i -o run --output-format csv -- python3 $B > $O/sq_${TAG}_${sk}_$i.log 2>&1 || exit $?
  done
done
