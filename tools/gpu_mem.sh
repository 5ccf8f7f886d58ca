#!/bin/bash
# Memory-path counters for k_link (TLB, L1->L2 latency, TA stalls), full kernel and stream-only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-m}
O=gpurun_out
mkdir -p $O
B="bench.py --steps 3 --warmup 1 --no-parity --no-cpu-baseline"
for sk in 0 32; do
  ZDL_SKIP=$sk timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ -d $O/pmc_tcp_${TAG}_$sk -o run --output-format csv -- python3 $B > $O/pmc_tcp_${TAG}_$sk.log 2>&1 || exit $?
  ZDL_SKIP=$sk timeout -s KILL 120 rocprofv3 --pmc TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES TCP_UTCL1_STALL_MULTI_MISS GRBM_GUI_ACTIVE -d $O/pmc_ta_${TAG}_$sk -o run --output-format csv -- python3 $B > $O/pmc_ta_${TAG}_$sk.log 2>&1 || exit $?
done
