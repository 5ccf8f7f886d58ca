#!/bin/bash
# k_js_spans instruction mix: one stats run and two SQ counter passes over the C2 JSON decode.
#   tools/gpu_js_pmc.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-js}
O=gpurun_out
mkdir -p $O
C="python3 tools/json_decode_run.py --reps 2"
timeout -k 10 240 $C > $O/js_run_$TAG.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/jss_$TAG -o run --output-format csv -- $C > $O/jss_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d $O/jsp1_$TAG -o run --output-format csv -- $C > $O/jsp1_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_FLAT -d $O/jsp2_$TAG -o run --output-format csv -- $C > $O/jsp2_$TAG.log 2>&1 || exit $?
exit 0
