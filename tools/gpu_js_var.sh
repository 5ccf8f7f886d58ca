#!/bin/bash
# k_js_fast variants: C2 JSON decode with the in-tree libzdl.so and with each
# zipkin_amd/libzdl_<v>.so given (ZDL_LIB_PATH), then SQ counters of the in-tree build.
#   tools/gpu_js_var.sh TAG v1 v2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
shift
O=gpurun_out
mkdir -p $O
timeout -k 10 240 python3 tools/json_decode_run.py --reps 3 > $O/jsv_${TAG}_a.log 2>&1 || exit $?
grep rep $O/jsv_${TAG}_a.log
for v in "$@"; do
  ZDL_LIB_PATH=$PWD/zipkin_amd/libzdl_$v.so timeout -k 10 240 python3 tools/json_decode_run.py --reps 3 > $O/jsv_${TAG}_$v.log 2>&1 || exit $?
  echo "variant $v"; grep rep $O/jsv_${TAG}_$v.log
done
C="python3 tools/json_decode_run.py --reps 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d $O/jsvp_$TAG -o run --output-format csv -- $C > $O/jsvp_$TAG.log 2>&1 || exit $?
exit 0
