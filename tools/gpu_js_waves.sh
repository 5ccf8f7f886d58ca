#!/bin/bash
# JSON fast path at 4 / 5 / 6 waves per SIMD (ZDL_JS_GLOBAL=2 / 3 / 4): the decode timed, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for v in 2 3 4 2 3 4; do
  ZDL_JS_GLOBAL=$v timeout -k 10 240 python3 tools/json_decode_run.py --reps 3 > $O/jsw_$v.log 2>&1 || exit $?
  echo "global=$v $(grep 'rep 2' $O/jsw_$v.log)"
done
exit 0
