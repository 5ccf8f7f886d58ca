#!/bin/bash
# JSON fast path reading HBM (default, ZDL_JS_GLOBAL=1), at 4 waves per SIMD (2), from the LDS
# window (0): the JSON GPU tests under 1 and 2, then the C2 decode timed under each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for v in 1 2; do
  ZDL_JS_GLOBAL=$v timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_json_v2.py > $O/jsg_tests_$v.log 2>&1 || { tail -30 $O/jsg_tests_$v.log; exit 1; }
  echo "tests global=$v: $(tail -1 $O/jsg_tests_$v.log)"
done
for v in 1 2 0 1 2 0; do
  ZDL_JS_GLOBAL=$v timeout -k 10 240 python3 tools/json_decode_run.py --reps 3 > $O/jsg_$v.log 2>&1 || exit $?
  echo "global=$v $(grep 'rep 2' $O/jsg_$v.log)"
done
exit 0
