#!/bin/bash
# JSON v2 fast path: the JSON / proto3 GPU tests, then the C2 JSON decode timed with the fast
# path and all-exact (ZDL_JS_EXACT=1), then the kernel stats of the fast-path run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-js}
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_json_v2.py tests/test_proto3.py tests/test_gpu_store.py > $O/jsab_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $O/jsab_tests_$TAG.log; exit 1; }
tail -3 $O/jsab_tests_$TAG.log
timeout -k 10 240 python3 tools/json_decode_run.py --reps 3 > $O/jsab_fast_$TAG.log 2>&1 || exit $?
ZDL_JS_EXACT=1 timeout -k 10 240 python3 tools/json_decode_run.py --reps 3 > $O/jsab_exact_$TAG.log 2>&1 || exit $?
grep rep $O/jsab_fast_$TAG.log $O/jsab_exact_$TAG.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/jsab_s_$TAG -o run --output-format csv -- python3 tools/json_decode_run.py --reps 2 > $O/jsab_s_$TAG.log 2>&1 || exit $?
exit 0
