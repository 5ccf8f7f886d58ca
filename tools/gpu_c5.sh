#!/bin/bash
# C5 work loop: the big-trace / sparse / store / scale GPU tests, C5 steps (two in flight and
# serial, phases) and a kernel timeline of the C5 run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-c5}
timeout -k 10 500 python -u -m pytest tests/test_gpu_giant.py tests/test_gpu_scale.py tests/test_gpu_store.py tests/test_gpu_parity.py tests/test_gpu_tree_stream.py -q -x --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests_$T.log; tail -2 $O/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/c5_run.py --steps 4 > $O/c5_$T.log 2>&1 || exit $?
tail -1 $O/c5_$T.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c5", round(d["ms_per_step"],3), round(d["ms_per_step_serial"],3), d["parity"], {k: round(v["ms"],3) for k, v in d["phases"].items()})'
bash tools/gpu_c5_trace.sh c5tl_$T || exit $?
exit 0
