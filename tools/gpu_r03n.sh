#!/bin/bash
# r03n: GPU suite, the default bench line, then per-kernel HBM traffic for C3 / C5 / decoders
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-r03n}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests_$T.log; tail -2 $O/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > $O/bench_$T.log 2>&1 || exit $?
tail -1 $O/bench_$T.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; s=c["store_get_dependencies"]; print("C2", d["value"], d["ms_per_step"], c["step_roofline_frac"], "store", s["get_dependencies_ms"], "facade", s["facade_get_dependencies_ms"], "C5", c["c5"]["ms_per_step"], c["c5"]["parity"], "ins", c["insertion_order"]["ms_per_step"])'
bash tools/gpu_pmc_all.sh $T || exit $?
exit 0
