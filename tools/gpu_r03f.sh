#!/bin/bash
# r03f: GPU suite, the default bench line (C2 + side legs incl. C5), then the lazy-tail A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${1:-r03f}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests_$T.log; tail -2 $O/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-traffic > $O/bench_$T.log 2>&1 || exit $?
tail -1 $O/bench_$T.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("C2", d["value"], d["ms_per_step"], c["ms_per_step_serial"], c["kernel_ms"]); print("C5", c["c5"]["ms_per_step"], c["c5"]["ms_per_step_serial"], {k: round(v["ms"], 3) for k, v in c["c5"]["phases"].items()})'
bash tools/gpu_ab_lazy.sh ${T}ab || exit $?
exit 0
