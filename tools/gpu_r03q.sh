#!/bin/bash
# r03q: GPU suite, smoke, the default bench line, the C3 line, rocprofv3 kernel stats of the
# bench's C2 run (no side legs) and of the JSON decode, C2 FETCH/WRITE passes, then the
# per-kernel HBM tables of C3 / C5 / both decoders (tools/gpu_pmc_all.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-r03q}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests_$T.log; tail -2 $O/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench_$T.log 2>&1 || exit $?
tail -1 $O/bench_$T.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; s=c["store_get_dependencies"]; j=c["json_v2_ingest"]; print("C2", d["value"], d["ms_per_step"], c["step_roofline_frac"], "json", j["device_ms"], j["roofline_frac"], "store", s["get_dependencies_ms"], "facade", s["facade_get_dependencies_ms"], "C5", c["c5"]["ms_per_step"], c["c5"]["parity"], "ins", c["insertion_order"]["ms_per_step"])'
timeout -k 10 300 python -u bench.py --config c3 --no-c5 > $O/bench_c3_$T.log 2>&1 || exit $?
B="bench.py --steps 10 --warmup 2 --inflight 1 --no-parity --no-cpu-baseline --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-h2d --no-c5 --no-traffic"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run --output-format csv -- python3 $B > $O/prof_${T}_bench.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$T -o run --output-format csv -- python3 $B > $O/pmc_fetch_$T.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$T -o run --output-format csv -- python3 $B > $O/pmc_write_$T.log 2>&1 || exit $?
bash tools/gpu_pmc_all.sh $T || exit $?
exit 0
