#!/bin/bash
# One GPU session of named steps, each under its own time limit, stopping at the first failure:
#   tests   the whole -m gpu suite + smoke()            (tools/gpu_check.sh TAG nobench)
#   bench   the default bench line                      (gpurun_out/bench_TAG.log)
#   c5      the C5 leg alone + its rocprofv3 kernel trace (tools/gpu_c5.sh TAG)
#   c3      the C3 per-GPU-shard bench line
#   sq      SQ / TCC counter passes of k_link at C2      (tools/gpu_sq.sh TAG)
#   hbm     per-kernel HBM traffic of C3 / C5 / JSON / proto3 (tools/gpu_pmc_all.sh TAG)
#   facade  the facades' insertion-order link and IMS getDependencies: wall clock, then a kernel
#           trace (tools/facade_prof.py; gpurun_out/facade_TAG*)
#   tools/gpu_session.sh TAG step...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out; mkdir -p $O
for step in "$@"; do
  case $step in
    tests) tools/gpu_check.sh $TAG nobench || exit $? ;;
    bench) timeout -k 10 400 python -u bench.py > $O/bench_$TAG.log 2>&1 || exit $?
           grep -v '^{' $O/bench_$TAG.log | tail -14 ;;
    c5) tools/gpu_c5.sh $TAG || exit $? ;;
    c3) timeout -k 10 300 python -u bench.py --config c3 > $O/bench_c3_$TAG.log 2>&1 || exit $?
        tail -1 $O/bench_c3_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c3", d["ms_per_step"], d["config"]["kernel_ms"]["k_link"], d["roofline"]["frac"], d["config"]["step_roofline_frac"], d["config"]["parity"])' ;;
    sq) SKIPS=0 tools/gpu_sq.sh $TAG || exit $? ;;
    hbm) tools/gpu_pmc_all.sh $TAG || exit $? ;;
    facade) timeout -k 10 200 python -u tools/facade_prof.py > $O/facade_$TAG.log 2>&1 || exit $?
            cat $O/facade_$TAG.log
            timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/facade_${TAG}_prof -o run --output-format csv -- python3 tools/facade_prof.py > $O/facade_${TAG}_prof.log 2>&1 || exit $?
            python3 tools/kstats.py $(find $O/facade_${TAG}_prof -name 'run_kernel_stats.csv' | head -1) | head -40 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
