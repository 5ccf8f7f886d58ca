#!/bin/bash
# Per-kernel HBM traffic for every kernel of C2, the C3 shard, C5 and the two decoders: for each
# command one rocprofv3 --kernel-trace --stats run (durations) and two PMC runs (FETCH_SIZE,
# WRITE_SIZE), joined by tools/kernel_hbm.py into gpurun_out/hbm_<name>_<TAG>.{txt,json}.
# (C2's k_link: bench.py's own FETCH_SIZE / WRITE_SIZE passes, roofline.traffic.)
#   tools/gpu_pmc_all.sh TAG [c2 c3 c5 json proto3]   (default: all five)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03}
O=gpurun_out
mkdir -p $O
run() {  # name timeout command...
  local n=$1 t=$2
  shift 2
  timeout -k 10 $t rocprofv3 --kernel-trace --stats -d $O/hs_${n}_$TAG -o run --output-format csv -- "$@" > $O/hs_${n}_$TAG.log 2>&1 || return $?
  timeout -s KILL $t rocprofv3 --pmc FETCH_SIZE -d $O/hf_${n}_$TAG -o run --output-format csv -- "$@" > $O/hf_${n}_$TAG.log 2>&1 || return $?
  timeout -s KILL $t rocprofv3 --pmc WRITE_SIZE -d $O/hw_${n}_$TAG -o run --output-format csv -- "$@" > $O/hw_${n}_$TAG.log 2>&1 || return $?
  python3 tools/kernel_hbm.py $(ls $O/hs_${n}_$TAG/*kernel_stats.csv $O/hs_${n}_$TAG/*/*kernel_stats.csv 2>/dev/null | head -1) \
    $O/hf_${n}_$TAG $O/hw_${n}_$TAG --json $O/hbm_${n}_$TAG.json --label "$n" > $O/hbm_${n}_$TAG.txt
}
B="bench.py --steps 3 --warmup 1 --inflight 1 --no-parity --no-cpu-baseline --no-traffic --no-c5 --no-c3-job --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-put-trace --no-insertion-order"
shift
WHICH=${*:-c2 c3 c5 json proto3}
for n in $WHICH; do
  case $n in
    c2) run c2 240 python3 $B --config c2 || exit $? ;;
    c3) run c3 300 python3 $B --config c3 || exit $? ;;
    c5) run c5 400 python3 tools/c5_run.py --no-parity --steps 2 --host-threads 1 || exit $? ;;
    json) run json 240 python3 tools/json_decode_run.py --reps 2 || exit $? ;;
    proto3) run proto3 240 python3 tools/json_decode_run.py --reps 2 --format proto3 || exit $? ;;
  esac
done
exit 0
