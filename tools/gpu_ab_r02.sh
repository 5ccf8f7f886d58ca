#!/bin/bash
# C2 k_link on one box: the round-2 tree (ab/r02src, its own bench.py and libzdl.so) against
# the current tree's A/B builds ab/<v>/libzdl.so; serial and two puts in flight, twice; rocprof
# of r02 and of the current build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out; mkdir -p $O
F="--steps 20 --warmup 3 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity"
j() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["config"]["kernel_ms"]["k_link"]*1e3,1), round(d["ms_per_step"]*1e3,1))'; }
for rep in 1 2; do
  (cd ab/r02src && timeout -k 10 120 python -u bench.py $F --inflight 1 > $O/abr_r02_1.log 2>&1) || exit $?
  (cd ab/r02src && timeout -k 10 120 python -u bench.py $F > $O/abr_r02_2.log 2>&1) || exit $?
  echo "r02 serial $(j $O/abr_r02_1.log) inflight2 $(j $O/abr_r02_2.log)"
  for v in cur prio0; do
    ZDL_LIB_PATH=$PWD/ab/$v/libzdl.so timeout -k 10 120 python -u bench.py $F --no-c5 --no-traffic --inflight 1 > $O/abr_${v}_1.log 2>&1 || exit $?
    ZDL_LIB_PATH=$PWD/ab/$v/libzdl.so timeout -k 10 120 python -u bench.py $F --no-c5 --no-traffic > $O/abr_${v}_2.log 2>&1 || exit $?
    echo "$v serial $(j $O/abr_${v}_1.log) inflight2 $(j $O/abr_${v}_2.log)"
  done
done
(cd ab/r02src && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/abr_prof_r02 -o run --output-format csv -- python3 bench.py $F --inflight 1 > $O/abr_prof_r02.log 2>&1) || exit $?
python3 tools/kstats.py $O/abr_prof_r02/run_kernel_stats.csv | head -4
exit 0
