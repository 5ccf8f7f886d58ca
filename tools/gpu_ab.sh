#!/bin/bash
# A/B of the libzdl variants in ab/*/libzdl.so (tools/ab_build.sh NAME "-D..." ...), one GPU call:
#   tools/gpu_ab.sh c2|c3|c5 [ROUNDS]
# c2 / c3: k_link (HIP events, serial leg) and the step, one and two steps in flight; c5: the
# step and its phases (tools/c5_run.py). Variants alternate inside each round, so box drift hits
# them alike. Every run has its own time limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
CFG=${1:-c2}; ROUNDS=${2:-2}
B="bench.py --config $CFG --no-c3-job --steps 12 --warmup 3 --warm-ms 100 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity --no-c5 --no-traffic --no-put-trace"
j() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; r=c.get("log_reduce"); print(round(c["kernel_ms"]["k_link"]*1e3,1), round(d["ms_per_step"]*1e3,1), "reduce", round(r["ms"]*1e3,1) if r else "-", r["entries"] if r else "")'; }
j5() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["ms_per_step_serial"],3), d["parity"], {k: round(v["ms"],3) for k,v in d["phases"].items()})'; }
for rep in $(seq $ROUNDS); do
  for d in ab/*/; do
    v=$(basename $d)
    L="ZDL_LIB_PATH=$PWD/$d/libzdl.so"
    if [ "$CFG" = c5 ]; then
      env $L timeout -k 10 200 python -u tools/c5_run.py --steps 12 > $O/ab_${CFG}_$v.log 2>&1 || exit $?
      echo "$v c5 (step, serial, parity, phases) $(j5 $O/ab_${CFG}_$v.log)"
    else
      env $L timeout -k 10 200 python -u $B --inflight 1 > $O/ab_${CFG}_1_$v.log 2>&1 || exit $?
      env $L timeout -k 10 200 python -u $B > $O/ab_${CFG}_2_$v.log 2>&1 || exit $?
      echo "$v $CFG serial (us k_link, step) $(j $O/ab_${CFG}_1_$v.log)  inflight2 $(j $O/ab_${CFG}_2_$v.log)"
    fi
  done
done
exit 0
