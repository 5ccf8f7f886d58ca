#!/bin/bash
# The 1B-span C3 job side leg (8 local ranks on one GPU) for each libzdl variant in ab/*/, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="bench.py --steps 5 --warm-ms 0 --no-parity --no-cpu-baseline --no-traffic --no-c5 --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-put-trace --no-insertion-order"
for r in $(seq ${1:-2}); do
  for d in ab/*/; do
    v=$(basename $d)
    ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 400 python3 $B > gpurun_out/job_ab_${v}_$r.log 2>&1 || exit $?
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; j=d['config']['c3_job']; p=j['phased']; print(sys.argv[2], 'job', round(j['ms_per_job_step'],2), 'puts', round(p['puts_ms'],2), 'link', round(p['link_phase_ms'],2), 'combine', round(p['combine_ms'],3))" gpurun_out/job_ab_${v}_$r.log $v
  done
done
