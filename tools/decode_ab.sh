#!/bin/bash
# The proto3 and JSON v2 ingest side legs for each libzdl variant in ab/*/, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="bench.py --steps 5 --warm-ms 0 --no-parity --no-cpu-baseline --no-traffic --no-c5 --no-c3-job --no-h2d --no-store --no-mysql-rows --no-put-trace --no-insertion-order"
for r in $(seq ${1:-2}); do
  for d in ab/*/; do
    v=$(basename $d)
    ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 400 python3 $B > gpurun_out/dec_ab_${v}_$r.log 2>&1 || exit $?
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; p=d['config']['proto3_ingest']; j=d['config']['json_v2_ingest']; print(sys.argv[2], 'proto3 call', round(p['call_ms'],2), 'kernel', round(p['kernel_ms'],2), p['parity'], '| json call', round(j['call_ms'],2), j['parity'])" gpurun_out/dec_ab_${v}_$r.log $v
  done
done
