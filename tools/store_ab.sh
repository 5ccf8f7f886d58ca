#!/bin/bash
# Store accept (zdl_store_append of the C2 batch, cold and warm) for each libzdl variant in ab/*/, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="bench.py --steps 5 --warm-ms 0 --no-cpu-baseline --no-traffic --no-c5 --no-c3-job --no-h2d --no-proto3 --no-json --no-mysql-rows --no-put-trace --no-insertion-order --no-parity"
for r in $(seq ${1:-2}); do
  for d in ab/*/; do
    v=$(basename $d)
    ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 300 python3 $B > gpurun_out/store_ab_${v}_$r.log 2>&1 || exit $?
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; g=d['config']['store_get_dependencies']; print(sys.argv[2], 'accept', round(g['accept_ms'],2), 'warm', round(g['accept_warm_ms'],2), 'query', round(g['get_dependencies_ms'],3))" gpurun_out/store_ab_${v}_$r.log $v
  done
done
