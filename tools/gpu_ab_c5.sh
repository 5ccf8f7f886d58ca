#!/bin/bash
# C5 A/B of ab/*/libzdl.so (tools/ab_build.sh) against the in-tree build: the giant-tier tests
# under each variant, then the C5 step (two host threads) and the k_big / k_tail phase, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for d in ab/*/; do
  v=$(basename $d)
  ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 400 python -u -m pytest tests/test_gpu_giant.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > $O/abc5_tests_$v.log 2>&1 || { tail -5 $O/abc5_tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 $O/abc5_tests_$v.log)"
done
j() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["ms_per_step_serial"],3), d["parity"], {k: round(v["ms"],3) for k,v in d["phases"].items()})'; }
for rep in 1 2; do
  timeout -k 10 200 python -u tools/c5_run.py --steps 12 > $O/abc5_base.log 2>&1 || exit $?
  echo "base $(j $O/abc5_base.log)"
  for d in ab/*/; do
    v=$(basename $d)
    ZDL_LIB_PATH=$PWD/$d/libzdl.so timeout -k 10 200 python -u tools/c5_run.py --steps 12 > $O/abc5_$v.log 2>&1 || exit $?
    echo "$v $(j $O/abc5_$v.log)"
  done
done
exit 0
