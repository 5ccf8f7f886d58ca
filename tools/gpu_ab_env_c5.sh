#!/bin/bash
# C5 A/B of one environment switch on the in-tree build: tools/gpu_ab_env_c5.sh VAR=VALUE
# (the giant / scale / tree / parity tests first, default build), then the C5 step twice each way.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_giant.py tests/test_gpu_scale.py tests/test_gpu_tree_stream.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/abenv_tests.log 2>&1 || { tail -5 $O/abenv_tests.log; exit 1; }
echo "tests: $(tail -1 $O/abenv_tests.log)"
j() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["ms_per_step_serial"],3), d["parity"], {k: round(v["ms"],3) for k,v in d["phases"].items()})'; }
for rep in 1 2; do
  timeout -k 10 200 python -u tools/c5_run.py --steps 16 > $O/abenv_new.log 2>&1 || exit $?
  echo "default $(j $O/abenv_new.log)"
  env "$1" timeout -k 10 200 python -u tools/c5_run.py --steps 16 > $O/abenv_old.log 2>&1 || exit $?
  echo "$1 $(j $O/abenv_old.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/abenv_prof -o run --output-format csv -- python3 tools/c5_run.py --no-parity --steps 4 --host-threads 1 > $O/abenv_prof.log 2>&1 || exit $?
grep -h "k_mid" $O/abenv_prof/run_kernel_stats.csv | cut -d, -f1-4
exit 0
