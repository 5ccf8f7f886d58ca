cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_local_world.py tests/test_gpu_put_trace.py tests/test_gpu_store.py -m gpu > $O/t_r05h.log 2>&1; rc=$?; tail -3 $O/t_r05h.log; [ $rc -ne 0 ] && exit $rc
tools/gpu_ab.sh c3 2 || exit $?
B="bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity --no-c5 --no-traffic --no-put-trace"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c3_r05h -o run --output-format csv -- python3 $B > $O/prof_c3_r05h.log 2>&1 || exit $?
python3 tools/kstats.py $(find $O/prof_c3_r05h -name 'run_kernel_stats.csv' | head -1) | head -30
