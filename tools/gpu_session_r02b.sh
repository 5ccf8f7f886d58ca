cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > $O/gpu_tests_r02b.log 2>&1; rc=$?; echo "pytest exit $rc" >> $O/gpu_tests_r02b.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > $O/bench_c3_r02b.log 2>&1 || exit $?
B="bench.py --steps 10 --warmup 2 --no-parity --no-cpu-baseline --config c3"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c3_r02b -o run --output-format csv -- python3 $B > $O/prof_c3_r02b_bench.log 2>&1 || exit $?
