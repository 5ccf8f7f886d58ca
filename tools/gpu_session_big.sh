cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
TAG=${1:-big}
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_tree.py -q -x --timeout 300 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1; rc=$?; echo "pytest exit $rc" >> $O/gpu_tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c5_$TAG.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c5_$TAG -o run --output-format csv -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-parity --no-cpu-baseline > $O/prof_c5_${TAG}_bench.log 2>&1 || exit $?
