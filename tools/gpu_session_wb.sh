# big-trace session: the big-trace GPU tests, C2 serial step + kernel stats, the k_tail cost
# model (per-dispatch k_mid / k_tail under rocprofv3), C5 bench + kernel stats
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
TAG=${1:-wb}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_parity.py > $O/gpu_tests_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2_$TAG -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline --no-h2d --no-proto3 --no-mysql-rows --no-insertion-order --no-parity > $O/prof_c2_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tc_$TAG -o run --output-format csv -- python3 tools/tail_cost.py --reps 2 > $O/tail_cost_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c5_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5_$TAG -o run --output-format csv -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-parity --no-cpu-baseline > $O/prof_c5_${TAG}_bench.log 2>&1 || exit $?
