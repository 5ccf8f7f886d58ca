set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_giant.py tests/test_gpu_scale.py -x -v --timeout 400 --timeout-method thread -k "giant or c5 or sparse or mid_size" > gpurun_out/r03a_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03a_tests.log; exit 1; }
tail -3 gpurun_out/r03a_tests.log
timeout -k 10 400 python -u bench.py --steps 20 --no-json --no-proto3 --no-mysql-rows --no-h2d --no-store --no-insertion-order > gpurun_out/r03a_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/r03a_bench.log; exit 1; }
tail -c 3000 gpurun_out/r03a_bench.log
