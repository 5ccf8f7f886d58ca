# C2 quick: bench (serial and 2 in flight) + kernel stats
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
TAG=${1:-c2}
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --inflight 1 --no-cpu-baseline --no-h2d --no-proto3 --no-mysql-rows --no-insertion-order --no-parity > $O/bench_c2s_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2_$TAG -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline --no-h2d --no-proto3 --no-mysql-rows --no-insertion-order --no-parity > $O/prof_c2_${TAG}_bench.log 2>&1 || exit $?
