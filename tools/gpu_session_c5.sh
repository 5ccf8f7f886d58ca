cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
TAG=${1:-c5}
timeout -k 10 500 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_$TAG.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-parity --no-cpu-baseline > $O/prof_${TAG}_bench.log 2>&1 || exit $?
