# A/B of library builds (ZDL_LIB_PATH): C2 serial step + kernel stats, k_tail cost model
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
TAG=${1:-ab}
for v in libzdl libzdl_inl libzdl_c; do
  export ZDL_LIB_PATH=$PWD/zipkin_amd/$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2_${TAG}_$v -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline --no-h2d --no-proto3 --no-mysql-rows --no-insertion-order --no-parity > $O/prof_c2_${TAG}_$v.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tc_${TAG}_$v -o run --output-format csv -- python3 tools/tail_cost.py --reps 1 --sizes 65,128,512,2048,32768 > $O/tail_cost_${TAG}_$v.log 2>&1 || exit $?
done
