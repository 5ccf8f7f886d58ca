cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --config c3 --no-c3-job --steps 10 --warmup 3 --no-cpu-baseline --no-h2d --no-proto3 --no-json --no-store --no-mysql-rows --no-insertion-order --no-parity --no-c5 --no-traffic --no-put-trace"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/c3tl -o run --output-format csv -- python3 $B > gpurun_out/c3tl_bench.log 2>&1 || exit $?
f=$(find gpurun_out/c3tl -name '*kernel_trace.csv' | head -1); d=$(dirname $f)
python3 tools/timeline.py $d --min-us 0 --marker "k_link" --from 6 --to 11 > gpurun_out/c3tl_timeline.txt 2>&1
exit 0
