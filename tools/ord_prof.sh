cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ordprof -o run --output-format csv -- python3 tools/facade_prof.py --no-store --reps 10 > $O/ordprof.log 2>&1 || exit $?
f=$(find $O/ordprof -name '*kernel_trace.csv' | head -1); d=$(dirname $f)
python3 tools/timeline.py $d --min-us 0 --marker "k_link" --from 8 --to 10 > $O/ordprof_timeline.txt 2>&1
bash tools/gpu_pmc_all.sh r06 c2 c3 c5
