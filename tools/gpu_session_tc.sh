# k_tail cost model under rocprofv3 (per-dispatch k_tail durations), wave_big on and off
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
TAG=${1:-tc}
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tc_$TAG -o run --output-format csv -- python3 tools/tail_cost.py --reps 2 > $O/tail_cost_$TAG.log 2>&1 || exit $?
ZDL_WAVE_BIG=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tc0_$TAG -o run --output-format csv -- python3 tools/tail_cost.py --reps 2 --sizes 65,128,192 > $O/tail_cost0_$TAG.log 2>&1 || exit $?
