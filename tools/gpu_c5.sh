#!/bin/bash
# C5 leg alone (8 steps, parity vs the C++ restatement) and one rocprofv3 kernel-trace of it
# (per-kernel stats + the timeline of every dispatch).
#   tools/gpu_c5.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-c5}
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/c5_run.py --steps 8 > $O/c5_$TAG.log 2>&1 || exit $?
tail -1 $O/c5_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c5", d["ms_per_step"], d["ms_per_step_serial"], d["parity"], {k: round(v["ms"],3) for k,v in d["phases"].items()})'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5prof_$TAG -o run --output-format csv -- python3 tools/c5_run.py --no-parity --steps 4 --host-threads 1 > $O/c5prof_$TAG.log 2>&1 || exit $?
python3 tools/timeline.py $O/c5prof_$TAG --min-us 20 > $O/c5_timeline_$TAG.txt 2>&1 || true
exit 0
