#!/bin/bash
# C5 timeline: kernel + memory-copy trace of the C5 leg (two steps in flight) for overlap analysis
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-c5tl}
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/$T -o run --output-format csv -- python3 tools/c5_run.py --no-parity --steps 4 > $O/$T.log 2>&1 || exit $?
tail -1 $O/$T.log | cut -c1-300
exit 0
