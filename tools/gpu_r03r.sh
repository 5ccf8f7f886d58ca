#!/bin/bash
# r03r: decoder GPU tests + JSON timing, then the C5 host-thread A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_js_ab.sh ${1:-r03r} && bash tools/gpu_c5_threads.sh ${1:-r03r}
