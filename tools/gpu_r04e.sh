#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_check.sh r04f nobench || exit $?
tools/gpu_c5.sh r04f
