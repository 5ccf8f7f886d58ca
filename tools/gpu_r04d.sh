#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_check.sh r04d nobench || exit $?
tools/gpu_ab_tree.sh r03
