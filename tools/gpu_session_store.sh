cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_store.py tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > $O/gpu_tests_store.log 2>&1; rc=$?; echo "pytest exit $rc" >> $O/gpu_tests_store.log; exit $rc
