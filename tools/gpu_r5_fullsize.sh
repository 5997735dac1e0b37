# round 5: the full-size training-step property test
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "full_size" > gpurun_out/fullsize_tests.log 2>&1 || exit $?
