# round 5: the whole GPU suite and smoke on the final tree (as the driver runs them)
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r5final.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r5final.log 2>&1 || exit $?
