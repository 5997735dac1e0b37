# round 5: the pack_multi GPU test (incl. the 16-layer flush case)
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "pack_multi" > gpurun_out/packtest.log 2>&1 || exit $?
