cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -s -k bf16_gradients -p no:cacheprovider > gpurun_out/ab_new.log 2>&1
YANERF_HIP_LIB=$GRAFT_REPO_ROOT/prebuilt/libyanerf_hip_head.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -s -k bf16_gradients -p no:cacheprovider > gpurun_out/ab_old.log 2>&1
timeout -k 10 300 python tools/microbench.py > gpurun_out/ab_micro_new.json 2>&1 || exit 1
YANERF_HIP_LIB=$GRAFT_REPO_ROOT/prebuilt/libyanerf_hip_head.so timeout -k 10 300 python tools/microbench.py > gpurun_out/ab_micro_old.json 2>&1
