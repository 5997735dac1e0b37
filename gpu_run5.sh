set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -rf -p no:cacheprovider > gpurun_out/gpu_tests5.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/gpu_tests5.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err
timeout -k 10 300 python tools/microbench.py > gpurun_out/micro5.json 2> gpurun_out/micro5.err
