#!/usr/bin/env bash
# GPU-box check used during development: parity tests, a short bench, the MLP microbench.
# usage (via gpurun): bash tools/gpu_check.sh TAG [bench args...]
set -u
TAG=${1:-run}; shift || true
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -rf -s -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/gpu_tests_$TAG.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --psnr-steps 0 "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
timeout -k 10 300 python tools/microbench.py > gpurun_out/micro_$TAG.json 2> gpurun_out/micro_$TAG.err
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/kt_$TAG" -o run --output-format csv -- python tools/microbench.py > gpurun_out/kt_$TAG.log 2>&1 || exit $?
