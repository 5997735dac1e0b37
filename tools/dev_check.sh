#!/usr/bin/env bash
# Development check on the GPU box: GPU parity tests then the per-kernel microbench (HIP events) and its kernel stats.
# usage (via gpurun): bash tools/dev_check.sh TAG [precisions]
set -u
TAG=${1:-dev}; PRECS=${2:-fp32,bf16,fp32x3}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/gpu_tests_$TAG.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/kt_micro.sh $TAG $PRECS
