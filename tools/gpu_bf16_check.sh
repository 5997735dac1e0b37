#!/usr/bin/env bash
# bf16-mode check: the bf16 GPU tests, then the MLP microbench and the step-time A/B for the in-tree library and
# (optionally) a variant library.
# usage (via gpurun): bash tools/gpu_bf16_check.sh TAG [variant.so]
set -u
TAG=${1:-b}; VAR=${2:-}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -k "bf16" -v --timeout 200 --timeout-method thread -p no:cacheprovider -s > gpurun_out/bf16tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/bf16tests_$TAG.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/microbench.py bf16 > gpurun_out/mb_$TAG.json 2>/dev/null || exit $?
timeout -k 10 300 python tools/ab_overlap.py bf16 > gpurun_out/ab_$TAG.json 2>/dev/null || exit $?
if [ -n "$VAR" ]; then
  YANERF_HIP_LIB=$GRAFT_REPO_ROOT/$VAR timeout -k 10 200 python tools/microbench.py bf16 > gpurun_out/mb_${TAG}_var.json 2>/dev/null || exit $?
  YANERF_HIP_LIB=$GRAFT_REPO_ROOT/$VAR timeout -k 10 300 python tools/ab_overlap.py bf16 > gpurun_out/ab_${TAG}_var.json 2>/dev/null || exit $?
fi
exit $rc
