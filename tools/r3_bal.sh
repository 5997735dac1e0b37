#!/usr/bin/env bash
# dW split-plan check: GPU suite on the in-tree library, then the bf16 MLP microbench against the variant libraries.
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_bal.log 2>&1 || exit $?
bash tools/ab_libs.sh bal bf16 build/bal0.so build/bal_r1.so build/bal_r3.so
