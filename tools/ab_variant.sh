#!/usr/bin/env bash
# A/B a prebuilt variant library against the in-tree build: the given GPU tests + the MLP microbench for both.
# usage (via gpurun): bash tools/ab_variant.sh prebuilt/libX.so "pytest -k expr" [PREC]
set -u
LIB=$1; KEXPR=${2:-bf16}; PREC=${3:-bf16}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
YANERF_HIP_LIB=$GRAFT_REPO_ROOT/$LIB timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_convergence.py -q -s -k "$KEXPR" -p no:cacheprovider > gpurun_out/abv_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/abv_tests.log
timeout -k 10 300 python tools/microbench.py $PREC > gpurun_out/abv_base.json 2>/dev/null || exit $?
YANERF_HIP_LIB=$GRAFT_REPO_ROOT/$LIB timeout -k 10 300 python tools/microbench.py $PREC > gpurun_out/abv_var.json 2>/dev/null || exit $?
timeout -k 10 300 python tools/microbench.py $PREC > gpurun_out/abv_base2.json 2>/dev/null
