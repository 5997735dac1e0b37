#!/usr/bin/env bash
# Round 4: the pruned kernel source against the round-3 library -- GPU suite + smoke on the in-tree (pruned) build, then
# the MLP microbench A/B (per-kernel times and gradient / output digests, which must be equal) against build/lib_r3final.so.
# usage (via gpurun): bash tools/r4_prune_check.sh TAG
set -u
TAG=${1:-pr}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
bash tools/ab_libs.sh ${TAG} fp32,bf16,fp32x3 build/lib_r3final.so
