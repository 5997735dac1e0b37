#!/usr/bin/env bash
# A/B microbench of variant libraries against the in-tree build, then the GPU tests matching a -k expression.
# usage (via gpurun): bash tools/ab_then_tests.sh TAG PREC "k-expression" lib1.so [lib2.so ...]
set -u
TAG=$1; PREC=$2; KEXPR=$3; shift 3
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_libs.sh $TAG $PREC "$@" || exit $?
bash tools/gpu_tests.sh $TAG "$KEXPR"
