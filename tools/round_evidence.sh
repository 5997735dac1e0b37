#!/usr/bin/env bash
# One call of round evidence on the current tree: GPU suite + smoke + default bench (round_check.sh), the kernel
# trace of the default bench command (prof_default_bench.sh), then the PMC FETCH/WRITE passes per precision.
# usage (via gpurun): bash tools/round_evidence.sh TAG
set -u
TAG=${1:-re}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/round_check.sh $TAG || exit $?
bash tools/prof_default_bench.sh ${TAG}_pd || exit $?
SKIP_KT=1 bash tools/gpu_profile.sh ${TAG}_pmc || exit $?
