#!/usr/bin/env bash
# kernel trace of the default bench command + PMC traffic per precision (the evidence half of round_evidence.sh)
set -u
TAG=${1:-r5p}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/prof_default_bench.sh ${TAG}_pd || exit $?
SKIP_KT=1 bash tools/gpu_profile.sh ${TAG}_pmc || exit $?
