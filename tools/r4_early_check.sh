#!/usr/bin/env bash
# GPU suite + smoke + default bench (round_check.sh), then the backward-schedule A/B (tools/ab_overlap.py)
# usage (via gpurun): bash tools/r4_early_check.sh TAG
set -u
TAG=${1:-ec}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/round_check.sh $TAG || exit $?
timeout -k 10 400 python tools/ab_overlap.py bf16 > gpurun_out/ab_overlap_$TAG.json 2> gpurun_out/ab_overlap_$TAG.err
