#!/usr/bin/env bash
# Step-time A/B of the backward schedules (serial / both / split / early) for the in-tree library and variant libraries.
# usage (via gpurun): bash tools/ab_sched.sh PRECS [lib ...]
set -u
PRECS=${1:-bf16}; shift || true
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_overlap.py $PRECS > gpurun_out/absched_base.json 2> gpurun_out/absched_base.err || exit $?
for lib in "$@"; do
  tag=$(basename $lib .so)
  YANERF_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 python tools/ab_overlap.py $PRECS > gpurun_out/absched_$tag.json 2> gpurun_out/absched_$tag.err || exit $?
done
