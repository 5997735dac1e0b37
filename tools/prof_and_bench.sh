#!/usr/bin/env bash
# Profiles (tools/gpu_profile.sh TAG) then the default bench command, as the driver runs it.
set -u
TAG=${1:-prof}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
if [ "${SKIP_PROFILE:-0}" != "1" ]; then bash tools/gpu_profile.sh "$TAG" || exit $?; fi
export TMPDIR=/tmp
start=$(date +%s)
timeout -k 10 900 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
echo "bench wall seconds: $(( $(date +%s) - start ))" >> gpurun_out/bench_default.err
