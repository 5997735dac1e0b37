#!/usr/bin/env bash
# Development timing ablations of the MLP forward (see YANERF_ABLATE in csrc/mlp.hip): builds one library per
# flag set into /tmp on the GPU box and runs the microbench against each.
set -u
TAG=${1:-abl}; shift
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for A in "$@"; do
  make -s -C yet-another-nerf_amd/csrc OUT=/tmp/libyanerf_abl$A.so EXTRA=-DYANERF_ABLATE=$A > /dev/null || exit 1
  YANERF_HIP_LIB=/tmp/libyanerf_abl$A.so timeout -k 10 200 python tools/microbench.py > gpurun_out/${TAG}_$A.json 2>gpurun_out/${TAG}_$A.err || exit $?
  echo "$A $(cat gpurun_out/${TAG}_$A.json)"
done
