#!/usr/bin/env bash
# Development A/B of compile-time variants: builds one library per "name=FLAGS" argument into /tmp on the GPU box
# and runs the MLP microbench against each (e.g. base= lowreg=-DYANERF_LOWREG=1 noheads=-DYANERF_ABLATE=8).
set -u
TAG=${1:-var}; shift
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for V in "$@"; do
  NAME=${V%%=*}; FLAGS=${V#*=}
  make -s -C yet-another-nerf_amd/csrc OUT=/tmp/libyanerf_$NAME.so EXTRA="$FLAGS" > /dev/null || exit 1
  YANERF_HIP_LIB=/tmp/libyanerf_$NAME.so timeout -k 10 200 python tools/microbench.py ${PREC:-} > gpurun_out/${TAG}_$NAME.json 2>gpurun_out/${TAG}_$NAME.err || exit $?
  echo "$NAME $(cat gpurun_out/${TAG}_$NAME.json)"
done
