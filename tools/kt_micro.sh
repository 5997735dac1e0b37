#!/usr/bin/env bash
# rocprofv3 kernel stats of the MLP microbench (per-kernel times), plus its HIP-event JSON.
# usage (via gpurun): bash tools/kt_micro.sh TAG [precisions]
set -u
TAG=${1:-km}; PRECS=${2:-fp32,bf16,fp32x3}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/microbench.py $PRECS > gpurun_out/micro_$TAG.json 2> gpurun_out/micro_$TAG.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/kt_$TAG" -o run --output-format csv -- python tools/microbench.py $PRECS > gpurun_out/kt_$TAG.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/kt_$TAG 30 > gpurun_out/kt_$TAG.txt
