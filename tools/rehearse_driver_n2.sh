#!/usr/bin/env bash
# One-card rehearsal of the driver's N-rank bench command with its default flags (secondary precisions, extras,
# PSNR and CPU legs as the defaults decide at N > 1): two ranks share cuda:0 over gloo (RCCL refuses two ranks on one
# card). Checks that the N-rank line comes out; not a measurement.
# usage (via gpurun): bash tools/rehearse_driver_n2.sh TAG
set -u
TAG=${1:-dn2}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export YANERF_DIST_BACKEND=gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 \
  > gpurun_out/bench_$TAG.raw 2> gpurun_out/bench_$TAG.err && grep "^{" gpurun_out/bench_$TAG.raw > gpurun_out/bench_$TAG.json
