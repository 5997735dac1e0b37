#!/usr/bin/env bash
# One-card rehearsal of the N-rank bench path: two ranks share cuda:0 over gloo (RCCL needs a card per rank), so the
# barrier / all-reduce / max-over-ranks / weak-scaling code runs as it will on an 8-GPU node. Not a measurement.
# usage (via gpurun): bash tools/rehearse_n2.sh TAG
set -u
TAG=${1:-n2}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export YANERF_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --psnr-steps 0 --secondary none \
  > gpurun_out/bench_$TAG.raw 2> gpurun_out/bench_$TAG.err && grep "^{" gpurun_out/bench_$TAG.raw > gpurun_out/bench_$TAG.json
