#!/usr/bin/env bash
# One-card attempt at the N-rank bench path over RCCL itself (the "nccl" backend): two ranks share cuda:0. RCCL may
# refuse two ranks on one device; the log says which. Not a measurement.
# usage (via gpurun): bash tools/rehearse_n2_rccl.sh TAG
set -u
TAG=${1:-n2rccl}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export NCCL_DEBUG=WARN
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --psnr-steps 0 --secondary none --no-cpu-baseline \
  > gpurun_out/bench_$TAG.raw 2> gpurun_out/bench_$TAG.err
rc=$?
echo "rc=$rc" >> gpurun_out/bench_$TAG.err
exit $rc
