#!/usr/bin/env bash
# The N-rank step schedule on one card: bench.py at world size 1 with a process group up (YANERF_PG_AT_WORLD1=1: RCCL,
# the two-bucket exchange with its collectives; bf16 "early": the coarse backward AND its bucket's all-reduce on the side
# stream) against the plain N=1 line, interleaved twice. usage (via gpurun): bash tools/rehearse_pg_world1.sh TAG
set -u
TAG=${1:-pg1}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 5 --no-extras --psnr-steps 0 --no-cpu-baseline --secondary bf16"
for r in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_plain_$r.json 2> gpurun_out/${TAG}_plain_$r.err || exit $?
  MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + r)) RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 YANERF_PG_AT_WORLD1=1 \
    timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_pg_$r.json 2> gpurun_out/${TAG}_pg_$r.err || exit $?
done
