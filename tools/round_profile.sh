#!/usr/bin/env bash
# Round-end evidence in one call: full GPU suite + smoke + default bench (round_check.sh), then the profiles
# (gpu_profile.sh: kernel trace of the bench + per-precision FETCH/WRITE passes), then bf16 PSNR runs.
# usage (via gpurun): bash tools/round_profile.sh TAG
set -u
TAG=${1:-rp}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/round_check.sh $TAG || exit $?
bash tools/gpu_profile.sh ${TAG}p || exit $?
timeout -k 10 200 python tools/psnr_synthetic.py --steps 2000 --precisions bf16 > gpurun_out/${TAG}_psnr2k.json || exit $?
timeout -k 10 300 python tools/psnr_synthetic.py --steps 10000 --precisions bf16 > gpurun_out/${TAG}_psnr10k.json || exit $?
