# round 5: 3,000-step convergence of the three precision modes on the procedural scene (100x100, Lego config,
# 4096 rays/step, density-layer bias 1.0 init), same seed
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python tools/psnr_synthetic.py --size 100 --rays 4096 --steps 3000 --seed 42 --precisions fp32,fp32x3,bf16 \
  --density-bias 1.0 > gpurun_out/psnr_long.json 2> gpurun_out/psnr_long.err || exit $?
