# round 5: this build's run of the reference-collapse configuration with the density-layer bias at 1.0 (the
# reference's own run of it: profiles/r5_reference_collapse.jsonl)
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for p in fp32 bf16; do
  timeout -k 10 300 python tools/psnr_synthetic.py --size 50 --rays 1024 --steps 1000 --seed 42 --precisions $p \
    --density-bias 1.0 > gpurun_out/collapse_ours_b1_$p.json 2>&1 || exit 1
done
