# round 5: the large-batch roofline leg of bench.py's extras, timed alone
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python - > gpurun_out/large_batch.json 2> gpurun_out/large_batch.err <<'PY'
import json, math, sys, torch
sys.argv = ["bench.py"]
import bench
from yanerf_amd.utils.config import Config
import yanerf_boot
cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml"))
pcfg = cfg.pipeline
dev = torch.device("cuda:0")
poses = torch.stack([torch.from_numpy(bench.synthetic_pose(th, -30.0)) for th in range(0, 360, 9)]).float().to(dev)
focal = torch.tensor([0.5 * 800 / math.tan(0.5 * 0.6911112)], device=dev)
image = torch.rand(1, 800, 800, 3, device=dev)
from yanerf_amd.train import NeRFTrainer
out = {}
for p, R_big in (("bf16", 4096), ("bf16", 16384), ("bf16", 65536), ("fp32", 16384)):
    tr = NeRFTrainer(pcfg, precision=p, device=dev, n_rays=R_big)
    for i in range(2):
        tr.step(poses[i:i + 1], focal, image)
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    for i in range(6):
        tr.step(poses[(2 + i) % 40][None], focal, image)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 6
    out[f"{p}_{R_big}"] = {"rays_per_s": round(R_big / dt, 1), "ms": round(1e3 * dt, 3),
                           "frac": round(bench.train_flops_per_ray(tr.Pc, tr.Pf) * R_big / dt / 1e12 / bench.PEAK_TFLOPS[p], 4),
                           "mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1)}
    print(json.dumps(out), file=sys.stderr, flush=True)
    del tr
    torch.cuda.empty_cache()
print(json.dumps(out))
PY
