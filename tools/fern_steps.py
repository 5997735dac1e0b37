#!/usr/bin/env python
"""BASELINE configs[3]'s single-GPU step (Fern 504x378, 64 + 128, 1024 rays, per-image bounds; bench.py extras
fern_64_128_train) run for a few steps, for a rocprofv3 kernel trace of the small-batch step (tools/step_timeline.py).
Development tool (GPU).   python tools/fern_steps.py [bf16|fp32] [steps] [eager|graph] [steps per graph] [default|serial|early|both|split] [hiprio]"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden")]
import yanerf_boot  # noqa: E402
from scene import synthetic_pose  # noqa: E402
from yanerf_amd.train import NeRFTrainer  # noqa: E402
from yanerf_amd.utils.config import Config  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 15
mode = sys.argv[3] if len(sys.argv) > 3 else "eager"
dev = torch.device("cuda:0")
fcfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/fern.yml")).pipeline
fcfg.renderer.n_pts_per_ray_fine_training = 128
fcfg.renderer.n_pts_per_ray_fine_evaluation = 128
fimg = torch.rand(1, 378, 504, 3, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
ffocal = torch.tensor([407.56], device=dev)
bounds = torch.tensor([[1.3, 5.9]])
poses = torch.stack([torch.from_numpy(synthetic_pose(th, -30.0, 4.0)) for th in np.linspace(-180, 180, 40,
                                                                                    endpoint=False)]).float().to(dev)
if len(sys.argv) > 6 and sys.argv[6] == "hiprio":  # the step's main stream at high priority, the side stream at default
    torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))
ov = sys.argv[5] if len(sys.argv) > 5 else "default"
ov = {"default": None, "serial": False}.get(ov, ov)
tr = NeRFTrainer(fcfg, precision=prec, device=dev, overlap=ov)
kw = dict(near=bounds[:, :1], far=bounds[:, 1:])
for i in range(3):
    tr.step(poses[i:i + 1], ffocal, fimg, **kw)
K = int(sys.argv[4]) if len(sys.argv) > 4 else 4
if mode == "graph":
    tr.capture_step(poses[0:K], ffocal, fimg, n_steps=K, **kw)
torch.cuda.synchronize()
t0 = time.perf_counter()
n_done = 0
for i in range(steps // K if mode == "graph" else steps):
    if mode == "graph":
        tr.replay_step(poses[(K * i) % 40:(K * i) % 40 + K], ffocal, **kw)
        n_done += K
    else:
        tr.step(poses[(3 + i) % 40][None], ffocal, fimg, **kw)
        n_done += 1
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / n_done
print(f"fern {prec} {mode} K={K if mode == 'graph' else 1} overlap={tr.overlap} "
      f"main-priority={torch.cuda.current_stream().priority}: {1e3 * dt:.4f} ms/step, "
      f"{tr.R / dt:.1f} rays/s", flush=True)
