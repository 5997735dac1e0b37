#!/usr/bin/env python
"""A/B of the fused bf16 step's main-stream priority: the step issued on a high-priority stream (priority -1) while the
trainer's side stream (the coarse backward under "early") keeps the default priority, against both at the default.
The hardware queue priority decides whose workgroups the command processor dispatches first when CUs free up, i.e.
whether the latency-critical main-stream kernels (composite, refinement, the fine forward) or the side stream's
backward get the freed CUs. Lego (4096 rays, 64 + 128) and Fern (1024 rays, 64 + 128), interleaved rounds.
Development tool (GPU); one JSON line.   python tools/prio_ab.py [bf16] [rounds]"""
import json
import math
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


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda:0")
    poses = torch.stack([torch.from_numpy(synthetic_pose(th, -30.0, 4.0)) for th in np.linspace(-180, 180, 40,
                                                                                        endpoint=False)]).float().to(dev)
    lego = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml")).pipeline
    fern = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/fern.yml")).pipeline
    fern.renderer.n_pts_per_ray_fine_training = 128
    cases = {
        "lego": (lego, torch.rand(1, 800, 800, 3, device=dev), torch.tensor([0.5 * 800 / math.tan(0.5 * 0.6911112)],
                                                                               device=dev), {}, 20),
        "fern": (fern, torch.rand(1, 378, 504, 3, device=dev), torch.tensor([407.56], device=dev),
                 dict(near=torch.tensor([[1.3]]), far=torch.tensor([[5.9]])), 40),
    }
    hi = torch.cuda.Stream(device=dev, priority=-1)
    res = {"precision": prec, "high_priority": hi.priority, "default_priority": torch.cuda.current_stream().priority}
    for name, (cfg, img, focal, kw, steps) in cases.items():
        trs = {m: NeRFTrainer(cfg, precision=prec, device=dev) for m in ("default", "hiprio")}
        best = {m: float("inf") for m in trs}
        for _ in range(rounds):
            for m, tr in trs.items():
                ctx = torch.cuda.stream(hi) if m == "hiprio" else torch.cuda.stream(torch.cuda.current_stream())
                with ctx:
                    for i in range(3):
                        tr.step(poses[i:i + 1], focal, img, **kw)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for i in range(steps):
                        tr.step(poses[i % 40][None], focal, img, **kw)
                    torch.cuda.synchronize()
                    best[m] = min(best[m], 1e3 * (time.perf_counter() - t0) / steps)
        res[name] = {m: round(v, 4) for m, v in best.items()}
        res[name]["overlap"] = trs["default"].overlap
        del trs
    print(json.dumps(res))


if __name__ == "__main__":
    main()
