#!/usr/bin/env python
"""A/B/C of the fused training step: serial, the whole coarse MLP backward on a side stream, or only its dW there (Lego config,
4096 rays, 64 + 128), interleaved in one process, per precision. Development tool; prints one JSON line."""
import json
import math
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import yanerf_boot  # noqa: E402,F401
from bench import synthetic_pose  # noqa: E402
from yanerf_amd.train import NeRFTrainer  # noqa: E402
from yanerf_amd.utils.config import Config  # noqa: E402


def main(steps=20, rounds=3):
    dev = torch.device("cuda:0")
    cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml"))
    image = torch.rand(1, 800, 800, 3, device=dev)
    poses = torch.stack([torch.from_numpy(synthetic_pose(th, -30.0)) for th in range(-180, 180, 9)]).to(dev)
    focal = torch.tensor([0.5 * 800 / math.tan(0.5 * 0.6911112)], device=dev)
    res = {}
    for prec in (sys.argv[1].split(",") if len(sys.argv) > 1 else ("fp32", "bf16", "fp32x3")):
        modes = (False, "both", "split", "early")
        trs = {ov: NeRFTrainer(cfg.pipeline, precision=prec, device=dev, overlap=ov) for ov in modes}
        best = {ov: float("inf") for ov in trs}
        for r in range(rounds):
            for ov, tr in trs.items():
                for i in range(3):
                    tr.step(poses[i][None], focal, image)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(steps):
                    tr.step(poses[i % len(poses)][None], focal, image)
                torch.cuda.synchronize()
                best[ov] = min(best[ov], (time.perf_counter() - t0) / steps * 1e3)
        res[prec] = {"ms_serial": round(best[False], 3), "ms_overlap": round(best["both"], 3),
                     "ms_split": round(best["split"], 3), "ms_early": round(best["early"], 3)}
        del trs
    print(json.dumps(res))


if __name__ == "__main__":
    main()
