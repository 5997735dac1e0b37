#!/usr/bin/env python
"""Diagnostic: does any MLP kernel write past the end of its workspace / saved buffer? Every buffer of the fused
trainer gets a guard region filled with a pattern; one training step per precision; report guard bytes changed."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden"), str(ROOT / "tests")]
import yanerf_boot  # noqa: E402,F401
from scene import synthetic_pose  # noqa: E402
from yanerf_amd.train import NeRFTrainer  # noqa: E402
from yanerf_amd.utils.config import Config  # noqa: E402

DEV = "cuda:0"
GUARD = 1 << 20


def guarded(t):
    big = torch.full((t.numel() + GUARD,), 0x5A, dtype=torch.uint8, device=DEV)
    return big, big[: t.numel()]


def main():
    cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml"))
    for precision in ("bf16", "fp32", "fp32x3"):
        for n_rays in (48, 4096):
            tr = NeRFTrainer(cfg.pipeline, precision=precision, device=DEV, n_rays=n_rays, overlap=False)
            bigs = {}
            for k in range(2):
                b, v = guarded(tr.ws[k])
                tr.ws[k] = v
                bigs[f"ws{k}"] = b
                b, v = guarded(tr.passes[k].saved)
                tr.passes[k].saved = v
                bigs[f"saved{k}"] = b
            pose = torch.from_numpy(synthetic_pose(10.0, -30.0, 4.0)).float()[None].to(DEV)
            img = torch.rand(1, 800, 800, 3, device=DEV)
            tr.step(pose, torch.tensor([1111.111], device=DEV), img)
            torch.cuda.synchronize()
            for name, b in bigs.items():
                n = b.numel() - GUARD
                g = b[n:]
                bad = (g != 0x5A).nonzero()
                if bad.numel():
                    print(f"{precision} R={n_rays} {name}: {bad.numel()} guard bytes written, first at +{int(bad[0])}, "
                          f"last at +{int(bad[-1])} (buffer {n} bytes)")
            print(f"{precision} R={n_rays} checked", flush=True)


if __name__ == "__main__":
    main()
