#!/usr/bin/env python
"""Which trainings of the procedural scene keep a density field and which collapse to the transparent solution (no
density anywhere, every ray's colour on its background-opacity last sample: the failure the reference's own comment
at nerf_mlp.py:69-71 warns about). One scene, several (seed, density-bias-at-init) runs of the fused fp32 trainer;
one JSON line per run (tools/psnr_synthetic.run). Development tool.

    python tools/density_collapse_probe.py [--steps 1500] [--save-best PATH]
"""
import argparse
import json
import sys
import tempfile
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
from psnr_synthetic import run  # noqa: E402
from synthetic_scene import write_scene  # noqa: E402

CONFIGS = [(42, None), (1, None), (7, None), (42, 0.5), (42, 1.0), (7, 1.0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--save-dir", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    with tempfile.TemporaryDirectory() as tmp:
        data = write_scene(Path(tmp) / "synthetic", 100, 40, 8, device="cuda")
        best = None
        for seed, bias in CONFIGS:
            save = Path(tmp) / f"trained_s{seed}_b{bias}.pth"
            r = run(data, "fp32", a.steps, dev, log=sys.stderr, save=save, seed=seed, density_bias=bias)
            print(json.dumps(r), flush=True)
            if r["rays_before_far_plane"] > 0.05 and (best is None or r["test_psnr_fine"] > best[0]["test_psnr_fine"]):
                best = (r, save)
        if a.save_dir and best is not None:  # the best non-collapsed run's checkpoint (one file: gpurun_out is capped)
            import shutil
            shutil.copy(best[1], Path(a.save_dir) / "trained_best.pth")
            print(json.dumps({"saved": best[1].name, **best[0]}), flush=True)


if __name__ == "__main__":
    main()
