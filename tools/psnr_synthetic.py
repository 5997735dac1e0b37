"""Train-then-test PSNR on the procedural nerf_synthetic-format scene, per precision mode (GPU).

Writes the scene (tools/synthetic_scene.py), loads it through BlenderDataset into HBM (DeviceImageSet), trains the
fused NeRFTrainer with the Lego pipeline config (64 + 128 samples, 4096 rays per step, lego.yml's Adam schedule with
the warm-up shortened to 10 % of the run) and scores the test views as the reference's eval does (PSNR of the mean
per-image MSE, fine and coarse stage). Prints one JSON line.

    python tools/psnr_synthetic.py [--steps 2000] [--size 100] [--precisions fp32,fp32x3,bf16]
"""
from __future__ import annotations

import argparse
import json
import math
import sys
import tempfile
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
import yanerf_boot  # noqa: E402,F401
from synthetic_scene import write_scene  # noqa: E402
from yanerf_amd.datasets import BlenderDataset, DeviceImageSet  # noqa: E402
from yanerf_amd.train import NeRFTrainer  # noqa: E402
from yanerf_amd.utils.config import Config  # noqa: E402


def run(data_dir: Path, precision: str, steps: int, dev, n_rays=4096, log=None, save=None, seed=42, density_bias=None):
    train = DeviceImageSet(BlenderDataset(str(data_dir), "train"), dev)
    test = DeviceImageSet(BlenderDataset(str(data_dir), "test", test_skip=1), dev)
    cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml"))
    pcfg = cfg.pipeline
    pcfg.ray_sampler.image_height, pcfg.ray_sampler.image_width = train.H, train.W
    runner = dict(cfg.runner)
    runner["warmup_steps"] = max(1, steps // 10)
    runner["lr_decay_iters"] = steps * 1.25  # reach ~0.16x the initial rate at the end, like lego.yml's 200k/250k
    tr = NeRFTrainer(pcfg, precision=precision, device=dev, n_rays=n_rays, runner_cfg=runner, seed=seed)
    if density_bias is not None:  # the reference zeroes it (nerf_mlp.py:69-71, "fixme: Sometimes this is not enough")
        with torch.no_grad():
            for m in tr.models:
                m.density_layer.bias.fill_(density_bias)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    it = 0
    epoch = 0
    while it < steps:
        for i in train.epoch_order(epoch, seed=42):
            if it >= steps:
                break
            pose, focal, img, _, _ = train.item(i)
            tr.step(pose, focal, img)
            it += 1
            if log and it % 500 == 0:  # progress (a long GPU run must keep writing)
                print(f"step {it}/{steps} {time.perf_counter() - t0:.1f} s", file=log, flush=True)
        epoch += 1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ev = tr.evaluate(test)
    # the transparent solution: no density anywhere and every ray's colour on its last (background-opacity) sample,
    # the collapse the reference's density-bias comment warns about; measured as the share of test rays whose fine
    # depth lies before the far plane
    pose0, focal0, _, _, _ = test.item(0)
    _, _, depth = tr.render(pose0, focal0, test.H, test.W)
    surface = float((depth.reshape(-1) < 0.95 * float(pcfg.ray_sampler.max_depth)).float().mean())
    if save:  # reference-format checkpoint of the trained models (analysis of trained activations / gradients)
        from yanerf_amd import checkpoint
        checkpoint.save_checkpoint(str(save), tr, epoch=steps)
    res = {"precision": precision, "steps": steps, "rays_per_step": n_rays, "train_s": round(dt, 2),
           "rays_per_s": round(steps * n_rays / dt, 1), "test_psnr_fine": round(ev["loss_rgb_psnr"], 3),
           "test_psnr_coarse": round(ev["loss_prev_stage_rgb_psnr"], 3), "test_views": len(test),
           "rays_before_far_plane": round(surface, 4), "seed": seed, "density_bias_init": density_bias,
           "size": train.H}
    if log:
        print(json.dumps(res), file=log, flush=True)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--size", type=int, default=100)
    ap.add_argument("--precisions", default="fp32,fp32x3,bf16")
    ap.add_argument("--data", default=None, help="existing scene dir (default: generate into a temp dir)")
    ap.add_argument("--save", default=None, help="write the last run's trained checkpoint to this file")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--rays", type=int, default=4096, help="rays per step")
    ap.add_argument("--density-bias", type=float, default=None, help="density-layer bias at init (reference: 0)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    with tempfile.TemporaryDirectory() as tmp:
        data = Path(a.data) if a.data else write_scene(Path(tmp) / "synthetic", a.size, 40, 8, device="cuda")
        out = {"scene": f"procedural blobs, {a.size}x{a.size}, 40 train / 8 test views, Lego config 64+128",
               "runs": [run(data, p, a.steps, dev, n_rays=a.rays, log=sys.stderr, save=a.save, seed=a.seed,
                            density_bias=a.density_bias)
                        for p in a.precisions.split(",")]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
