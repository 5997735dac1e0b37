#!/usr/bin/env python
"""Does the REFERENCE itself collapse to the transparent solution on the procedural scene at its own initialisation?
(with the density-layer bias zeroed at init, nerf_mlp.py:69-71, this scene trains into "no density
anywhere, every ray's colour on its background-opacity last sample"; measured on the fused HIP trainer, round 4.)

Runs the reference's own training loop on the CPU, in this build container only (it imports /root/reference with the
golden generator's stand-ins): the registry pipeline from lego.yml at the scene's size, torch.optim.Adam with the runner
schedule (runners/apis.py:66-89; warm-up and decay shortened as tools/psnr_synthetic.py does), the scene's training
views in DeviceImageSet.epoch_order, then the reference's EVALUATION render of the test views: test PSNR of the mean
MSE (runners/utils.py:270-283) and `rays_before_far_plane`, the share of test-view-0 rays whose fine depth lies before
0.95 x far (the collapse measure tools/psnr_synthetic.py reports for the HIP trainer). The initial weights are the
reference's own seeded init, which the fused trainer reproduces bit for bit under the same seed (checked here), so the
HIP run of the same configuration (tools/psnr_synthetic.py --size --rays --steps --seed, reference init) starts from
the same network. One JSON line.

    python tools/reference_collapse_run.py --size 50 --rays 1024 --steps 500 --seed 42 [--threads 6]
"""
from __future__ import annotations

import argparse
import json
import math
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests" / "golden"))
sys.path.insert(0, str(ROOT / "tools"))
sys.path.append(str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=50)
    ap.add_argument("--rays", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--threads", type=int, default=6)
    ap.add_argument("--density-bias", type=float, default=None, help="density-layer bias at init (reference: 0)")
    a = ap.parse_args()
    import make_golden as MG  # the reference import (stand-ins for its missing third-party modules)
    import torch
    torch.set_num_threads(a.threads)
    import yanerf_boot  # noqa: F401
    from synthetic_scene import write_scene
    from yanerf_amd.datasets import BlenderDataset, DeviceImageSet
    from yanerf_amd.pipelines.models import MODELS as OUR_MODELS
    from yanerf.runners.utils import create_lr_scheduler, warmup_lr_scheduler

    cfg = MG.Config.fromfile(str(MG.REF / "configs/nerf/lego.yml"))
    pcfg = cfg.pipeline
    pcfg.ray_sampler.image_height = pcfg.ray_sampler.image_width = a.size
    pcfg.ray_sampler.n_rays_per_image_sampled_from_mask = a.rays
    runner = cfg.runner
    runner["warmup_steps"] = max(1, a.steps // 10)  # as tools/psnr_synthetic.run
    runner["lr_decay_iters"] = a.steps * 1.25
    with tempfile.TemporaryDirectory() as tmp:
        data = write_scene(Path(tmp) / "synthetic", a.size, 40, 8, device="cpu")
        train = DeviceImageSet(BlenderDataset(str(data), "train"), "cpu")
        test = DeviceImageSet(BlenderDataset(str(data), "test", test_skip=1), "cpu")
    torch.manual_seed(a.seed)
    pipe = MG.PIPELINES.build(pcfg)
    # the fused trainer builds its two NeRFMLPs under torch.manual_seed(seed) (train.NeRFTrainer): same init
    with torch.random.fork_rng(devices=[]):
        torch.manual_seed(a.seed)
        mc = dict(pcfg.model)
        ours = [OUR_MODELS.build(dict(mc)) for _ in range(2)]
    for f, m in zip(pipe.implicit_functions, ours):
        sd_ref, sd_our = f._fn.state_dict(), m.state_dict()
        assert all(torch.equal(sd_ref[k], sd_our[k]) for k in sd_ref), "seeded init differs from the fused trainer's"
    if a.density_bias is not None:
        with torch.no_grad():
            for f in pipe.implicit_functions:
                f._fn.density_layer.bias.fill_(a.density_bias)
    opt = torch.optim.Adam([{"params": pipe.parameters(), "init_lr": runner.init_lr}], lr=runner.init_lr,
                           weight_decay=runner.weight_decay)
    sched = create_lr_scheduler(opt, runner)
    pipe.train()
    t0 = time.perf_counter()
    it, epoch = 0, 0
    while it < a.steps:
        for i in train.epoch_order(epoch, seed=42):
            if it >= a.steps:
                break
            pose, focal, img, _, _ = train.item(i)
            sched(iter=it)
            if runner["warmup_steps"] > 0 and it <= runner["warmup_steps"]:
                warmup_lr_scheduler(opt, it, runner["warmup_steps"], runner["warmup_lr"])
            opt.zero_grad()
            preds = pipe(poses=pose, focal_lengths=focal, image_rgb=img, evaluation_mode=MG.EvaluationMode.TRAINING)
            preds["objective"].mean().backward()
            opt.step()
            it += 1
            if it % 50 == 0:
                print(f"step {it}/{a.steps} {time.perf_counter() - t0:.0f} s objective "
                      f"{float(preds['objective'].mean()):.5f}", file=sys.stderr, flush=True)
        epoch += 1
    dt = time.perf_counter() - t0
    pipe.eval()
    mse_f, mse_c, surface = [], [], None
    with torch.no_grad():
        for i in range(len(test)):
            pose, focal, img, _, _ = test.item(i)
            preds = pipe(poses=pose, focal_lengths=focal, image_rgb=img, image_height=test.H, image_width=test.W,
                         evaluation_mode=MG.EvaluationMode.EVALUATION)
            mse_f.append(float(preds["loss_rgb_mse"]))
            mse_c.append(float(preds["loss_prev_stage_rgb_mse"]))
            if i == 0:
                depth = preds["rendered_depths"].reshape(-1)
                surface = float((depth < 0.95 * float(pcfg.ray_sampler.max_depth)).float().mean())
    mf, mc_ = sum(mse_f) / len(mse_f), sum(mse_c) / len(mse_c)
    print(json.dumps({"implementation": "reference (CPU, its own training loop)", "steps": a.steps,
                      "rays_per_step": a.rays, "size": a.size, "seed": a.seed, "density_bias_init": a.density_bias,
                      "train_s": round(dt, 1), "test_psnr_fine": round(-10 * math.log10(mf), 3),
                      "test_psnr_coarse": round(-10 * math.log10(mc_), 3), "test_views": len(test),
                      "rays_before_far_plane": round(surface, 4), "threads": a.threads}), flush=True)


if __name__ == "__main__":
    main()
