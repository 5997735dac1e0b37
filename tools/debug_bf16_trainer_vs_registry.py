#!/usr/bin/env python
"""Diagnostic: the fused trainer step vs the registry pipeline (same injected draws) in bf16 -- where do their
gradients differ, and is either path run-to-run deterministic?"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden"), str(ROOT / "tests")]
import yanerf_boot  # noqa: E402,F401
from test_gpu_trainer import lego_cfg, make_trainer, pipeline_state, t  # noqa: E402
from yanerf_amd import ops  # noqa: E402
from yanerf_amd.pipelines import PIPELINES  # noqa: E402
from yanerf_amd.pipelines.utils import EvaluationMode  # noqa: E402

DEV = "cuda:0"


def main(precision="bf16"):
    g = dict(np.load(ROOT / "tests/golden/train_step_lego.npz"))
    R = int(g["n_rays"])
    cfg = lego_cfg().pipeline
    cfg.ray_sampler.n_rays_per_image_sampled_from_mask = R
    cfg.model.precision = precision
    img = torch.zeros(1, 800, 800, 3, device=DEV)
    img.view(1, -1, 3)[0, torch.as_tensor(g["pixel_ids"][0], device=DEV)] = t(g["gt_rgb"])

    def draws():
        return dict(pixel_ids=t(g["pixel_ids"], torch.int64), jitter_u=t(g["jitter_u"]),
                    noise=[t(g["noise_coarse"]), t(g["noise_fine"])], pdf_u=t(g["pdf_u"]))

    def registry():
        pipe = PIPELINES.build(cfg).to(DEV)
        pipe.load_state_dict(pipeline_state(g["seeds"]), strict=False)
        pipe.train()
        with ops.injected_randomness(**draws()):
            preds = pipe(poses=t(g["pose"]), focal_lengths=t(g["focal"]), image_rgb=img,
                         evaluation_mode=EvaluationMode.TRAINING)
        preds["objective"].mean().backward()
        torch.cuda.synchronize()
        return {f"{i}:{k}": p.grad.detach().cpu().numpy().copy() for i, f in enumerate(pipe.implicit_functions)
                for k, p in f._fn.named_parameters()}

    def fused(overlap=None):
        tr = make_trainer(precision, g["seeds"], n_rays=R, overlap=overlap)
        with ops.injected_randomness(**draws()):
            tr.step(t(g["pose"]), t(g["focal"]), img)
        torch.cuda.synchronize()
        return {f"{i}:{k}": p.grad.detach().cpu().numpy().copy() for i, m in enumerate(tr.models)
                for k, p in m.named_parameters()}

    runs = {"reg_a": registry(), "reg_b": registry(), "fused_a": fused(), "fused_b": fused(),
            "fused_serial": fused(False)}
    base = runs["reg_a"]
    for name, r in runs.items():
        for k, v in r.items():
            ref = base[k]
            d = np.abs(v - ref)
            bad = d > 1e-3 * max(np.abs(ref).max(), 1e-30)
            if bad.any():
                idx = np.argwhere(bad)
                rows = np.unique(idx[:, 0]) if idx.shape[1] > 1 else idx[:, 0]
                cols = np.unique(idx[:, 1]) if idx.shape[1] > 1 else []
                print(f"{name} vs reg_a {k}: {bad.sum()} bad, max {d.max():.3e}, rows {rows[:20]} cols {cols[:40]}"
                      f" finite={np.isfinite(v).all()}")
    print("done")


if __name__ == "__main__":
    main(*(sys.argv[1:]))
