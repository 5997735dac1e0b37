#!/usr/bin/env python
"""Diagnostic: bf16 fused step with the coarse backward on the side stream vs serial. Compare the fine pass's backward
workspace sections (point-major bf16 dZ rows) and saved activations between the two schedules."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden"), str(ROOT / "tests")]
import yanerf_boot  # noqa: E402,F401
from test_gpu_trainer import make_trainer, t  # noqa: E402
from yanerf_amd import ops  # noqa: E402

DEV = "cuda:0"


def run(overlap, g, img, R):
    tr = make_trainer("bf16", g["seeds"], n_rays=R, overlap=overlap)
    draws = dict(pixel_ids=t(g["pixel_ids"], torch.int64), jitter_u=t(g["jitter_u"]),
                 noise=[t(g["noise_coarse"]), t(g["noise_fine"])], pdf_u=t(g["pdf_u"]))
    with ops.injected_randomness(**draws):
        tr.step(t(g["pose"]), t(g["focal"]), img)
    torch.cuda.synchronize()
    return tr


def main():
    g = dict(np.load(ROOT / "tests/golden/train_step_lego.npz"))
    R = int(g["n_rays"])
    img = torch.zeros(1, 800, 800, 3, device=DEV)
    img.view(1, -1, 3)[0, torch.as_tensor(g["pixel_ids"][0], device=DEV)] = t(g["gt_rgb"])
    a = run(False, g, img, R)
    for trial in range(3):
        b = run("both", g, img, R)
        for k in range(2):
            N = R * a.passes[k].P
            Npad = (N + 127) // 128 * 128
            wa = a.ws[k].view(torch.int16)[: 2448 * Npad].cpu().numpy()
            wb = b.ws[k].view(torch.int16)[: 2448 * Npad].cpu().numpy()
            secs = {"dz": (0, 2048 * Npad, 256), "dy": (2048 * Npad, 2304 * Npad, 256),
                    "dzc": (2304 * Npad, 2432 * Npad, 128), "du": (2432 * Npad, 2448 * Npad, 16)}
            for name, (lo, hi, w) in secs.items():
                d = np.nonzero(wa[lo:hi] != wb[lo:hi])[0]
                if name == "du":
                    d = d[np.isin(d % 16, [0, 1, 2, 8])]
                if d.size:
                    pts = np.unique((d % (hi - lo if name != "dz" else 256 * Npad)) // w)
                    feats = np.unique(d % w)
                    print(f"trial {trial} pass {k} {name}: {d.size} differ; points {pts[:24]} ({pts.size}) "
                          f"features {feats[:24]} ({feats.size})")
            sa = a.passes[k].saved.cpu().numpy()
            sb = b.passes[k].saved.cpu().numpy()
            print(f"trial {trial} pass {k}: saved bytes differ: {(sa != sb).sum()}")
            ga = torch.cat([p.grad.reshape(-1) for p in a.models[k].parameters()]).cpu().numpy()
            gb = torch.cat([p.grad.reshape(-1) for p in b.models[k].parameters()]).cpu().numpy()
            print(f"trial {trial} pass {k}: grads differ: {(ga != gb).sum()}")
    print("done")


if __name__ == "__main__":
    main()
