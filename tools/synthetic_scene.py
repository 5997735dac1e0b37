"""A procedural nerf_synthetic-format scene for PSNR measurements (no dataset can be fetched here).

The radiance field is analytic: a few coloured Gaussian density blobs inside the unit cube. Ground-truth views are
rendered with the reference's own emission-absorption model (renderer.py:154-239: alpha = 1 - exp(-sigma * delta *
|d|), transmittance = exclusive cumprod, black background as in lego.yml) by dense quadrature (1024 samples on
[near, far]) in float64, with the reference's pinhole convention (ray_samplers/utils.py:12-24, ray_sampler.py:
296-314: integer pixel coordinates, principal point W/2, H/2, unnormalised directions). The views are written as
`transforms_{train,test}.json` + RGBA PNGs (alpha = opacity, as Blender renders), so training reads them back through
the BlenderDataset loader like the real Lego data.

    python tools/synthetic_scene.py OUT_DIR [--size 100] [--train 40] [--test 8]
"""
from __future__ import annotations

import argparse
import json
import math
from pathlib import Path

import numpy as np
import torch

CAMERA_ANGLE_X = 0.6911112070083618  # nerf_synthetic lego
BLOBS = [  # centre, radius, peak density, colour
    ((0.0, 0.0, 0.0), 0.45, 30.0, (0.9, 0.6, 0.2)),
    ((0.55, 0.3, 0.1), 0.25, 40.0, (0.2, 0.7, 0.9)),
    ((-0.5, -0.35, 0.25), 0.3, 35.0, (0.8, 0.2, 0.5)),
    ((0.1, -0.55, -0.45), 0.2, 50.0, (0.3, 0.9, 0.3)),
    ((-0.2, 0.5, -0.5), 0.22, 45.0, (0.95, 0.95, 0.9)),
]


def field(x: torch.Tensor):
    """sigma [...] and rgb [..., 3] at points x [..., 3] (view independent)."""
    centre = torch.tensor([b[0] for b in BLOBS], dtype=x.dtype, device=x.device)        # [B,3]
    inv2r2 = torch.tensor([1.0 / (2 * b[1] * b[1]) for b in BLOBS], dtype=x.dtype, device=x.device)
    peak = torch.tensor([b[2] for b in BLOBS], dtype=x.dtype, device=x.device)
    rgb = torch.tensor([b[3] for b in BLOBS], dtype=x.dtype, device=x.device)           # [B,3]
    d2 = ((x[..., None, :] - centre) ** 2).sum(-1)                                      # [...,B]
    s = peak * torch.exp(-d2 * inv2r2)
    sig = s.sum(-1)
    col = s @ rgb
    return sig, col / sig.clamp_min(1e-12)[..., None]


def pose_spherical(theta_deg: float, phi_deg: float, radius: float) -> np.ndarray:
    """Blender-convention camera-to-world (camera looks down its -z), as the nerf_synthetic transforms store it."""
    def tr(t):
        return np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, t], [0, 0, 0, 1]], np.float64)

    def rphi(p):
        c, s = math.cos(p), math.sin(p)
        return np.array([[1, 0, 0, 0], [0, c, -s, 0], [0, s, c, 0], [0, 0, 0, 1]], np.float64)

    def rth(t):
        c, s = math.cos(t), math.sin(t)
        return np.array([[c, 0, -s, 0], [0, 1, 0, 0], [s, 0, c, 0], [0, 0, 0, 1]], np.float64)

    c2w = rth(math.radians(theta_deg)) @ rphi(math.radians(phi_deg)) @ tr(radius)
    return np.array([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], np.float64) @ c2w


@torch.no_grad()
def render_view(c2w_blender: np.ndarray, H: int, W: int, near=2.0, far=6.0, n=1024, device="cpu"):
    """RGBA [H, W, 4] in [0, 1] of the analytic field."""
    pose = torch.tensor(c2w_blender @ np.diag([1.0, -1.0, -1.0, 1.0]), dtype=torch.float64, device=device)
    focal = 0.5 * W / math.tan(0.5 * CAMERA_ANGLE_X)
    y, x = torch.meshgrid(torch.arange(H, dtype=torch.float64, device=device),
                          torch.arange(W, dtype=torch.float64, device=device), indexing="ij")
    cam = torch.stack([(x - W / 2) / focal, (y - H / 2) / focal, torch.ones_like(x)], -1)
    d = cam @ pose[:3, :3].T
    o = pose[:3, 3].expand_as(d)
    t = torch.linspace(near, far, n, dtype=torch.float64, device=device)
    rgb = torch.zeros(H, W, 3, dtype=torch.float64, device=device)
    acc = torch.zeros(H, W, dtype=torch.float64, device=device)
    trans = torch.ones(H, W, dtype=torch.float64, device=device)
    delta = ((t[1] - t[0]) * d.norm(dim=-1))[..., None]                                  # [H,W,1]
    CH = 64  # samples per vectorised chunk; transmittance carried across chunks
    for k0 in range(0, n, CH):
        tk = t[k0:k0 + CH]
        s, c = field(o[..., None, :] + tk[:, None] * d[..., None, :])                    # [H,W,CH], [H,W,CH,3]
        a = 1.0 - torch.exp(-s * delta)
        tr = trans[..., None] * torch.cumprod(torch.cat([torch.ones_like(a[..., :1]), 1.0 - a[..., :-1]], -1), -1)
        w = a * tr
        rgb += (w[..., None] * c).sum(-2)
        acc += w.sum(-1)
        trans = tr[..., -1] * (1.0 - a[..., -1])
    return torch.cat([rgb, acc[..., None]], -1).clamp(0, 1).float().cpu().numpy()


def write_scene(out: Path, size=100, n_train=40, n_test=8, device=None):
    from PIL import Image
    device = device or ("cuda" if torch.cuda.is_available() else "cpu")
    out = Path(out)
    rng = np.random.default_rng(0)
    for split, n in (("train", n_train), ("test", n_test)):
        (out / split).mkdir(parents=True, exist_ok=True)
        frames = []
        for i in range(n):
            if split == "train":
                th, ph = rng.uniform(-180, 180), rng.uniform(-60, -10)
            else:
                th, ph = -180 + 360 * (i + 0.5) / n, -30.0
            c2w = pose_spherical(th, ph, 4.0)
            img = render_view(c2w, size, size, device=device)
            Image.fromarray((img * 255 + 0.5).astype(np.uint8), "RGBA").save(out / split / f"r_{i}.png")
            frames.append({"file_path": f"./{split}/r_{i}", "rotation": 0.0, "transform_matrix": c2w.tolist()})
        (out / f"transforms_{split}.json").write_text(json.dumps({"camera_angle_x": CAMERA_ANGLE_X,
                                                                   "frames": frames}))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--size", type=int, default=100)
    ap.add_argument("--train", type=int, default=40)
    ap.add_argument("--test", type=int, default=8)
    a = ap.parse_args()
    print(write_scene(Path(a.out), a.size, a.train, a.test))
