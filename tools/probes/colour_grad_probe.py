"""Probe: colour-layer weight gradient (direction and hidden columns) vs the oracle for one (precision, R, P),
printing the relative L2 per column block and the worst rows. Development aid for the ragged-ray test."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "tests" / "golden"), str(ROOT / "tools")]
import yanerf_boot  # noqa: F401,E402
from oracle import nerf_oracle as O  # noqa: E402
from weights import LEGO_ARCH, make_nerf_mlp_params  # noqa: E402
from yanerf_amd.pipelines.models import MODELS  # noqa: E402

prec, R, P = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rng = np.random.default_rng(R * 1000 + P)
o = (rng.standard_normal((R, 3)) * 0.3 + [0, 0, 4]).astype(np.float32)
d = rng.standard_normal((R, 3)).astype(np.float32)
z = np.sort(rng.uniform(2, 6, (R, P)).astype(np.float32), -1)
gs = rng.standard_normal((R, P, 1)).astype(np.float32)
gr = rng.standard_normal((R, P, 3)).astype(np.float32)
m = MODELS.build(dict(type="NeRFMLP", **LEGO_ARCH, precision=prec)).to("cuda:0")
params = make_nerf_mlp_params(LEGO_ARCH, 5)
m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
arch = O.MLPArch.from_dict(LEGO_ARCH)
sig_o, rgb_o, cache = O.nerf_mlp_forward(params, arch, o, d, z)
ref = O.nerf_mlp_backward(params, arch, cache, gs.reshape(sig_o.shape), gr.reshape(rgb_o.shape))
t = lambda x: torch.as_tensor(x, device="cuda:0")
out = m(t(o), t(d), t(z))
((out["rays_densities"] * t(gs)).sum() + (out["rays_features"] * t(gr)).sum()).backward()
for name, p in m.named_parameters():
    w = p.grad.detach().float().cpu().numpy().astype(np.float64)
    r = np.asarray(ref[name], np.float64).reshape(w.shape)
    rel = np.linalg.norm(w - r) / max(np.linalg.norm(r), 1e-30)
    line = f"{prec} R={R} P={P} {name}: rel {rel:.2e}"
    if name == "color_layer.0.weight":
        for cols in (slice(256, None), slice(0, 256)):
            e = np.abs(w[:, cols] - r[:, cols])
            line += f" | cols {cols.start}: rel {np.linalg.norm(e) / np.linalg.norm(r[:, cols]):.2e}"
            line += f" worst rows {np.argsort(-e.max(1))[:4].tolist()} cols {np.argsort(-e.max(0))[:4].tolist()}"
    print(line, flush=True)
