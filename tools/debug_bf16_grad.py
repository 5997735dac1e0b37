"""Development probe: bf16-mode density-bias gradient (exactly sum(g_sigma) in the reference) at several sizes."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import yanerf_boot  # noqa: E402,F401
from yanerf_amd.pipelines.models import MODELS  # noqa: E402

dev = torch.device("cuda:0")
for prec in ("fp32", "bf16", "fp32x3"):
    for R, P in ((4, 64), (16, 64), (64, 64), (1024, 64), (3, 50)):
        torch.manual_seed(0)
        m = MODELS.build(dict(type="NeRFMLP", precision=prec)).to(dev)
        o = torch.randn(R, 3, device=dev) * 0.2 + torch.tensor([0.0, 0.0, 4.0], device=dev)
        d = torch.randn(R, 3, device=dev)
        z = torch.sort(torch.rand(R, P, device=dev) * 4 + 2, -1)[0]
        out = m(o, d, z)
        gs = torch.randn_like(out["rays_densities"])
        gr = torch.randn_like(out["rays_features"])
        ((out["rays_densities"] * gs).sum() + (out["rays_features"] * gr).sum()).backward()
        exact = gs.double().sum().item()
        got = m.density_layer.bias.grad.double().item()
        # intermediate_linear bias grad vs color-layer: compare the sum over points of dY
        print(f"{prec:7s} R={R:5d} P={P:3d} N={R*P:6d}: density bias grad {got:.6f} exact {exact:.6f} rel {abs(got-exact)/abs(exact):.2e}",
              flush=True)
