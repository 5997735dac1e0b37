"""Golden vectors for the conditional NeRFMLP (latent_dim > 0, global codes), made by running the REFERENCE model.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_golden_conditional.py

The reference's tests/configs/pipelines/models/nerf_conditional_mlp.yml architecture (Lego MLP + latent_dim 2) with
seeded weights (weights.make_nerf_mlp_params), a batch of 3 elements with their own codes ([B, 1, latent_dim], as the
IdentityMapper feature extractor stacks them): outputs, parameter gradients and code gradients for fixed upstream
gradients -> tests/golden/mlp_conditional.npz.
"""
from __future__ import annotations

import os
import sys
import types
import zlib
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REF = Path(os.environ.get("YANERF_REFERENCE", "/root/reference"))
sys.path.insert(0, str(HERE / "_stubs"))
sys.path.insert(0, str(REF))
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parents[1]))  # the oracle (test infrastructure) for the input-margin check

import torch  # noqa: E402

_six = types.ModuleType("torch._six")
_six.string_classes = (str, bytes)
sys.modules.setdefault("torch._six", _six)

from weights import LEGO_ARCH, checksum, make_nerf_mlp_params  # noqa: E402

from yanerf.pipelines.models import MODELS  # noqa: E402
from yanerf.utils.config import Config  # noqa: E402

ARCH = dict(LEGO_ARCH, latent_dim=2)


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def main():
    cfg = dict(type="NeRFMLP", **ARCH, harmonic_functions_xyz_append_intput=True,
               harmonic_functions_dir_append_intput=True, input_xyz=True, input_dir=True)
    model = MODELS.build(Config(dict(model=cfg)).model)
    params = make_nerf_mlp_params(ARCH, 77)
    assert set(model.state_dict().keys()) == set(params.keys())
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    # inputs whose trunk pre-activations all stay >= 1e-6 away from the ReLU kink: the kernels fold a code into the
    # bias (a different fp32 summation order than the reference's concatenated matmul), and a pre-activation within
    # a few ulp of 0 may take the other side of the kink and flip a whole unit's gradient (measured: |z| = 5.6e-8).
    from oracle import nerf_oracle as O
    arch_o = O.MLPArch.from_dict(ARCH)
    B, R, P = 3, 4, 24
    for gseed in range(9, 200):
        g = torch.Generator().manual_seed(gseed)
        o = torch.randn(B, R, 1, 3, generator=g) * 0.5 + torch.tensor([0.0, 0.0, 4.0])
        dvec = torch.randn(B, R, 1, 3, generator=g)
        dvec[..., 2] -= 1.5
        t = torch.sort(torch.rand(B, R, 1, P, generator=g) * 4.0 + 2.0, dim=-1)[0]
        codes = (torch.randn(B, 1, ARCH["latent_dim"], generator=g) * 2.0).requires_grad_(True)
        margin = np.inf
        for b in range(B):
            _, _, cache = O.nerf_mlp_forward(params, arch_o, o[b].numpy(), dvec[b].numpy(), t[b].numpy(),
                                             code=codes[b].detach().numpy().reshape(-1))
            for li in range(ARCH["n_layers"]):
                z = cache.layer_in[li] @ params[f"xyz_encoder.mlp.{li}.0.weight"].T + \
                    params[f"xyz_encoder.mlp.{li}.0.bias"]
                margin = min(margin, float(np.abs(z).min()))
        if margin >= 1e-6:
            break
    print("input seed", gseed, "min |pre-activation|", margin)
    res = model(o, dvec, t, global_codes=codes)
    sig, rgb = res["rays_densities"], res["rays_features"]
    gs = torch.randn(sig.shape, generator=g)
    gc = torch.randn(rgb.shape, generator=g)
    model.zero_grad()
    ((sig * gs).sum() + (rgb * gc).sum()).backward()
    d = dict(origins=np32(o), directions=np32(dvec), lengths=np32(t), codes=np32(codes), sigma=np32(sig),
             rgb=np32(rgb), g_sigma=np32(gs), g_rgb=np32(gc), g_codes=np32(codes.grad), seed=np.int64(77),
             checksum=checksum(params))
    for name, p in model.named_parameters():
        gr = np32(p.grad)
        if gr.size <= 4096:
            d[f"grad:{name}"] = gr
        else:
            rng = np.random.Generator(np.random.PCG64(zlib.crc32(name.encode())))
            idx = rng.choice(gr.size, size=512, replace=False)
            d[f"gradidx:{name}"] = idx.astype(np.int64)
            d[f"gradval:{name}"] = gr.reshape(-1)[idx]
            d[f"gradsum:{name}"] = np.array([gr.astype(np.float64).sum(), np.linalg.norm(gr.astype(np.float64))])
    # the mismatch error (nerf_mlp.py:162-163)
    try:
        model(o, dvec, t, global_codes=torch.randn(B, 1, 3))
        d["error_on_bad_code"] = np.array(False)
    except ValueError:
        d["error_on_bad_code"] = np.array(True)
    np.savez_compressed(HERE / "mlp_conditional.npz", **d)
    print("wrote", HERE / "mlp_conditional.npz")


if __name__ == "__main__":
    main()
