#!/usr/bin/env python
"""Dump the fp32 coarse stage of the gated evaluation renders, stage by stage, for offline comparison with the reference
run in the HIP kernels' summation order (make_golden.hip_order_model): the rays (the registry RaySampler's EVALUATION
bundle), the coarse MLP's saved activations (harmonic embedding, H_0..H_7 post-ReLU, Y: the training-forward rows of
csrc/mlp.hip), sigma / rgb and the composite weights. Development tool (GPU); writes gpurun_out/coarse_dump/<case>.npz.

    python tools/dump_coarse_stage.py [fp32|fp32x3]
"""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "tests" / "golden")]
import yanerf_boot  # noqa: E402,F401
from parity_gates import hip_relu_masks  # noqa: E402,F401  (the saved-row layout mirror)
from weights import LEGO_ARCH, load_trained_params, make_nerf_mlp_params  # noqa: E402

DEV = "cuda:0"


def saved_rows(saved, n_points, n_layers=8):
    npad = -(-n_points // 64) * 64
    units = (npad * 4 + 255) // 256
    if units % 2 == 0:
        units += 1
    ld = units * 256 // 4
    rows = 64 + 256 * n_layers + 256 + 32 + 128
    return saved[: rows * ld * 4].view(torch.float32).view(rows, ld)[:, :n_points].cpu().numpy()


def main():
    from yanerf_amd import _C, ops
    from yanerf_amd.pipelines import PIPELINES
    from yanerf_amd.pipelines.utils import EvaluationMode
    from yanerf_amd.utils.config import Config
    from scene import forward_pose, synthetic_pose
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    out = ROOT / "gpurun_out" / "coarse_dump"
    out.mkdir(parents=True, exist_ok=True)
    lego = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml")).pipeline
    fern = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/fern.yml")).pipeline
    g_tr = np.load(ROOT / "tests/golden/render_trained.npz")
    cases = {
        "lego": (lego, [make_nerf_mlp_params(LEGO_ARCH, s) for s in (11, 12)], synthetic_pose(30.0, -30.0, 4.0)[None],
                 [1111.1111], 16, 16, 800, {}),
        "trained": (lego, load_trained_params(), g_tr["pose"], g_tr["focal"], 25, 25, 100, {}),
        "fern": (fern, [make_nerf_mlp_params(LEGO_ARCH, s) for s in (41, 42)], forward_pose()[None], [407.6], 9, 12,
                 None, dict(min_depth=torch.tensor([[1.3125]], device=DEV), max_depth=torch.tensor([[7.25]], device=DEV))),
    }
    L = _C.lib()
    for name, (pcfg, params, pose, focal, H, W, hw, bounds) in cases.items():
        cfg = Config(dict(p=dict(pcfg))).p
        cfg.model.precision = prec
        if hw is not None:
            cfg.ray_sampler.image_height = cfg.ray_sampler.image_width = hw
        pipe = PIPELINES.build(cfg).to(DEV)
        for f, p in zip(pipe.implicit_functions, params):
            f._fn.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
        pipe.eval()
        pose_t = torch.as_tensor(np.asarray(pose, np.float32), device=DEV).reshape(1, 3, 4)
        focal_t = torch.as_tensor(np.asarray(focal, np.float32), device=DEV).reshape(1)
        with torch.no_grad():
            rb = pipe.ray_sampler(pose_t, focal_t, evaluation_mode=EvaluationMode.EVALUATION, image_height=H,
                                  image_width=W, **bounds)
        R = H * W
        o, d, z = (x.reshape(R, -1).contiguous() for x in (rb.origins, rb.directions, rb.lengths))
        P = z.shape[1]
        model = pipe.implicit_functions[0]._fn
        spec = model.spec()
        packed = ops.mlp_pack(spec, model.hip_params())
        saved = torch.empty(L.yanerf_mlp_saved_bytes(ctypes.byref(spec.desc()), spec.precision, R * P),
                            dtype=torch.uint8, device=DEV)
        sigma = torch.empty(R * P, device=DEV)
        rgb = torch.empty(R * P, 3, device=DEV)
        _C.check(L.yanerf_mlp_forward(ctypes.byref(spec.desc()), spec.precision, ops._p(packed), ops._p(o), ops._p(d),
                                      ops._p(z), R, P, ops._p(sigma), ops._p(rgb), ops._p(saved), ops._stream()), "fwd")
        march = pipe.renderer._raymarcher
        with torch.no_grad():
            fo = model(o, d, z)
            _, _, _, w, _ = march(**fo, ray_lengths=z, ray_directions=d)
        torch.cuda.synchronize()
        rows = saved_rows(saved, R * P)
        np_ = min(R * P, 1024)  # the activations of the first 1,024 points (the whole tile set would be ~100 MB)
        np.savez_compressed(out / f"{name}_{prec}.npz", o=o.cpu().numpy(), d=d.cpu().numpy(), z=z.cpu().numpy(),
                            pe_all=rows[:64].T.copy(), pe=rows[:64, :np_].T.copy(),
                            h=rows[64:64 + 8 * 256, :np_].reshape(8, 256, -1).transpose(0, 2, 1).copy(),
                            y=rows[64 + 8 * 256:64 + 9 * 256, :np_].T.copy(), sigma=sigma.cpu().numpy(),
                            sigma_eval=fo["rays_densities"].reshape(-1).cpu().numpy(), rgb=rgb.cpu().numpy(),
                            w=w.reshape(R, P).cpu().numpy())
        print(name, prec, "dumped", R, P, flush=True)


if __name__ == "__main__":
    main()
