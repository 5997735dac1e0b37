"""Shared parity gate for end-to-end (two-pass) renders.

The reference's sample_pdf is ill-conditioned where the coarse weights put (almost) no mass: its normalised pdf there
is ~1e-5, exactly at the `denom < 1e-5` branch (renderers/utils.py:128-129), and a bin whose pdf is 1e-5..1e-3 turns
an ulp of the CDF into a large move of the sample inside the bin. So an ulp-level difference in the coarse weights can
move a fine sample by up to a bin width, and with it the fine render. The gate therefore splits the rays by their
refined depths:

  * rays whose refined depths (computed from OUR coarse weights) equal the ones computed from the REFERENCE's coarse
    weights (<= z_tol) must match the reference strictly (RGB <= strict, depth <= strict_depth);
  * every other ray must match the reference's fine stage evaluated at OUR refined depths (the oracle's MLP +
    raymarcher on those rays, `fine_at`) just as strictly: its difference from the reference is then fully accounted
    for by the depths it was given, which the coarse-stage and sample_pdf parity tests pin separately.

Nothing is gated statistically: every element either matches the reference or is shown to be the reference's own
function of the depths the coarse stage produced.
"""
from __future__ import annotations

import numpy as np


def oracle_fine_at(O, params_f, arch, origins, directions, raymarch_opts, bg=(0.0, 0.0, 0.0)):
    """fine_at(rows, z) -> (rgb [n,3], depth [n]): the oracle's fine MLP + raymarcher on rays `rows` at depths z."""
    origins = np.asarray(origins, np.float32).reshape(-1, 3)
    directions = np.asarray(directions, np.float32).reshape(-1, 3)

    def fine_at(rows, z):
        o, d = origins[rows], directions[rows]
        s, c, _ = O.nerf_mlp_forward(params_f, arch, o, d, z)
        f, dep, _, _, _ = O.raymarch_forward(s, c, z, d, raymarch_opts, default_bg=bg)
        return f, np.asarray(dep).reshape(-1)

    return fine_at


def split_gate(rgb, rgb_ref, z, z_ref, depth=None, depth_ref=None, *, fine_at=None, strict=1e-5, strict_depth=1e-4,
               z_tol=2e-5, tag=""):
    R = len(z)
    rgb = np.asarray(rgb, np.float64).reshape(R, -1)
    rgb_ref = np.asarray(rgb_ref, np.float64).reshape(R, -1)
    z, z_ref = np.asarray(z, np.float32).reshape(R, -1), np.asarray(z_ref, np.float32).reshape(R, -1)
    zerr = np.abs(z.astype(np.float64) - z_ref).max(axis=-1)
    same = zerr <= z_tol
    flip = np.nonzero(~same)[0]
    err = np.abs(rgb - rgb_ref).max(axis=-1)
    report = dict(rays=R, rays_with_other_depths=int(flip.size), rgb_above_1e4=int((err > 1e-4).sum()),
                  max_rgb_err_same_depths=float(err[same].max()) if same.any() else 0.0,
                  max_rgb_err_other_depths_vs_reference=float(err[flip].max()) if flip.size else 0.0)
    if depth is not None:
        depth = np.asarray(depth, np.float64).reshape(-1)
        derr = np.abs(depth - np.asarray(depth_ref, np.float64).reshape(-1))
        report["max_depth_err_same_depths"] = float(derr[same].max()) if same.any() else 0.0
    if flip.size and fine_at is not None:
        f_o, d_o = fine_at(flip, z[flip])
        e2 = np.abs(rgb[flip] - np.asarray(f_o, np.float64).reshape(flip.size, -1)).max(axis=-1)
        report["max_rgb_err_other_depths_vs_oracle_at_our_depths"] = float(e2.max())
        if depth is not None:
            report["max_depth_err_other_depths_vs_oracle_at_our_depths"] = float(
                np.abs(depth[flip] - np.asarray(d_o, np.float64)).max())
    print(f"split_gate {tag}: {report}")
    assert report["max_rgb_err_same_depths"] <= strict, report
    if depth is not None:
        assert report["max_depth_err_same_depths"] <= strict_depth, report
    if flip.size:
        assert fine_at is not None, f"{flip.size} rays with other refined depths and no fine_at to account for them"
        assert report["max_rgb_err_other_depths_vs_oracle_at_our_depths"] <= strict, report
        if depth is not None:
            assert report["max_depth_err_other_depths_vs_oracle_at_our_depths"] <= strict_depth, report
    return report
