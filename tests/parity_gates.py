"""Shared parity gates for end-to-end (two-pass) renders.

The reference's sample_pdf replaces `denom < 1e-5` by 1 (renderers/utils.py:128-129): for rays with sum(w) ~ 1 the
empty bins' pdf sits exactly at that threshold, so an ulp-level difference in the coarse weights can move a fine sample
across a bin. The end-to-end gate therefore splits the rays by their refined depths:

  * rays whose refined depths (computed from OUR coarse weights) equal the ones computed from the REFERENCE's coarse
    weights (<= z_tol) must match the reference strictly (RGB <= strict, depth <= strict_depth);
  * every other ray is a flagged boundary flip: it may differ (bounded by `hard`), and the flips are counted.

So every element above the strict tolerance is accounted for by a ray whose refined samples differ.
"""
from __future__ import annotations

import numpy as np


def split_gate(rgb, rgb_ref, z, z_ref, depth=None, depth_ref=None, *, strict=1e-5, strict_depth=1e-4, z_tol=2e-5,
               hard=5e-4, hard_depth=5e-3, max_flip_frac=0.02, tag=""):
    rgb = np.asarray(rgb, np.float64).reshape(len(z), -1)
    rgb_ref = np.asarray(rgb_ref, np.float64).reshape(len(z), -1)
    z, z_ref = np.asarray(z, np.float64), np.asarray(z_ref, np.float64)
    zerr = np.abs(z - z_ref).max(axis=-1)
    same = zerr <= z_tol
    err = np.abs(rgb - rgb_ref).max(axis=-1)
    n_flip = int((~same).sum())
    report = dict(rays=len(z), flips=n_flip, above_1e4=int((err > 1e-4).sum()),
                  max_err_same_z=float(err[same].max()) if same.any() else 0.0,
                  max_err_flip=float(err[~same].max()) if n_flip else 0.0)
    if depth is not None:
        derr = np.abs(np.asarray(depth, np.float64).reshape(-1) - np.asarray(depth_ref, np.float64).reshape(-1))
        report["max_depth_err_same_z"] = float(derr[same].max()) if same.any() else 0.0
        report["max_depth_err_flip"] = float(derr[~same].max()) if n_flip else 0.0
    print(f"split_gate {tag}: {report}")
    assert report["max_err_same_z"] <= strict, report
    assert report["max_err_flip"] <= hard, report
    assert n_flip <= max_flip_frac * len(z) + 1, report
    # every element above 1e-4 lies on a flagged ray
    assert not np.any((err > 1e-4) & same), report
    if depth is not None:
        assert report["max_depth_err_same_z"] <= strict_depth, report
        assert report["max_depth_err_flip"] <= hard_depth, report
    return report
