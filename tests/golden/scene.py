"""Synthetic camera poses for golden vectors (test infrastructure).

A camera on a sphere around the origin, Blender/nerf_synthetic c2w convention,
followed by the reference's axis flip `pose @ diag(1,-1,-1,1)`
(reference yanerf/dataset/blender_dataset.py:58-60, 69).
"""
import math

import numpy as np


def synthetic_pose(theta_deg: float, phi_deg: float, radius: float) -> np.ndarray:
    def trans_t(t):
        return np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, t], [0, 0, 0, 1]], dtype=np.float64)

    def rot_phi(phi):
        c, s = math.cos(phi), math.sin(phi)
        return np.array([[1, 0, 0, 0], [0, c, -s, 0], [0, s, c, 0], [0, 0, 0, 1]], dtype=np.float64)

    def rot_theta(th):
        c, s = math.cos(th), math.sin(th)
        return np.array([[c, 0, -s, 0], [0, 1, 0, 0], [s, 0, c, 0], [0, 0, 0, 1]], dtype=np.float64)

    c2w = trans_t(radius)
    c2w = rot_phi(phi_deg / 180.0 * math.pi) @ c2w
    c2w = rot_theta(theta_deg / 180.0 * math.pi) @ c2w
    c2w = np.array([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], dtype=np.float64) @ c2w
    flip = np.diag([1.0, -1.0, -1.0, 1.0])
    return (c2w @ flip)[:3, :4].astype(np.float32)


def forward_pose(shift: float = 0.0) -> np.ndarray:
    """A forward-facing LLFF-style camera (identity rotation, looking down -z) used by the Fern-config goldens and
    tests: c2w [3, 4] with the camera at (0.1 + shift, -0.05, 4)."""
    pose = np.eye(4, dtype=np.float32)[:3].copy()
    pose[:, 3] = [0.1 + shift, -0.05, 4.0]
    return pose

