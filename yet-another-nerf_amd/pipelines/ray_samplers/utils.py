from enum import Enum

import torch

from ..utils import EvaluationMode, RayBundle  # noqa: F401


class RenderSamplingMode(Enum):  # ray_samplers/utils.py:7-9
    MASK_SAMPLE = "mask_sample"
    FULL_GRID = "full_grid"


def get_xy_grid(image_height, image_width, device=None):
    """(H, W, 2) integer-valued pixel grid, last dim (x=col, y=row) (ray_samplers/utils.py:12-24)."""
    ys = torch.arange(image_height, dtype=torch.float32, device=device)
    xs = torch.arange(image_width, dtype=torch.float32, device=device)
    gy, gx = torch.meshgrid(ys, xs, indexing="ij")
    return torch.stack((gx, gy), dim=-1)
