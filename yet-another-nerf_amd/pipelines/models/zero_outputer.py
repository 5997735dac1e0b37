"""ZeroOutputer: debug model returning zero density/colour (reference models/zero_outputer.py:13-36).
Used as the fake network of the reference's known-answer pipeline test."""
import warnings
from typing import Optional

import torch

from .builder import MODELS


@MODELS.register_module()
class ZeroOutputer(torch.nn.Module):
    def __init__(self) -> None:
        super().__init__()
        warnings.warn("Should not use ZeroOutputer, Debug only.")

    def forward(self, origins, directions, lengths, global_codes: Optional[torch.Tensor] = None, **kwargs):
        B, *spatial, _ = origins.shape
        P = lengths.shape[-1]
        return dict(rays_densities=origins.new_zeros(B, *spatial, P, 1),
                    rays_features=origins.new_zeros(B, *spatial, P, 3), aux={})
