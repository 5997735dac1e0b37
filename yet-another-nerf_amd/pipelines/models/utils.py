"""Parameter-holding building blocks of NeRFMLP (reference yanerf/pipelines/models/utils.py).

HarmonicEmbedding and LinearWithRepeat keep the reference's constructors, buffers, parameter names and
initialisation so NeRFMLP's state_dict and seeded initialisation match the reference exactly. NeRFMLP never
calls their forward: the fused `yanerf_mlp_forward` kernel evaluates the embedding and the LinearWithRepeat
term itself. Their forward methods are kept for API completeness as plain tensor algebra (models/utils.py:
90-103, 207-211) and are not part of the HIP hot path.
"""
from __future__ import annotations

import math
from typing import Tuple

import torch
import torch.nn.functional as F
from torch.nn import Parameter, init


class HarmonicEmbedding(torch.nn.Module):
    def __init__(self, n_harmonic_functions: int = 6, omega_0: float = 1.0, logspace: bool = True,
                 append_input: bool = True) -> None:
        super().__init__()
        if logspace:
            freqs = 2.0 ** torch.arange(n_harmonic_functions, dtype=torch.float32)
        else:
            freqs = torch.linspace(1.0, 2.0 ** (n_harmonic_functions - 1), n_harmonic_functions, dtype=torch.float32)
        self.register_buffer("_frequencies", freqs * omega_0, persistent=False)
        self.append_input = append_input
        self.logspace = logspace
        self.omega_0 = omega_0

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        e = (x[..., None] * self._frequencies).reshape(*x.shape[:-1], -1)
        return torch.cat((e.sin(), e.cos(), x) if self.append_input else (e.sin(), e.cos()), dim=-1)

    @staticmethod
    def get_output_dim_static(input_dims: int, n_harmonic_functions: int, append_input: bool) -> int:
        return input_dims * (2 * n_harmonic_functions + int(append_input))

    def get_output_dim(self, input_dims: int = 3) -> int:
        return self.get_output_dim_static(input_dims, len(self._frequencies), self.append_input)


class LinearWithRepeat(torch.nn.Module):
    """Linear over cat([x (..., k, n1), y (..., n2) broadcast over k]) without materialising the repeat."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, device=None, dtype=None) -> None:
        super().__init__()
        kw = {"device": device, "dtype": dtype}
        self.in_features = in_features
        self.out_features = out_features
        self.weight = Parameter(torch.empty((out_features, in_features), **kw))
        if bias:
            self.bias = Parameter(torch.empty(out_features, **kw))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        # same draws as torch.nn.Linear (models/utils.py:197-205)
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in, _ = init._calculate_fan_in_and_fan_out(self.weight)
            bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
            init.uniform_(self.bias, -bound, bound)

    def forward(self, input: Tuple[torch.Tensor, torch.Tensor]) -> torch.Tensor:
        n1 = input[0].shape[-1]
        return F.linear(input[0], self.weight[:, :n1], self.bias) + F.linear(input[1], self.weight[:, n1:],
                                                                               None).unsqueeze(-2)


def ray_bundle_to_ray_points(rays_origins, rays_directions, rays_lengths):
    """x = o + t d (models/utils.py:214-245)."""
    return rays_origins[..., None, :] + rays_lengths[..., :, None] * rays_directions[..., None, :]
