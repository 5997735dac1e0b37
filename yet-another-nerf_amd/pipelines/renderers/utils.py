"""RendererOutput, RayPointRefiner and sample_pdf on the HIP path (reference yanerf/pipelines/renderers/utils.py)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, Optional

import torch

from ... import ops
from ..utils import RayBundle


@dataclass
class RendererOutput:  # renderers/utils.py:11-33
    features: torch.Tensor
    depths: torch.Tensor
    alpha_masks: torch.Tensor
    prev_stage: Optional["RendererOutput"] = None
    normals: Optional[torch.Tensor] = None
    points: Optional[torch.Tensor] = None
    aux: Dict[str, Any] = field(default_factory=lambda: {})


class RayPointRefiner(torch.nn.Module):
    """Importance resampling of ray depths from the previous pass's weights (renderers/utils.py:36-69):
    `yanerf_refine` does midpoints, inverse-CDF sampling on weights[..., 1:-1], concat and sort in one kernel."""

    def __init__(self, n_pts_per_ray: int, random_sampling: bool, add_input_samples: bool = True) -> None:
        super().__init__()
        self.n_pts_per_ray = n_pts_per_ray
        self.random_sampling = random_sampling
        self.add_input_samples = add_input_samples

    def forward(self, origins, directions, lengths, xys, ray_weights):
        with torch.no_grad():
            u = ops.INJECT.take("pdf_u") if self.random_sampling else None
            zi = ops.INJECT.take("z_fine")
            if zi is not None:  # test mode: the reference's own refined depths replace this pass's refinement
                tot = self.n_pts_per_ray + (lengths.shape[-1] if self.add_input_samples else 0)
                z = zi.to(lengths.device, torch.float32).reshape(*lengths.shape[:-1], tot).contiguous()
            else:
                z = ops.refine(lengths, ray_weights, self.n_pts_per_ray, det=not self.random_sampling,
                               add_input=self.add_input_samples, u=u)
        return RayBundle(origins=origins, directions=directions, lengths=z, xys=xys)


def sample_pdf(bins: torch.Tensor, weights: torch.Tensor, n_samples: int, det: bool = False, eps: float = 1e-5,
               u: Optional[torch.Tensor] = None):
    """Inverse-CDF sampling (renderers/utils.py:72-158) as the `yanerf_sample_pdf` kernel."""
    if eps != 1e-5:
        raise NotImplementedError("the HIP sample_pdf uses the reference's eps = 1e-5")
    return ops.sample_pdf(bins, weights, n_samples, det=det, u=u)


def sample_pdf_python(bins, weights, N_samples, det=False, eps=1e-5):
    return sample_pdf(bins, weights, N_samples, det=det, eps=eps)
