"""Multi-pass emission-absorption renderer on the HIP path
(reference yanerf/pipelines/renderers/multipass_emission_absorpsion_renderer.py).

Same constructor/forward/recursion as the reference; the raymarcher is the fused `yanerf_composite_forward`
/ `yanerf_composite_backward` kernel pair (one wave64 per ray; double-precision transmittance scan)."""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Tuple, Union

import torch

from ... import ops
from ..utils import EvaluationMode, RayBundle
from .builder import RENDERERS
from .utils import RayPointRefiner, RendererOutput


@RENDERERS.register_module()
class MultipassEmissionAbsorpsionRenderer(torch.nn.Module):
    def __init__(
        self,
        n_pts_per_ray_fine_training: int = 64,
        n_pts_per_ray_fine_evaluation: int = 64,
        stratified_sampling_coarse_training: bool = True,
        stratified_sampling_coarse_evaluation: bool = False,
        append_coarse_samples_to_fine: bool = True,
        bg_color: Tuple[float, ...] = (0.0,),
        density_noise_std_train: float = 0.0,
        capping_function: str = "exponential",
        weight_function: str = "product",
        background_opacity: float = 1e10,
        blend_output: bool = False,
        background_density_bias: float = 0.0,
        hard_background: bool = False,
    ) -> None:
        super().__init__()
        self.density_noise_std_train = density_noise_std_train
        self._refiners = {
            EvaluationMode.TRAINING: RayPointRefiner(n_pts_per_ray_fine_training, stratified_sampling_coarse_training,
                                                     append_coarse_samples_to_fine),
            EvaluationMode.EVALUATION: RayPointRefiner(n_pts_per_ray_fine_evaluation,
                                                       stratified_sampling_coarse_evaluation,
                                                       append_coarse_samples_to_fine),
        }
        self._raymarcher = EmissionAbsorptionRaymarcher(
            surface_thickness=1, bg_color=bg_color, capping_function=capping_function,
            weight_function=weight_function, background_opacity=background_opacity, blend_output=blend_output,
            hard_background=hard_background, background_density_bias=background_density_bias)

    def forward(self, origins, directions, lengths, xys, bg_color: Optional[torch.Tensor], *,
                implicit_functions: List[Callable], evaluation_mode: EvaluationMode = EvaluationMode.EVALUATION,
                **kwargs):
        if not implicit_functions:
            raise ValueError("EA renderer expects implicit functions")
        return self._run_raymarcher(origins, directions, lengths, xys, bg_color, implicit_functions, None,
                                    evaluation_mode, **kwargs)

    def _run_raymarcher(self, origins, directions, lengths, xys, bg_color, implicit_functions, prev_stage,
                        evaluation_mode, **kwargs):
        noise_std = self.density_noise_std_train if evaluation_mode == EvaluationMode.TRAINING else 0.0
        features, depths, alpha_masks, weights, aux = self._raymarcher(
            **implicit_functions[0](origins, directions, lengths, **kwargs), ray_lengths=lengths,
            ray_directions=directions, density_noise_std=noise_std, bg_color=bg_color)
        aux["weights"] = weights
        output = RendererOutput(features=features, depths=depths, alpha_masks=alpha_masks, aux=aux,
                                prev_stage=prev_stage)
        if len(implicit_functions) > 1:
            rb: RayBundle = self._refiners[evaluation_mode](origins, directions, lengths, xys, weights)
            output = self._run_raymarcher(*rb, bg_color, implicit_functions[1:], output, evaluation_mode, **kwargs)
        return output


class EmissionAbsorptionRaymarcher(torch.nn.Module):
    """EA compositing (renderer.py:120-239) as the fused composite kernels."""

    def __init__(self, surface_thickness: int = 1, bg_color: Union[Tuple[float, ...], torch.Tensor] = (0.0,),
                 capping_function: str = "exponential", weight_function: str = "product",
                 background_opacity: float = 1e10, density_relu: bool = True, blend_output: bool = True,
                 background_density_bias: float = 0.0, hard_background: bool = False) -> None:
        super().__init__()
        if surface_thickness != 1:
            raise NotImplementedError("surface_thickness != 1 is not on the HIP path (the reference always uses 1)")
        if capping_function not in ("exponential", "cap1"):
            raise KeyError(capping_function)
        if weight_function not in ("product", "minimum"):
            raise KeyError(weight_function)
        if not isinstance(bg_color, torch.Tensor):
            bg_color = torch.tensor(bg_color, dtype=torch.float32)
        self.register_buffer("_bg_color", bg_color, persistent=False)
        self.surface_thickness = surface_thickness
        self.cfg = ops.RaymarchCfg(capping_function=capping_function, weight_function=weight_function,
                                   background_opacity=background_opacity, density_relu=density_relu,
                                   blend_output=blend_output, background_density_bias=background_density_bias,
                                   hard_background=hard_background,
                                   bg_color=tuple(float(x) for x in bg_color.reshape(-1).tolist()))

    def forward(self, rays_densities: torch.Tensor, rays_features: torch.Tensor, aux: Dict[str, Any],
                ray_lengths: torch.Tensor, ray_directions: torch.Tensor, density_noise_std: float = 0.0,
                bg_color: Optional[torch.Tensor] = None):
        _check_raymarcher_inputs(rays_densities, rays_features, ray_lengths, z_can_be_none=True,
                                 features_can_be_none=False, density_1d=True)
        C = rays_features.shape[-1]
        if bg_color is not None:
            if bg_color.shape[-1] not in (1, C):
                raise ValueError(f"Wrong number of background color channels: _bg_color {bg_color.shape} vs. "
                                 f"features {rays_features.shape}.")
            bg_color = bg_color.expand(*rays_features.shape[:-2], C)
        elif len(self.cfg.bg_color) not in (1, C):
            raise ValueError(f"Wrong number of background color channels: _bg_color {self._bg_color.shape} vs. "
                             f"features {rays_features.shape}.")
        noise = ops.INJECT.take("noise") if density_noise_std > 0.0 else None
        feats, depths, alpha, weights = ops.composite(self.cfg, rays_densities, rays_features, ray_lengths,
                                                      ray_directions, bg=bg_color, noise_std=density_noise_std,
                                                      noise=noise)
        return feats, depths, alpha, weights, aux


def _check_raymarcher_inputs(rays_densities, rays_features, rays_z, features_can_be_none=False, z_can_be_none=False,
                             density_1d=True) -> None:
    """Shape validation with the reference's ValueErrors (renderer.py:242-278)."""
    if not torch.is_tensor(rays_densities):
        raise ValueError("rays_densities has to be an instance of torch.Tensor.")
    if not z_can_be_none and not torch.is_tensor(rays_z):
        raise ValueError("rays_z has to be an instance of torch.Tensor.")
    if not features_can_be_none and not torch.is_tensor(rays_features):
        raise ValueError("rays_features has to be an instance of torch.Tensor.")
    if rays_densities.ndim < 1:
        raise ValueError("rays_densities have to have at least one dimension.")
    if density_1d and rays_densities.shape[-1] != 1:
        raise ValueError("The size of the last dimension of rays_densities has to be one.")
    rays_shape = rays_densities.shape[:-1]
    if not z_can_be_none and rays_z.shape != rays_shape:
        raise ValueError("rays_z have to be of the same shape as rays_densities.")
    if not features_can_be_none and rays_features.shape[:-1] != rays_shape:
        raise ValueError("The first to previous to last dimensions of rays_features have to be the same as all "
                         "dimensions of rays_densities.")
