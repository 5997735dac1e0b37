"""RaySampler on the HIP path (reference yanerf/pipelines/ray_samplers/ray_sampler.py).

Same constructor/forward contract as the reference. Ray origins/directions/depths (incl. stratified jitter)
come from the `yanerf_raygen` kernel; uniform training pixel selection (no mask, no sampling prob) is done
in-kernel (keyed Philox permutation = sampling without replacement); masked / weighted selection keeps
torch.multinomial semantics (`_safe_multinomial`) on the device and hands the ids to the kernel."""
from __future__ import annotations

from typing import List, Optional, Tuple, Union

import torch

from ... import ops
from .builder import RAY_SAMPLERS
from .utils import EvaluationMode, RayBundle, RenderSamplingMode


@RAY_SAMPLERS.register_module()
class RaySampler(torch.nn.Module):
    def __init__(
        self,
        image_width: int = 400,
        image_height: int = 400,
        scene_center: Tuple[float, float, float] = (0.0, 0.0, 0.0),
        scene_extent: float = 0.0,
        sampling_mode_training: str = "mask_sample",
        sampling_mode_evaluation: str = "full_grid",
        n_pts_per_ray_training: int = 64,
        n_pts_per_ray_evaluation: int = 64,
        n_rays_per_image_sampled_from_mask: int = 1024,
        min_depth: float = 0.1,
        max_depth: float = 8.0,
        stratified_point_sampling_training: bool = True,
        stratified_point_sampling_evaluation: bool = False,
    ) -> None:
        super().__init__()
        self.image_width = image_width
        self.image_height = image_height
        self._sampling_mode = {
            EvaluationMode.TRAINING: RenderSamplingMode(sampling_mode_training),
            EvaluationMode.EVALUATION: RenderSamplingMode(sampling_mode_evaluation),
        }
        self._cfg = {
            EvaluationMode.TRAINING: dict(
                n_pts=n_pts_per_ray_training,
                n_rays=n_rays_per_image_sampled_from_mask
                if self._sampling_mode[EvaluationMode.TRAINING] == RenderSamplingMode.MASK_SAMPLE else None,
                stratified=stratified_point_sampling_training),
            EvaluationMode.EVALUATION: dict(
                n_pts=n_pts_per_ray_evaluation,
                n_rays=n_rays_per_image_sampled_from_mask
                if self._sampling_mode[EvaluationMode.EVALUATION] == RenderSamplingMode.MASK_SAMPLE else None,
                stratified=stratified_point_sampling_evaluation),
        }
        self._min_depth = min_depth
        self._max_depth = max_depth
        self.register_buffer("scene_center", torch.tensor(scene_center, dtype=torch.float32), persistent=False)
        self.scene_extent = scene_extent
        self._grid_ids = {}

    def _full_ids(self, H: int, W: int, B: int, device) -> torch.Tensor:
        key = (H, W, str(device))
        if key not in self._grid_ids:
            self._grid_ids[key] = torch.arange(H * W, dtype=torch.int64, device=device)
        return self._grid_ids[key][None].expand(B, -1)

    def forward(
        self,
        poses: torch.Tensor,
        focal_lengths: torch.Tensor,
        evaluation_mode: EvaluationMode,
        *,
        mask: Optional[torch.Tensor] = None,
        sampling_prob_mask: Optional[torch.Tensor] = None,
        image_height: Optional[int] = None,
        image_width: Optional[int] = None,
        min_depth: Optional[float] = None,
        max_depth: Optional[float] = None,
        n_rays_per_image: Union[None, int, List[int]] = None,
    ) -> RayBundle:
        cfg = self._cfg[evaluation_mode]
        B = poses.shape[0]
        device = poses.device
        sample_mask = None
        if self._sampling_mode[evaluation_mode] == RenderSamplingMode.MASK_SAMPLE and mask is not None:
            # ray_sampler.py:82-96 (resized to the configured image size)
            sample_mask = torch.nn.functional.interpolate(mask, size=[self.image_height, self.image_width],
                                                          mode="nearest")[:, 0]
        if min_depth is None and max_depth is None and self.scene_extent > 0.0:
            min_depth, max_depth = get_min_max_depth_bounds(poses, self.scene_center, self.scene_extent)
        if image_height is None or image_width is None:
            H, W = self.image_height, self.image_width
        else:
            H, W = image_height, image_width
        num_rays = n_rays_per_image or cfg["n_rays"]
        if sample_mask is not None and num_rays is None:
            num_rays = int(sample_mask.sum(dim=(1, 2)).min().int().item())
        # ray_sampler.py:280-283: tensor bounds collapse to their mean (LLFF per-image near/far)
        near = min_depth if min_depth is not None else self._min_depth
        far = max_depth if max_depth is not None else self._max_depth
        # (ops.depth_bounds: device tensors are averaged on the device and read by the kernel -- no host sync)
        jitter = None
        if cfg["stratified"]:
            inj = ops.INJECT.take("jitter_u")
            jitter = inj if inj is not None else "philox"
        common = dict(n_pts=cfg["n_pts"], near=near, far=far, cfg_w=self.image_width, cfg_h=self.image_height,
                      grid_hw=(H, W), jitter=jitter)
        if num_rays is None:
            o, d, z, xys, _ = ops.raygen(poses, focal_lengths, pixel_ids=self._full_ids(H, W, B, device), **common)
            spatial = (H, W)
        else:
            ids = ops.INJECT.take("pixel_ids")
            if ids is None and (sample_mask is not None or sampling_prob_mask is not None):
                ids = self._weighted_ids(B, H, W, num_rays, sample_mask, sampling_prob_mask, device)
            if ids is not None:
                o, d, z, xys, _ = ops.raygen(poses, focal_lengths, pixel_ids=ids, **common)
            else:
                if not isinstance(num_rays, int):
                    num_rays = int(sum(num_rays))
                o, d, z, xys, _ = ops.raygen(poses, focal_lengths, n_rays=num_rays, **common)
            spatial = (o.shape[1], 1)
        P = cfg["n_pts"]
        return RayBundle(origins=o.view(B, *spatial, 3), directions=d.view(B, *spatial, 3),
                         lengths=z.view(B, *spatial, P), xys=xys.view(B, *spatial, 2))

    @staticmethod
    def _sampling_weights(B, H, W, num_rays, mask, sampling_prob_mask, device):
        """The multinomial weights of masked / probability-weighted sampling (ray_sampler.py:181-216): [B, H*W], or
        [B, L, H*W] for a layered (B, L, H, W) sampling_prob_mask (num_rays then a list of L counts)."""
        weights = mask.reshape(B, -1) if mask is not None else torch.ones(B, H * W, device=device)
        if sampling_prob_mask is not None:
            if tuple(sampling_prob_mask.shape) == (B, H, W):
                weights = weights * sampling_prob_mask.reshape(B, -1)
            elif sampling_prob_mask.dim() == 4:
                if isinstance(num_rays, int):
                    num_rays = [num_rays]
                if tuple(sampling_prob_mask[:, 0].shape) != (B, H, W):
                    raise ValueError(f"Invalid `sampling_prob_mask`: `sampling_prob_mask.shape` "
                                     f"{sampling_prob_mask.shape}, must align with {(B, H, W, 2)}")
                if sampling_prob_mask.shape[1] != len(num_rays):
                    raise ValueError(f"Invalid number of sampling layers: sampling_prob_mask.shape[1] "
                                     f"{sampling_prob_mask.shape[1]} vs. len(num_rays) {len(num_rays)}")
                L = len(num_rays)
                weights = weights.unsqueeze(1).expand(-1, L, -1) * sampling_prob_mask.reshape(B, L, -1)
            else:
                raise ValueError(f"Invalida `sampling_prob_mask`, shape of {sampling_prob_mask.shape}, want (B, H, W) "
                                 f"or (B, L, H, W)")
        return weights, num_rays

    @staticmethod
    def _weighted_ids(B, H, W, num_rays, mask, sampling_prob_mask, device):
        """Pixel ids for masked / probability-weighted sampling (ray_sampler.py:181-227)."""
        weights, num_rays = RaySampler._sampling_weights(B, H, W, num_rays, mask, sampling_prob_mask, device)
        if weights.dim() == 2:
            return _safe_multinomial(weights, num_rays)
        return torch.cat([_safe_multinomial(weights[:, i], num_rays[i]) for i in range(len(num_rays))], dim=-1)


def _safe_multinomial(input: torch.Tensor, num_samples: int) -> torch.Tensor:
    """Sampling without replacement when there are enough non-zero weights, else with replacement
    (ray_sampler.py:317-358)."""
    try:
        res = torch.multinomial(input, num_samples, replacement=False)
    except RuntimeError:
        res = torch.multinomial(input, num_samples, replacement=True)
        no_repl = (input > 0.0).sum(dim=-1) >= num_samples
        res[no_repl] = torch.multinomial(input[no_repl], num_samples, replacement=False)
        return res
    repl = (input > 0.0).sum(dim=-1) < num_samples
    if repl.any():
        res[repl] = torch.multinomial(input[repl], num_samples, replacement=True)
    return res


def get_min_max_depth_bounds(poses, scene_center, scene_extent):
    """near/far from the camera-to-scene-centre distance (ray_sampler.py:389-401)."""
    cam_center = poses[:, :, -1]
    center_dist = ((cam_center - (poses[:, :3, :-1]) @ scene_center) ** 2).sum(dim=-1).clamp(0.001).sqrt()
    center_dist = center_dist.clamp(scene_extent + 1e-3)
    return (center_dist - scene_extent).mean().item(), (center_dist + scene_extent).mean().item()
