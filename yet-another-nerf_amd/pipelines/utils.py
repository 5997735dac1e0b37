"""Pipeline-level types and view metrics (reference yanerf/pipelines/utils.py).

RayBundle / EvaluationMode / PartialFunctionWrapper keep the reference's names and fields so callers are
unchanged. The metrics are caller-side (per-image MSE / huber on already rendered rays) and run as plain torch
ops on whatever device the renders live on; the hot path itself is in ..ops."""
from __future__ import annotations

from enum import Enum
from typing import Any, Dict, NamedTuple, Optional, Tuple

import math

import torch


class EvaluationMode(Enum):  # pipelines/utils.py:8-10
    TRAINING = "training"
    EVALUATION = "evaluation"


class RayBundle(NamedTuple):  # pipelines/utils.py:13-17
    origins: torch.Tensor
    directions: torch.Tensor
    lengths: torch.Tensor
    xys: torch.Tensor


class PartialFunctionWrapper(torch.nn.Module):
    """Binds extracted features as extra kwargs of a model call (pipelines/utils.py:20-33)."""

    def __init__(self, fn: torch.nn.Module):
        super().__init__()
        self._fn = fn
        self.bound_args: Dict[str, Any] = {}

    def bind_args(self, **bound_args):
        self.bound_args = bound_args

    def unbind_args(self):
        self.bound_args = {}

    def forward(self, *args, **kwargs):
        return self._fn(*args, **{**kwargs, **self.bound_args})


def sample_grid(tensor: torch.Tensor, image_sampling_grid: torch.Tensor) -> torch.Tensor:
    """Gather (B,H,W,C) at integer pixel coords (B,...,2) -> (B,...,C) (pipelines/utils.py:272-296)."""
    B, *sp, C = tensor.shape
    H, W = sp
    if bool((image_sampling_grid[..., 0].max() >= W).item()):
        raise AssertionError("Invalid ray_sampler.image_width")
    if bool((image_sampling_grid[..., 1].max() >= H).item()):
        raise AssertionError("Invalid ray_sampler.image_height")
    _, *gs, _ = image_sampling_grid.shape
    flat = tensor.reshape(B, -1, C)
    g = image_sampling_grid.reshape(B, -1, 2)
    idx = (g[:, :, 0] + W * g[:, :, 1]).long()[:, :, None].expand(-1, -1, C)
    return torch.gather(flat, -2, idx).view(B, *gs, C)


@torch.no_grad()
def scatter_rays_to_image(tensor, image_sampling_grid, image_height, image_width, bg_color=None):
    """Inverse of sample_grid for visualisation (pipelines/utils.py:299-323), as the yanerf_scatter_rays HIP kernels
    (fill + scatter; device tensors only, like every op of this package)."""
    from .. import ops
    return ops.scatter_rays(tensor, image_sampling_grid, image_height, image_width, bg_color)


def safe_sqrt(A: torch.Tensor, eps: float = 1e-4) -> torch.Tensor:
    return (torch.clamp(A, 0.0) + eps).sqrt()


def huber(dfsq: torch.Tensor, scaling: float = 0.03) -> torch.Tensor:  # pipelines/utils.py:150-158
    return (safe_sqrt(1 + dfsq / (scaling * scaling), eps=1e-4) - 1) * scaling


def calc_mse(x, y, mask=None):
    if mask is None:
        return torch.mean((x - y) ** 2, dim=-1)
    return (((x - y) ** 2) * mask).sum(dim=-1) / mask.expand_as(x).sum(dim=-1).clamp(1e-5)


def calc_psnr(x, y, mask=None, base: float = 1.0):
    mse = calc_mse(x, y, mask=mask)
    return torch.log10(mse.clamp(1e-10)) * (-10.0) + 20.0 * math.log10(base)


def mse2psnr(mse: float) -> float:
    """runners/utils.py:270-283: PSNR of the MEAN mse over a split."""
    return -10.0 * math.log10(max(float(mse), 1e-10))


def _rgb_metrics(images, images_pred, loss_reweight_masks=None):  # pipelines/utils.py:185-197
    B, *rest = images.shape
    images = images.reshape(B, -1)
    images_pred = images_pred.reshape(B, -1)
    diff = (images_pred - images) ** 2
    if loss_reweight_masks is not None:
        diff = diff * loss_reweight_masks.reshape(B, *rest).reshape(B, -1)
    sq = diff.mean(dim=-1)
    return {"rgb_huber": huber(sq, scaling=0.03), "rgb_mse": sq}


def estimate_depth_scale_factor(pred, gt, mask, clamp_thr):
    xy = pred * gt * mask
    xx = pred * pred * mask
    return xy.mean((1, 2, 3)) / torch.clamp(xx.mean((1, 2, 3)), clamp_thr)


def eval_depth(pred, gt, crop=1, mask=None, get_best_scale=True, mask_thr=0.5, best_scale_clamp_thr=1e-4):
    if crop > 0:
        gt = gt[:, :, crop:-crop, crop:-crop]
        pred = pred[:, :, crop:-crop, crop:-crop]
    if mask is not None:
        if crop > 0:
            mask = mask[:, :, crop:-crop, crop:-crop]
        gt = gt * (mask > mask_thr).float()
    dmask = (gt > 0.0).float()
    dmask_mass = torch.clamp(dmask.sum((1, 2, 3)), 1e-4)
    if get_best_scale:
        pred = pred * estimate_depth_scale_factor(pred, gt, dmask, best_scale_clamp_thr)[:, None, None, None]
    df = gt - pred
    return (dmask * (df ** 2)).sum((1, 2, 3)) / dmask_mass, (dmask * df.abs()).sum((1, 2, 3)) / dmask_mass


class ViewMetrics(torch.nn.Module):
    """Per-image rgb huber/mse (+ depth) against GT gathered at the rendered pixels (pipelines/utils.py:36-134)."""

    def forward(self, image_sampling_grid, images=None, images_pred=None, depths=None, depths_pred=None,
                loss_reweight_masks=None, keys_prefix: str = "loss_"):
        def _sg(t):
            return None if t is None else sample_grid(t, image_sampling_grid)

        images, depths, loss_reweight_masks = _sg(images), _sg(depths), _sg(loss_reweight_masks)
        preds = {}
        if images is not None and images_pred is not None:
            preds.update(_rgb_metrics(images, images_pred, loss_reweight_masks))
        if depths is not None and depths_pred is not None:
            _, abs_ = eval_depth(depths_pred, depths, get_best_scale=True, mask=None, crop=0)
            preds["depth_abs"] = abs_.mean(dim=-1)
        if keys_prefix is not None:
            preds = {keys_prefix + k: v for k, v in preds.items()}
        return preds
