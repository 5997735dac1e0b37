"""NeRFPipeline: the caller of the hot path (reference yanerf/pipelines/nerf_pipeline.py).

Same constructor and forward contract: builds the ray sampler / models / renderer from the registries, renders
(chunked over rays in full-grid evaluation, exactly as the reference's _chunk_generator splits them), computes
view metrics per stage and the weighted objective."""
from __future__ import annotations

import collections
import dataclasses
import logging
import math
from typing import Any, Callable, Dict, List, Optional, Sequence, Union

import torch

from .builder import PIPELINES
from .feature_extractors import FEATURE_EXTRACTORS
from .models import MODELS
from .ray_samplers import RAY_SAMPLERS
from .ray_samplers.utils import RenderSamplingMode
from .renderers import RENDERERS
from .renderers.utils import RendererOutput
from .utils import EvaluationMode, PartialFunctionWrapper, RayBundle, ViewMetrics, sample_grid

logger = logging.getLogger(__name__)


@PIPELINES.register_module()
class NeRFPipeline(torch.nn.Module):
    def __init__(self, ray_sampler, model, feature_extractor, renderer, chunk_size_grid: int, num_passes: int,
                 loss_weights: Dict[str, float] = {"loss_rgb_mse": 1.0, "loss_prev_stage_rgb_mse": 1.0},
                 output_rasterized_mc: bool = False) -> None:
        super().__init__()
        self.ray_sampler = RAY_SAMPLERS.build(ray_sampler)
        self.render_image_height = ray_sampler["image_height"]
        self.render_image_width = ray_sampler["image_width"]
        self.sampling_mode_training = RenderSamplingMode.MASK_SAMPLE
        self.sampling_mode_evaluation = RenderSamplingMode.FULL_GRID
        if isinstance(model, Sequence) and not isinstance(model, dict) and len(model) != num_passes:
            logger.info(f"Rewrite `num_pass` from {num_passes} to {len(model)}.")
            num_passes = len(model)
        self.num_passes = num_passes
        if not isinstance(model, Sequence) or isinstance(model, dict):
            model = [model] * num_passes  # independent instances: coarse and fine MLPs (nerf_pipeline.py:84-88)
        self.implicit_functions = torch.nn.ModuleList([PartialFunctionWrapper(MODELS.build(m)) for m in model])
        fe = feature_extractor
        if not isinstance(fe, Sequence) or isinstance(fe, dict):
            fe = [fe]
        self.feature_extractors = torch.nn.ModuleList([FEATURE_EXTRACTORS.build(f) for f in fe])
        self.renderer = RENDERERS.build(renderer)
        bg = renderer["bg_color"] if "bg_color" in renderer else (0.0,)
        if not isinstance(bg, torch.Tensor):
            bg = torch.tensor(bg)
        self.register_buffer("bg_color", bg, persistent=False)
        self.chunk_size_grid = chunk_size_grid
        self.output_rasterized_mc = output_rasterized_mc
        self.loss_weights = dict(loss_weights)
        self.view_metrics = ViewMetrics()

    def forward(self, *, poses: torch.Tensor, focal_lengths: torch.Tensor, image_height: Optional[int] = None,
                image_width: Optional[int] = None, min_depth: Optional[float] = None,
                max_depth: Optional[float] = None, mask_crop: Optional[torch.Tensor] = None,
                sampling_prob_mask: Optional[torch.Tensor] = None,
                n_rays_per_image: Union[None, int, List[int]] = None, bg_image_rgb: Optional[torch.Tensor] = None,
                image_rgb: Optional[torch.Tensor] = None, depth_map: Optional[torch.Tensor] = None,
                evaluation_mode: EvaluationMode = EvaluationMode.EVALUATION, **kwargs):
        training = evaluation_mode == EvaluationMode.TRAINING
        sampling_mode = self.sampling_mode_training if training else self.sampling_mode_evaluation
        ray_bundle: RayBundle = self.ray_sampler(
            poses, focal_lengths, evaluation_mode=evaluation_mode,
            mask=mask_crop if mask_crop is not None and sampling_mode == RenderSamplingMode.MASK_SAMPLE else None,
            sampling_prob_mask=sampling_prob_mask if training else None,
            n_rays_per_image=n_rays_per_image if training else None, image_height=image_height,
            image_width=image_width, min_depth=min_depth, max_depth=max_depth)
        xys = ray_bundle.xys
        bg_color = sample_grid(bg_image_rgb, xys) if bg_image_rgb is not None else None

        extracted = collections.defaultdict(list)
        for fe in self.feature_extractors:
            for k, v in fe(**kwargs).items():
                extracted[k].append(v)
        for k, vs in list(extracted.items()):
            if isinstance(vs[0], torch.Tensor):
                extracted[k] = torch.stack(vs, dim=1)
            else:
                if len(vs) != 1:
                    raise KeyError(f"{k} has multiple {type(vs[0])} values.")
                extracted[k] = vs[0]
        for f in self.implicit_functions:
            f.bind_args(**extracted)
        rendered: RendererOutput = self._render(*ray_bundle, bg_color=bg_color, sampling_mode=sampling_mode,
                                                implicit_functions=self.implicit_functions,
                                                evaluation_mode=evaluation_mode)
        for f in self.implicit_functions:
            f.unbind_args()

        preds = self._get_view_metrics(rendered, xys, image_rgb, depth_map)
        blob = {}
        if sampling_mode == RenderSamplingMode.MASK_SAMPLE:
            if self.output_rasterized_mc:
                blob = {"rendered_images": rendered.features, "rendered_depths": rendered.depths,
                        "rendered_alpha_masks": rendered.alpha_masks}
                blob = self._rasterize_mc_samples(xys, None, image_height, image_width, blob)
        elif sampling_mode == RenderSamplingMode.FULL_GRID:
            blob = {"rendered_images": rendered.features, "rendered_depths": rendered.depths,
                    "rendered_alpha_masks": rendered.alpha_masks}
        else:
            raise ValueError(f"Invalid RenderSamplingMode: {sampling_mode}.")
        preds.update(blob)
        objective = self._get_objective(preds)
        if objective is not None:
            preds["objective"] = objective
        return preds

    def _render(self, origins, directions, lengths, xys, *, bg_color, sampling_mode, **kwargs):
        if sampling_mode == RenderSamplingMode.FULL_GRID and self.chunk_size_grid > 0:
            chunks = [self.renderer(*a, **kw) for a, kw in
                      _chunk_generator(self.chunk_size_grid, origins, directions, lengths, xys, bg_color, **kwargs)]
            return cat_dataclass(chunks, lambda batch: _tensor_collator(batch, lengths.shape[:-1]))
        return self.renderer(origins=origins, directions=directions, lengths=lengths, xys=xys, bg_color=bg_color,
                             **kwargs)

    def _get_view_metrics(self, raymarched: RendererOutput, xys, image_rgb=None, depth_map=None,
                          keys_prefix: str = "loss_"):
        metrics = self.view_metrics(image_sampling_grid=xys, images_pred=raymarched.features, images=image_rgb,
                                    depths_pred=raymarched.depths, depths=depth_map, keys_prefix=keys_prefix)
        prev, prefix = raymarched.prev_stage, keys_prefix
        while prev is not None:
            prefix = prefix + "prev_stage_"
            metrics.update(self.view_metrics(image_sampling_grid=xys, images_pred=prev.features, images=image_rgb,
                                             depths_pred=prev.depths, depths=depth_map, keys_prefix=prefix))
            prev = prev.prev_stage
        return metrics

    def _get_objective(self, preds) -> Optional[torch.Tensor]:
        for k in self.loss_weights:
            if k not in preds:
                logger.warning(f"loss name is not found: {k}")
        terms = [preds[k] * float(w) for k, w in self.loss_weights.items() if k in preds and w != 0.0]
        if not terms:
            logger.warning("No main objective found.")
            return None
        return sum(terms)

    def _rasterize_mc_samples(self, xys, bg_color, image_height, image_width, rendered):
        if image_height is None or image_width is None:
            image_height, image_width = self.render_image_height, self.render_image_width
        # scatter_rays_to_image per tensor (nerf_pipeline.py:307-324), with ONE read-back of the kernels' out-of-image
        # flag for all of them (the same xys) instead of one host sync per tensor
        from .. import ops
        out = {k: ops.scatter_rays(v, xys, image_height, image_width, bg_color, check=False) for k, v in rendered.items()}
        if out:
            ops.check_scatter_bounds(xys.device)
        return out


def _chunk_generator(chunk_size: int, origins, directions, lengths, xys, bg_color=None, *args, **kwargs):
    """Split the ray grid into ceil(R * P / chunk_size) contiguous ray chunks (nerf_pipeline.py:333-377)."""
    B, *spatial, P = lengths.shape
    n_rays = math.prod(spatial)
    n_chunks = -(-n_rays * max(P, 1) // chunk_size)
    per = -(-n_rays // n_chunks)
    for s in range(0, n_rays, per):
        e = min(s + per, n_rays)
        bg = None if bg_color is None else bg_color.reshape(B, -1, 1, bg_color.shape[-1])[:, s:e]
        yield [origins.reshape(B, -1, 1, origins.shape[-1])[:, s:e],
               directions.reshape(B, -1, 1, directions.shape[-1])[:, s:e],
               lengths.reshape(B, -1, 1, P)[:, s:e], xys.reshape(B, -1, 1, xys.shape[-1])[:, s:e], bg, *args], kwargs


def _tensor_collator(batch, new_dims):
    return torch.cat(batch, dim=1).reshape(*new_dims, *batch[0].shape[3:])


def cat_dataclass(batch, tensor_collator: Callable):
    """Concatenate every tensor field (and nested prev_stage / aux dicts) of a list of dataclasses
    (nerf_pipeline.py:394-426)."""
    elem = batch[0]
    out: Dict[str, Any] = {}
    for f in dataclasses.fields(elem):
        v = getattr(elem, f.name)
        if v is None:
            out[f.name] = None
        elif torch.is_tensor(v):
            out[f.name] = tensor_collator([getattr(e, f.name) for e in batch])
        elif dataclasses.is_dataclass(v):
            out[f.name] = cat_dataclass([getattr(e, f.name) for e in batch], tensor_collator)
        elif isinstance(v, collections.abc.Mapping):
            out[f.name] = {k: tensor_collator([getattr(e, f.name)[k] for e in batch]) if v[k] is not None else None
                           for k in v}
        else:
            raise ValueError("Unsupported field type for concatenation")
    return type(elem)(**out)
