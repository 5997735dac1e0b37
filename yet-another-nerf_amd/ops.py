"""Torch-facing wrappers of the HIP hot path (autograd Functions over the C ABI in include/yanerf_hip.h).

Tensors stay in PyTorch's caching allocator; kernels run on torch's current HIP stream. Every op requires
ROCm device tensors and raises otherwise: there is no CPU/torch fallback for the hot path.
"""
from __future__ import annotations

import ctypes
from contextlib import contextmanager
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch

from . import _C

_F32 = torch.float32


# ----------------------------------------------------------------------------------------- helpers
def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _dev(*ts: Optional[torch.Tensor]) -> None:
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                "yanerf_amd runs the NeRF hot path only as HIP kernels on a ROCm device; got a CPU tensor. "
                "(The reference's --device cpu path is not part of this package.)"
            )


def _f32c(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if t is None:
        return None
    if t.dtype != _F32:
        t = t.float()
    return t.contiguous()


class _Rng:
    """Philox (seed, offset) stream. The module-level RNG (used by the registry ops) follows torch.manual_seed; a
    stream built with an explicit seed (the fused trainer's, seed + rank as scripts/run.py:70-71 seeds each rank)
    is independent of torch's global generator."""

    def __init__(self, seed: Optional[int] = None):
        self._fixed = seed is not None
        self._seed = None if seed is None else int(seed) & 0xFFFFFFFFFFFFFFFF
        self._offset = 0

    def next(self, n: int = 1) -> Tuple[int, int]:
        if not self._fixed:
            seed = torch.initial_seed() & 0xFFFFFFFFFFFFFFFF
            if seed != self._seed:
                self._seed, self._offset = seed, 0
        off = self._offset
        self._offset += max(int(n), 1)
        return self._seed, off

    def get_state(self) -> Tuple[int, int]:
        return self._seed, self._offset

    def set_state(self, state: Tuple[int, int]) -> None:
        self._seed, self._offset = state


RNG = _Rng()


def philox_stream(seed: int) -> _Rng:
    return _Rng(seed)


class _Injection:
    """Test mode: queues of random draws captured from the reference (tests/golden) that replace the Philox
    stream, consumed in call order by the kernels that need randomness."""

    def __init__(self):
        self.queues = None

    def take(self, name: str):
        if self.queues and self.queues.get(name):
            return self.queues[name].pop(0)
        return None


INJECT = _Injection()


@contextmanager
def injected_randomness(**queues):
    """with injected_randomness(pixel_ids=t, jitter_u=t, noise=[nc, nf], pdf_u=t[, z_fine=t]): ...
    Consumed by the registry ops and by NeRFTrainer.step alike (pixel ids, stratified jitter, the coarse then the
    fine density noise, the refinement uniforms), in the order the reference draws them. `z_fine` (optional) is the
    reference's refined depths (RayPointRefiner.forward's output, renderers/utils.py:48-69): given, the fine pass runs
    at exactly those depths instead of this build's refinement, so the fine stage and its gradients can be held to
    strict gates independent of sample_pdf's ill-conditioned branch (tests/parity_gates.py)."""
    INJECT.queues = {k: list(v) if isinstance(v, (list, tuple)) else [v] for k, v in queues.items()}
    try:
        yield
    finally:
        INJECT.queues = None


# ----------------------------------------------------------------------------------------- ray generation
def depth_bounds(near, far, dev):
    """(near, far, bounds): floats pass through; tensor bounds collapse to their means (ray_sampler.py:280-283:
    `.mean().item()`). Host tensors are averaged on the host; device tensors are averaged ON the device into
    `bounds` [2] (the kernel reads them there), so a step fed device-resident LLFF bounds never syncs the host."""
    def dev_mean(x):
        return isinstance(x, torch.Tensor) and x.device.type != "cpu"

    if dev_mean(near) or dev_mean(far):
        vals = [x.float().mean().reshape(1) if isinstance(x, torch.Tensor) else torch.tensor([float(x)])
                for x in (near, far)]
        return 0.0, 0.0, torch.cat([v.to(dev, non_blocking=True) for v in vals]).contiguous()
    near = near.float().mean().item() if isinstance(near, torch.Tensor) else float(near)
    far = far.float().mean().item() if isinstance(far, torch.Tensor) else float(far)
    return near, far, None


def raygen(poses: torch.Tensor, focal: torch.Tensor, *, n_pts: int, near, far, cfg_w: int, cfg_h: int,
           xy: Optional[torch.Tensor] = None, pixel_ids: Optional[torch.Tensor] = None, n_rays: Optional[int] = None,
           grid_hw: Optional[Tuple[int, int]] = None, jitter: Optional[object] = None):
    """_xy_to_ray_bundle (ray_sampler.py:249-314) on the GPU. Pixel source: `xy` [B,R,2] float, `pixel_ids`
    [B,R] int64 into grid_hw, or neither (uniform sampling without replacement of n_rays pixels).
    jitter: None, "philox", or a [B,R,P] tensor of injected uniforms. near / far: floats or tensors (depth_bounds).
    Returns origins [B,R,3], directions [B,R,3], lengths [B,R,P], xys [B,R,2], ids [B,R] (or None)."""
    _dev(poses, focal, xy, pixel_ids)
    B = poses.shape[0]
    poses = _f32c(poses[:, :3, :4])
    focal = _f32c(focal.reshape(B))
    if xy is not None:
        xy = _f32c(xy.reshape(B, -1, 2))
        R = xy.shape[1]
    elif pixel_ids is not None:
        pixel_ids = pixel_ids.reshape(B, -1).to(torch.int64).contiguous()
        R = pixel_ids.shape[1]
    else:
        R = int(n_rays)
    gh, gw = grid_hw if grid_hw is not None else (cfg_h, cfg_w)
    dev = poses.device
    o = torch.empty(B, R, 3, device=dev, dtype=_F32)
    d = torch.empty(B, R, 3, device=dev, dtype=_F32)
    z = torch.empty(B, R, n_pts, device=dev, dtype=_F32)
    xys = torch.empty(B, R, 2, device=dev, dtype=_F32)
    ids = torch.empty(B, R, device=dev, dtype=torch.int64) if xy is None else None
    if jitter is None:
        mode, ju = 0, None
    elif isinstance(jitter, torch.Tensor):
        _dev(jitter)
        mode, ju = 1, _f32c(jitter.reshape(B, R, n_pts))
    else:
        mode, ju = 2, None
    near, far, bounds = depth_bounds(near, far, dev)
    seed, off = RNG.next(B * R * n_pts)
    _C.check(_C.lib().yanerf_raygen(_p(poses), _p(focal), _p(xy), _p(pixel_ids), B, R, gw, gh, float(cfg_w),
                                    float(cfg_h), float(near), float(far), n_pts, mode, _p(ju), seed, off, _p(o), _p(d),
                                    _p(z), _p(xys), _p(ids), _p(bounds), None, _stream()), "yanerf_raygen")
    return o, d, z, xys, ids


# ----------------------------------------------------------------------------------------- NeRF MLP
@dataclass
class MlpSpec:
    n_layers: int = 8
    input_skips: Sequence[int] = (5,)
    n_harmonic_functions_xyz: int = 10
    n_harmonic_functions_dir: int = 4
    append_xyz: bool = True
    append_dir: bool = True
    n_hidden_neurons_xyz: int = 256
    n_hidden_neurons_dir: int = 128
    color_dim: int = 3
    precision: int = _C.PREC_F32

    def desc(self) -> _C.MlpDesc:
        mask = 0
        for s in self.input_skips:
            if 0 < s < self.n_layers:
                mask |= 1 << int(s)
        return _C.MlpDesc(self.n_layers, mask, self.n_harmonic_functions_xyz, self.n_harmonic_functions_dir,
                          int(self.append_xyz), int(self.append_dir), self.n_hidden_neurons_xyz,
                          self.n_hidden_neurons_dir, self.color_dim)

    def validate(self) -> None:
        d = self.desc()
        n = _C.lib().yanerf_mlp_num_params(ctypes.byref(d))
        if n < 0:
            raise ValueError(f"NeRFMLP configuration not supported by the HIP path: "
                             f"{_C.lib().yanerf_last_error().decode()}")


def mlp_pack(spec: MlpSpec, params: Sequence[torch.Tensor], out: Optional[torch.Tensor] = None) -> torch.Tensor:
    d = spec.desc()
    nbytes = _C.lib().yanerf_mlp_packed_bytes(ctypes.byref(d), spec.precision)
    if nbytes < 0:
        _C.check(1, "yanerf_mlp_packed_bytes")
    ps = [_f32c(p.detach()) for p in params]
    _dev(*ps)
    if out is None or out.numel() < nbytes:
        out = torch.empty(nbytes, dtype=torch.uint8, device=ps[0].device)
    arr = _C.ptr_array([p.data_ptr() for p in ps])
    _C.check(_C.lib().yanerf_mlp_pack(ctypes.byref(d), spec.precision, arr, _p(out), _stream()), "yanerf_mlp_pack")
    return out


class _MLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec: MlpSpec, packed: torch.Tensor, origins, directions, lengths, *params):
        lead = lengths.shape[:-1]
        P = lengths.shape[-1]
        R = lengths[..., 0].numel()
        o = _f32c(origins.reshape(R, 3))
        dvec = _f32c(directions.reshape(R, 3))
        t = _f32c(lengths.reshape(R, P))
        dev = t.device
        d = spec.desc()
        need_bwd = any(ctx.needs_input_grad[5:])
        saved = None
        if need_bwd:
            nb = _C.lib().yanerf_mlp_saved_bytes(ctypes.byref(d), spec.precision, R * P)
            saved = torch.empty(nb, dtype=torch.uint8, device=dev)
        sigma = torch.empty(R * P, dtype=_F32, device=dev)
        rgb = torch.empty(R * P, spec.color_dim, dtype=_F32, device=dev)
        _C.check(_C.lib().yanerf_mlp_forward(ctypes.byref(d), spec.precision, _p(packed), _p(o), _p(dvec), _p(t), R,
                                             P, _p(sigma), _p(rgb), _p(saved), _stream()), "yanerf_mlp_forward")
        if need_bwd:
            ctx.spec = spec
            ctx.saved_ws = saved
            ctx.R, ctx.P = R, P
            ctx.save_for_backward(packed, rgb, *params)
        return sigma.view(*lead, P, 1), rgb.view(*lead, P, spec.color_dim)

    @staticmethod
    def backward(ctx, g_sigma, g_rgb):
        spec: MlpSpec = ctx.spec
        packed, rgb, *params = ctx.saved_tensors
        R, P = ctx.R, ctx.P
        dev = rgb.device
        gs = torch.zeros(R * P, dtype=_F32, device=dev) if g_sigma is None else _f32c(g_sigma.reshape(R * P))
        gr = torch.zeros(R * P, spec.color_dim, dtype=_F32, device=dev) if g_rgb is None else _f32c(
            g_rgb.reshape(R * P, spec.color_dim))
        grads = [torch.empty(p.shape, dtype=_F32, device=dev) for p in params]
        d = spec.desc()
        wsb = _C.lib().yanerf_mlp_bwd_workspace_bytes(ctypes.byref(d), spec.precision, R * P)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        arr = _C.ptr_array([g.data_ptr() for g in grads])
        _C.check(_C.lib().yanerf_mlp_backward(ctypes.byref(d), spec.precision, _p(packed), _p(ctx.saved_ws), _p(rgb),
                                              _p(gs), _p(gr), R, P, arr, _p(ws), _stream()), "yanerf_mlp_backward")
        ctx.saved_ws = None
        grads = [g.to(p.dtype) for g, p in zip(grads, params)]
        return (None, None, None, None, None, *grads)


def mlp_forward(spec: MlpSpec, packed: torch.Tensor, origins, directions, lengths, params: Sequence[torch.Tensor]):
    _dev(origins, directions, lengths, packed)
    return _MLPFn.apply(spec, packed, origins, directions, lengths, *params)


# ----------------------------------------------------------------------------------------- compositing
@dataclass
class RaymarchCfg:
    capping_function: str = "exponential"
    weight_function: str = "product"
    background_opacity: float = 1e10
    density_relu: bool = True
    blend_output: bool = True
    background_density_bias: float = 0.0
    hard_background: bool = False
    bg_color: Tuple[float, ...] = (0.0,)

    def opts(self, noise_mode: int = 0, noise_std: float = 0.0, seed: int = 0, offset: int = 0,
             rng_base: Optional[int] = None) -> _C.RaymarchOpts:
        """rng_base: device address of a u64 added to `offset` by the kernel (the trainer's device step state)."""
        caps = {"exponential": 0, "cap1": 1}
        wfn = {"product": 0, "minimum": 1}
        if self.capping_function not in caps:
            raise ValueError(f"unknown capping_function {self.capping_function}")
        if self.weight_function not in wfn:
            raise ValueError(f"unknown weight_function {self.weight_function}")
        bg = list(self.bg_color)[:4]
        if len(bg) > 4:
            raise ValueError("bg_color with more than 4 channels is not supported")
        arr = (ctypes.c_float * 4)(*(bg + [0.0] * (4 - len(bg))))
        return _C.RaymarchOpts(caps[self.capping_function], wfn[self.weight_function], int(self.blend_output),
                               int(self.hard_background), int(self.density_relu), float(self.background_opacity),
                               float(self.background_density_bias), arr, len(bg), noise_mode, float(noise_std),
                               seed, offset, rng_base)


class _CompositeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, opts_bytes: bytes, sigma_raw, rgb, lengths, directions, bg, noise):
        o = _C.RaymarchOpts.from_buffer_copy(opts_bytes)
        lead = lengths.shape[:-1]
        P = lengths.shape[-1]
        R = lengths[..., 0].numel()
        C = rgb.shape[-1]
        s = _f32c(sigma_raw.reshape(R, P))
        c = _f32c(rgb.reshape(R, P, C))
        t = _f32c(lengths.reshape(R, P))
        dv = _f32c(directions.reshape(R, 3))
        bgt = None if bg is None else _f32c(bg.expand(*lead, C).reshape(R, C))
        nz = None if noise is None else _f32c(noise.reshape(R, P))
        dev = t.device
        feats = torch.empty(R, C, dtype=_F32, device=dev)
        depth = torch.empty(R, dtype=_F32, device=dev)
        alpha = torch.empty(R, dtype=_F32, device=dev)
        w = torch.empty(R, P, dtype=_F32, device=dev)
        _C.check(_C.lib().yanerf_composite_forward(ctypes.byref(o), _p(s), _p(c), _p(t), _p(dv), _p(bgt), _p(nz), R,
                                                   P, C, _p(feats), _p(depth), _p(alpha), _p(w), _stream()),
                 "yanerf_composite_forward")
        ctx.opts_bytes = opts_bytes
        ctx.dims = (R, P, C, lead)
        ctx.has_bg = bgt is not None
        ctx.save_for_backward(s, c, t, dv, bgt if bgt is not None else s, nz if nz is not None else s)
        ctx.has_nz = nz is not None
        ctx.mark_non_differentiable(w)
        return (feats.view(*lead, C), depth.view(*lead, 1), alpha.view(*lead, 1), w.view(*lead, P))

    @staticmethod
    def backward(ctx, g_feats, g_depth, g_alpha, g_w):
        R, P, C, lead = ctx.dims
        s, c, t, dv, bgt, nz = ctx.saved_tensors
        bgt = bgt if ctx.has_bg else None
        nz = nz if ctx.has_nz else None
        o = _C.RaymarchOpts.from_buffer_copy(ctx.opts_bytes)
        dev = s.device
        gf = torch.zeros(R, C, dtype=_F32, device=dev) if g_feats is None else _f32c(g_feats.reshape(R, C))
        gd = None if g_depth is None else _f32c(g_depth.reshape(R))
        ga = None if g_alpha is None else _f32c(g_alpha.reshape(R))
        g_sigma = torch.empty(R, P, dtype=_F32, device=dev)
        g_rgb = torch.empty(R, P, C, dtype=_F32, device=dev)
        _C.check(_C.lib().yanerf_composite_backward(ctypes.byref(o), _p(s), _p(c), _p(t), _p(dv), _p(bgt), _p(nz),
                                                    _p(gf), _p(gd), _p(ga), R, P, C, _p(g_sigma), _p(g_rgb), _stream()),
                 "yanerf_composite_backward")
        return (None, g_sigma.view(*lead, P, 1), g_rgb.view(*lead, P, C), None, None, None, None)


def composite(cfg: RaymarchCfg, sigma_raw, rgb, lengths, directions, *, bg=None, noise_std: float = 0.0,
              noise: Optional[torch.Tensor] = None):
    """EmissionAbsorptionRaymarcher.forward on the GPU -> (features, depths, alpha, weights).
    noise: injected N(0,1) draws [..., P] (test mode); otherwise Philox normals when noise_std > 0."""
    _dev(sigma_raw, rgb, lengths, directions, bg, noise)
    R = lengths[..., 0].numel()
    P = lengths.shape[-1]
    if noise_std > 0.0:
        if noise is not None:
            o = cfg.opts(1, noise_std)
        else:
            seed, off = RNG.next(R * P)
            o = cfg.opts(2, noise_std, seed, off)
    else:
        o = cfg.opts(0, 0.0)
        noise = None
    return _CompositeFn.apply(bytes(o), sigma_raw, rgb, lengths, directions, bg, noise)


# ----------------------------------------------------------------------------------------- importance sampling
def sample_pdf(bins: torch.Tensor, weights: torch.Tensor, n_samples: int, det: bool = False,
               u: Optional[torch.Tensor] = None) -> torch.Tensor:
    """sample_pdf_python (renderers/utils.py:83-158). bins [..., nb+1], weights [..., nb]."""
    _dev(bins, weights, u)
    nb = weights.shape[-1]
    R = weights[..., 0].numel()
    b = _f32c(bins.reshape(R, nb + 1))
    w = _f32c(weights.reshape(R, nb))
    uu = None if (det or u is None) else _f32c(u.reshape(R, n_samples))
    out = torch.empty(R, n_samples, dtype=_F32, device=b.device)
    seed, off = RNG.next(R * n_samples)
    _C.check(_C.lib().yanerf_sample_pdf(_p(b), _p(w), R, nb, n_samples, int(det), _p(uu), seed, off, _p(out),
                                        _stream()), "yanerf_sample_pdf")
    return out.view(*weights.shape[:-1], n_samples)


def refine(lengths: torch.Tensor, ray_weights: torch.Tensor, n_fine: int, det: bool, add_input: bool = True,
           u: Optional[torch.Tensor] = None) -> torch.Tensor:
    """RayPointRefiner.forward's z computation (renderers/utils.py:48-65): midpoints, sample_pdf, cat, sort."""
    _dev(lengths, ray_weights, u)
    P = lengths.shape[-1]
    R = lengths[..., 0].numel()
    z = _f32c(lengths.detach().reshape(R, P))
    w = _f32c(ray_weights.detach().reshape(R, P))
    uu = None if (det or u is None) else _f32c(u.reshape(R, n_fine))
    tot = P + n_fine if add_input else n_fine
    out = torch.empty(R, tot, dtype=_F32, device=z.device)
    seed, off = RNG.next(R * n_fine)
    _C.check(_C.lib().yanerf_refine(_p(z), _p(w), R, P, n_fine, int(det), _p(uu), seed, off, int(add_input), _p(out),
                                    None, _stream()), "yanerf_refine")
    return out.view(*lengths.shape[:-1], tot)


# ----------------------------------------------------------------------------------------- loss / optimizer
def rgb_loss(pred: torch.Tensor, image: torch.Tensor, xys: torch.Tensor, scale: float):
    """Per-ray squared error vs the image gathered at integer xys, and d(scale*sum sq)/dpred."""
    _dev(pred, image, xys)
    B, H, W, C = image.shape
    R = pred.numel() // (B * C)
    pr = _f32c(pred.reshape(B, R, C))
    img = _f32c(image)
    xy = _f32c(xys.reshape(B, R, 2))
    sq = torch.empty(B, R, dtype=_F32, device=pr.device)
    g = torch.empty(B, R, C, dtype=_F32, device=pr.device)
    _C.check(_C.lib().yanerf_rgb_loss(_p(pr), _p(img), _p(xy), B, R, H, W, C, float(scale), _p(sq), _p(g), _stream()),
             "yanerf_rgb_loss")
    return sq, g


_OOB_FLAGS: dict = {}  # device -> sticky int32 out-of-image flag of yanerf_scatter_rays (set by the kernel, never cleared
# by it; cleared here when it is reported)


def _oob_flag(dev) -> torch.Tensor:
    f = _OOB_FLAGS.get(dev)
    if f is None:
        f = _OOB_FLAGS[dev] = torch.zeros(1, dtype=torch.int32, device=dev)
    return f


def check_scatter_bounds(dev) -> None:
    """Raise if any yanerf_scatter_rays call on `dev` since the last check met a pixel index outside its image (one
    host read-back for any number of scatter calls; skipped while a stream is being captured into a graph)."""
    f = _OOB_FLAGS.get(dev)
    if f is None or torch.cuda.is_current_stream_capturing():
        return
    if int(f.item()):
        f.zero_()
        raise RuntimeError("scatter_rays_to_image: a ray's pixel index x + W * y lies outside the image (torch's "
                           "scatter_ raises on it: index out of bounds)")


@torch.no_grad()
def scatter_rays(values: torch.Tensor, xys: torch.Tensor, image_height: int, image_width: int,
                 bg_color: Optional[torch.Tensor] = None, check: bool = True) -> torch.Tensor:
    """scatter_rays_to_image (pipelines/utils.py:299-323) on the device: values [B, *spatial, C] at integer-valued
    xys [B, *spatial, 2] onto a new [B, H, W, C] image filled with bg_color (when its last dim is C) or zeros. A host
    bg_color (the reference's own test passes a CPU tensor) is moved to the device; one whose last dim is not C is
    ignored, as the reference ignores it. A pixel index outside the image raises, as the reference's scatter_ does:
    the kernel sets a sticky per-device flag and `check_scatter_bounds` reads it back -- here when `check` (a caller
    scattering several tensors at the same xys passes check=False for all but the last: one host sync, not one per
    tensor)."""
    if bg_color is not None and bg_color.shape[-1] != values.shape[-1]:
        bg_color = None
    if bg_color is not None and not bg_color.is_cuda:
        bg_color = bg_color.to(values.device)
    _dev(values, xys, bg_color)
    B, *ts, C = values.shape
    _, *gs, _ = xys.shape
    assert ts == gs, f"{ts} vs. {gs}"
    v = _f32c(values.reshape(B, -1, C))
    xy = _f32c(xys.reshape(B, -1, 2))
    bg = None
    if bg_color is not None and bg_color.shape[-1] == C:
        if bg_color.numel() != C:
            raise NotImplementedError("scatter_rays: a per-pixel bg_color (the reference's _rasterize_mc_samples "
                                      "passes None); only a [C] background is supported")
        bg = _f32c(bg_color.reshape(C))
    out = torch.empty(B, int(image_height), int(image_width), C, dtype=_F32, device=v.device)
    _C.check(_C.lib().yanerf_scatter_rays(_p(v), _p(xy), B, v.shape[1], C, int(image_height), int(image_width),
                                          _p(bg), _p(out), _p(_oob_flag(v.device)), _stream()), "yanerf_scatter_rays")
    if check:
        check_scatter_bounds(v.device)
    return out if values.dtype == _F32 else out.to(values.dtype)


def adam_step(params: torch.Tensor, grads: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, *, lr: float,
              betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, step: int) -> None:
    _dev(params, grads, exp_avg, exp_avg_sq)
    _C.check(_C.lib().yanerf_adam(_p(params), _p(grads), _p(exp_avg), _p(exp_avg_sq), params.numel(), float(lr),
                                  float(betas[0]), float(betas[1]), float(eps), float(weight_decay), int(step),
                                  _stream()), "yanerf_adam")
