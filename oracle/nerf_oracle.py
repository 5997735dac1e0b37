"""CPU ORACLE for the yet-another-nerf volumetric-rendering hot path.

TEST INFRASTRUCTURE ONLY. This module is a numpy restatement of the reference's
algorithm (xk-huang/yet-another-nerf, snapshot v0) and exists solely as the
checker for the HIP path. Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import it. The product path
(yet-another-nerf_amd/) never imports, links or calls anything under oracle/.

Parity pinning: every function here is checked against golden vectors produced
by running the reference itself in the build container
(tests/golden/make_golden.py -> tests/golden/*.npz; see tests/test_oracle_golden.py).

Arithmetic mirrors the reference: float32 everywhere, except the cumulative sums,
which torch's CPU kernel accumulates in double (at::acc_type<float,false>) and
which are restated in float64 here.

Citations are `path:line` into /root/reference.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

f32 = np.float32


# ============================================================================ helpers
def torch_linspace(start: float, end: float, n: int) -> np.ndarray:
    """torch.linspace on CPU for float32: start + step*i on the first half, end - step*(n-1-i) on the second
    (aten RangeFactoriesKernel linspace_kernel), each a FUSED multiply-add in the compiled kernel (bit for bit against
    torch.linspace on 449,515 values: tools/linspace_model.py). The fma is emulated in float64: step * i is exact there
    (24-bit x <= 24-bit), so only the add rounds, then once more to float32 (a double rounding that never occurred in
    the check). Used at ray_sampler.py:285-291, renderers/utils.py:109."""
    start, end = f32(start), f32(end)
    if n == 1:
        return np.array([start], dtype=f32)
    step = f32((end - start) / f32(n - 1))
    i = np.arange(n)
    half = n // 2
    s64, i64 = np.float64(step), i.astype(np.float64)
    out = np.where(i < half, s64 * i64 + np.float64(start), -s64 * (n - 1 - i64) + np.float64(end))
    return out.astype(np.float32).astype(f32)


def cumsum_acc64(x: np.ndarray, axis: int = -1) -> np.ndarray:
    """torch.cumsum on CPU accumulates float32 in double and rounds each output to float32."""
    return np.cumsum(x.astype(np.float64), axis=axis).astype(f32)


def torch_sum_lastdim(x: np.ndarray) -> np.ndarray:
    """float32 `x.sum(-1, keepdim=True)` in torch's CPU order (aten ReduceOpsKernel cascade_sum ->
    vectorized_inner_sum with 8-wide vectors and a 4-way ILP row_sum; pinned bit-exact against torch in the
    build container). The normalizer's rounding decides sample_pdf's `denom < eps` branch
    (renderers/utils.py:128-129), so it is restated exactly rather than with numpy's pairwise sum."""
    x = x.astype(f32)
    n = x.shape[-1]
    V = 8
    nv = n // V
    vs = [x[..., i * V:(i + 1) * V] for i in range(nv)]
    size_ilp = nv // 4
    assert size_ilp < 16, "exact restatement covers rows shorter than 512"
    if size_ilp >= 1:
        ps = [vs[k].copy() for k in range(4)]
        for i in range(1, size_ilp):
            for k in range(4):
                ps[k] = (ps[k] + vs[4 * i + k]).astype(f32)
    else:
        ps = [np.zeros(x.shape[:-1] + (V,), f32) for _ in range(4)]
    for i in range(size_ilp * 4, nv):
        ps[0] = (ps[0] + vs[i]).astype(f32)
    for k in range(1, 4):
        ps[0] = (ps[0] + ps[k]).astype(f32)
    acc = np.zeros(x.shape[:-1], f32)
    for k in range(nv * V, n):
        acc = (acc + x[..., k]).astype(f32)
    if nv > 0:
        for lane in range(V):
            acc = (acc + ps[0][..., lane]).astype(f32)
    return acc[..., None]


def relu(x):
    return np.maximum(x, f32(0.0)).astype(f32)


def sigmoid(x):
    return (f32(1.0) / (f32(1.0) + np.exp(-x))).astype(f32)


# ============================================================================ ray sampler
def get_xy_grid(H: int, W: int) -> np.ndarray:
    """ray_samplers/utils.py:12-24: (H, W, 2) grid, last dim = (x=col, y=row), integer-valued."""
    ys = torch_linspace(0, H - 1, H)
    xs = torch_linspace(0, W - 1, W)
    gy, gx = np.meshgrid(ys, xs, indexing="ij")
    return np.stack([gx, gy], axis=-1).astype(f32)


def jiggle_within_stratas(z: np.ndarray, u: np.ndarray) -> np.ndarray:
    """ray_sampler.py:361-386."""
    mids = f32(0.5) * (z[..., 1:] + z[..., :-1])
    upper = np.concatenate([mids, z[..., -1:]], -1)
    lower = np.concatenate([z[..., :1], mids], -1)
    return (lower + (upper - lower) * u).astype(f32)


def xy_to_ray_bundle(poses: np.ndarray, cfg_W: int, cfg_H: int, focal: np.ndarray, xy: np.ndarray,
                     near: float, far: float, P: int, jitter_u: Optional[np.ndarray] = None):
    """ray_sampler.py:249-314. poses (B,3,4); xy (B,*S,2); returns origins, directions, lengths, xys.
    Quirk reproduced: the principal point uses the CONFIGURED width/height (cfg_W, cfg_H), not an override."""
    B = xy.shape[0]
    S = xy.shape[1:-1]
    z = torch_linspace(near, far, P)
    lengths = np.broadcast_to(z, (B, *S, P)).astype(f32)
    if jitter_u is not None:
        lengths = jiggle_within_stratas(lengths, jitter_u.reshape(lengths.shape))
    pz = poses.reshape(B, *([1] * len(S)), 3, 4)
    origins = np.broadcast_to(pz[..., 3], (B, *S, 3)).astype(f32)
    fz = focal.reshape(B, *([1] * len(S))).astype(f32)
    v = np.stack([(xy[..., 0] - f32(cfg_W * 0.5)) / fz, (xy[..., 1] - f32(cfg_H * 0.5)) / fz,
                  np.ones(xy.shape[:-1], f32)], -1).astype(f32)
    prod = pz[..., :3, :3] * v[..., None, :]
    directions = ((prod[..., 0] + prod[..., 1]) + prod[..., 2]).astype(f32)
    return origins, directions, lengths, xy.astype(f32)


def sample_rays_eval(poses, focal, cfg_W, cfg_H, near, far, P, H=None, W=None):
    """_RaySampler.forward FULL_GRID branch (ray_sampler.py:164-246)."""
    B = poses.shape[0]
    H = cfg_H if H is None else H
    W = cfg_W if W is None else W
    xy = np.broadcast_to(get_xy_grid(H, W), (B, H, W, 2))
    return xy_to_ray_bundle(poses, cfg_W, cfg_H, focal, xy, near, far, P)


def sample_rays_train(poses, focal, cfg_W, cfg_H, near, far, P, pixel_ids, jitter_u):
    """MASK_SAMPLE branch with injected multinomial ids (ray_sampler.py:181-229) and stratified jitter."""
    B = poses.shape[0]
    grid = get_xy_grid(cfg_H, cfg_W).reshape(-1, 2)
    xy = grid[pixel_ids][:, :, None, :]  # (B, n, 1, 2)
    return xy_to_ray_bundle(poses, cfg_W, cfg_H, focal, xy, near, far, P, jitter_u)


# ============================================================================ NeRF MLP
def harmonic_embedding(x: np.ndarray, n_freq: int, append_input: bool = True) -> np.ndarray:
    """models/utils.py:17-103: [sin(x_i*2^k) (i-major,k-minor), cos(...), x]."""
    freqs = (f32(2.0) ** np.arange(n_freq, dtype=f32)).astype(f32)
    e = (x[..., None] * freqs).reshape(*x.shape[:-1], -1).astype(f32)
    parts = [np.sin(e).astype(f32), np.cos(e).astype(f32)] + ([x.astype(f32)] if append_input else [])
    return np.concatenate(parts, -1)


def normalize(d: np.ndarray) -> np.ndarray:
    """torch.nn.functional.normalize(d, dim=-1) (nerf_mlp.py:105)."""
    n = np.sqrt(np.sum(d.astype(f32) * d, -1, keepdims=True)).astype(f32)
    return (d / np.maximum(n, f32(1e-12))).astype(f32)


@dataclass
class MLPArch:
    n_layers: int = 8
    input_skips: Sequence[int] = (5,)
    n_harmonic_functions_xyz: int = 10
    n_hidden_neurons_xyz: int = 256
    n_harmonic_functions_dir: int = 4
    n_hidden_neurons_dir: int = 128
    color_dim: int = 3

    @staticmethod
    def from_dict(d: dict) -> "MLPArch":
        keys = MLPArch.__dataclass_fields__.keys()
        return MLPArch(**{k: v for k, v in d.items() if k in keys})


@dataclass
class MLPCache:
    embed: np.ndarray = None
    layer_in: List[np.ndarray] = field(default_factory=list)
    layer_out: List[np.ndarray] = field(default_factory=list)
    features: np.ndarray = None
    dir_embed: np.ndarray = None
    inter: np.ndarray = None
    c0: np.ndarray = None
    rgb: np.ndarray = None
    n_rays: int = 0
    P: int = 0
    layer_pre: List[np.ndarray] = field(default_factory=list)  # trunk pre-activations (before the ReLU)
    c0_pre: np.ndarray = None  # colour hidden pre-activation
    trunk_masks: Optional[List[np.ndarray]] = None  # the ReLU decisions used (None: the activations' own, y > 0)
    color_mask: Optional[np.ndarray] = None


def linear(x, W, b):
    y = x @ W.T.astype(f32)
    if b is not None:
        y = y + b
    return y.astype(f32)


def _relu_with(z: np.ndarray, mask: Optional[np.ndarray]) -> np.ndarray:
    """relu(z), or -- with an injected ReLU decision per unit -- z where mask, 0 elsewhere."""
    return relu(z) if mask is None else np.where(mask, z, f32(0.0)).astype(f32)


def nerf_mlp_forward(params: Dict[str, np.ndarray], arch: MLPArch, origins, directions, lengths, code=None,
                     relu_masks: Optional[dict] = None):
    """NeRFMLP.forward (nerf_mlp.py:117-177) with MLPWithInputSkips (nerf_mlp.py:267-289) and
    LinearWithRepeat (models/utils.py:207-211). origins/directions (..., 3), lengths (..., P).
    `code` (latent_dim,): one batch element's global code, appended to every point's xyz embedding
    (create_embeddings_for_implicit_function / broadcast_global_code, nerf_mlp.py:299-335).
    relu_masks (test support): {"trunk": [n_layers bool (R*P, hidden)], "color": bool (R*P, hidden_dir)} -- the
    ReLU decisions of another fp32 evaluation of the same network (the reference's, recorded in the golden, or the
    HIP kernels'), used instead of this evaluation's own signs, forward and backward: a pre-activation within
    rounding of zero can fall on either side of the kink in two correct fp32 implementations, and with it that
    unit's whole gradient contribution (tests/parity_gates.py).
    Returns sigma (..., P, 1), rgb (..., P, C), cache."""
    lead = lengths.shape[:-1]
    P = lengths.shape[-1]
    R = int(np.prod(lead)) if lead else 1
    o = origins.reshape(R, 3).astype(f32)
    d = directions.reshape(R, 3).astype(f32)
    t = lengths.reshape(R, P).astype(f32)
    pts = (o[:, None, :] + t[:, :, None] * d[:, None, :]).astype(f32)  # models/utils.py:244
    embed = harmonic_embedding(pts.reshape(R * P, 3), arch.n_harmonic_functions_xyz)
    if code is not None:
        embed = np.concatenate([embed, np.broadcast_to(np.asarray(code, f32), (R * P, len(code)))], -1)
    cache = MLPCache(embed=embed, n_rays=R, P=P)
    if relu_masks is not None:
        cache.trunk_masks = [np.asarray(m, bool).reshape(R * P, -1) for m in relu_masks["trunk"]]
        cache.color_mask = np.asarray(relu_masks["color"], bool).reshape(R * P, -1)
    y = embed
    for li in range(arch.n_layers):
        if li in arch.input_skips:
            y = np.concatenate([y, embed], -1)
        cache.layer_in.append(y)
        z = linear(y, params[f"xyz_encoder.mlp.{li}.0.weight"], params[f"xyz_encoder.mlp.{li}.0.bias"])
        cache.layer_pre.append(z)
        y = _relu_with(z, None if cache.trunk_masks is None else cache.trunk_masks[li])
        cache.layer_out.append(y)
    feats = y
    cache.features = feats
    sigma = linear(feats, params["density_layer.weight"], params["density_layer.bias"])
    dir_embed = harmonic_embedding(normalize(d), arch.n_harmonic_functions_dir)  # (R, 27)
    cache.dir_embed = dir_embed
    inter = linear(feats, params["intermediate_linear.weight"], params["intermediate_linear.bias"])
    cache.inter = inter
    Wc = params["color_layer.0.weight"]
    n1 = inter.shape[-1]
    out1 = linear(inter, Wc[:, :n1], params["color_layer.0.bias"]).reshape(R, P, -1)
    out2 = linear(dir_embed, Wc[:, n1:], None)
    c0_pre = (out1 + out2[:, None, :]).astype(f32).reshape(R * P, -1)
    cache.c0_pre = c0_pre
    c0 = _relu_with(c0_pre, cache.color_mask)
    cache.c0 = c0
    rgb = sigmoid(linear(c0, params["color_layer.2.weight"], params["color_layer.2.bias"]))
    cache.rgb = rgb
    return sigma.reshape(*lead, P, 1), rgb.reshape(*lead, P, -1), cache


def nerf_mlp_backward(params: Dict[str, np.ndarray], arch: MLPArch, cache: MLPCache, g_sigma, g_rgb,
                      abs_terms: bool = False):
    """Manual reverse-mode of nerf_mlp_forward; returns {param_name: grad} (autograd semantics of the
    reference modules: ReLU grad where output > 0; sigmoid grad y(1-y)). Every parameter gradient is a sum over the
    points; abs_terms=True also returns, per gradient element, the sum of the ABSOLUTE values of its terms (float64),
    the scale of the fp32 summation-order error any implementation's sum of those terms carries (parity_gates.SUM_REL)."""
    R, P = cache.n_rays, cache.P
    N = R * P
    gs = g_sigma.reshape(N, 1).astype(f32)
    gr = g_rgb.reshape(N, -1).astype(f32)
    grads: Dict[str, np.ndarray] = {}
    absg: Dict[str, np.ndarray] = {}

    def a(x):
        return np.abs(np.asarray(x, np.float64))

    def reduce(name, g, x=None):  # grads[name] = g^T x (or the column sums of g), and its |terms| sums
        grads[name] = (g.T @ x).astype(f32) if x is not None else g.sum(0).astype(f32)
        if abs_terms:
            absg[name] = a(g).T @ a(x) if x is not None else a(g).sum(0)

    rgb = cache.rgb
    gu = (gr * (f32(1.0) - rgb) * rgb).astype(f32)
    reduce("color_layer.2.weight", gu, cache.c0)
    reduce("color_layer.2.bias", gu)
    gc0 = (gu @ params["color_layer.2.weight"]).astype(f32)
    gz = np.where(cache.c0 > 0 if cache.color_mask is None else cache.color_mask, gc0, f32(0.0)).astype(f32)
    n1 = cache.inter.shape[-1]
    gW1 = (gz.T @ cache.inter).astype(f32)
    gz_ray = gz.reshape(R, P, -1).sum(1).astype(f32)
    gW2 = (gz_ray.T @ cache.dir_embed).astype(f32)
    grads["color_layer.0.weight"] = np.concatenate([gW1, gW2], 1)
    if abs_terms:
        absg["color_layer.0.weight"] = np.concatenate(
            [a(gz).T @ a(cache.inter), a(gz).reshape(R, P, -1).sum(1).T @ a(cache.dir_embed)], 1)
    reduce("color_layer.0.bias", gz)
    g_inter = (gz @ params["color_layer.0.weight"][:, :n1]).astype(f32)
    reduce("intermediate_linear.weight", g_inter, cache.features)
    reduce("intermediate_linear.bias", g_inter)
    reduce("density_layer.weight", gs, cache.features)
    reduce("density_layer.bias", gs)
    gy = (g_inter @ params["intermediate_linear.weight"] + gs @ params["density_layer.weight"]).astype(f32)
    for li in reversed(range(arch.n_layers)):
        y = cache.layer_out[li]
        gzl = np.where(y > 0 if cache.trunk_masks is None else cache.trunk_masks[li], gy, f32(0.0)).astype(f32)
        W = params[f"xyz_encoder.mlp.{li}.0.weight"]
        reduce(f"xyz_encoder.mlp.{li}.0.weight", gzl, cache.layer_in[li])
        reduce(f"xyz_encoder.mlp.{li}.0.bias", gzl)
        if li == 0:
            break
        gin = (gzl @ W).astype(f32)
        gy = gin[:, : gin.shape[1] - cache.embed.shape[1]] if li in arch.input_skips else gin
    return (grads, absg) if abs_terms else grads


# ============================================================================ raymarcher
@dataclass
class RaymarchOpts:
    capping_function: str = "exponential"
    weight_function: str = "product"
    background_opacity: float = 1e10
    blend_output: bool = False
    background_density_bias: float = 0.0
    hard_background: bool = False
    density_relu: bool = True


def _cap(x, kind):
    if kind == "exponential":
        return (f32(1.0) - np.exp(-x)).astype(f32)
    return np.minimum(x, f32(1.0)).astype(f32)


def _cap_grad(x, kind):
    if kind == "exponential":
        return np.exp(-x).astype(f32)
    return (x <= 1.0).astype(f32)


def raymarch_forward(densities, features, lengths, directions, opts: RaymarchOpts, noise=None, bg=None,
                     default_bg=(0.0,)):
    """EmissionAbsorptionRaymarcher.forward (multipass_emission_absorpsion_renderer.py:154-239).
    densities (R,P,1), features (R,P,C), lengths (R,P), directions (R,3), noise (R,P) already * std.
    Returns features (R,C), depths (R,1), opacities (R,1), weights (R,P), ctx."""
    dens = densities[..., 0].astype(f32)
    t = lengths.astype(f32)
    deltas = np.concatenate([t[..., 1:] - t[..., :-1], np.full(t[..., :1].shape, f32(opts.background_opacity))], -1)
    dn = np.sqrt(np.sum(directions.astype(f32) ** 2, -1)).astype(f32)
    deltas = (deltas * dn[..., None]).astype(f32)
    pre = dens if noise is None else (dens + noise).astype(f32)
    s = (relu(pre) + f32(opts.background_density_bias)).astype(f32) if opts.density_relu else pre
    wd = (deltas * s).astype(f32)
    capped = _cap(wd, opts.capping_function)
    cs = cumsum_acc64(wd)
    op = _cap(cs, opts.capping_function)
    opac = op[..., -1:]
    absorp = np.roll(f32(1.0) - op, 1, axis=-1).astype(f32)
    absorp[..., :1] = 1.0
    if opts.weight_function == "product":
        w = (capped * absorp).astype(f32)
    else:
        w = np.minimum(capped, absorp).astype(f32)
    depths = np.sum(w * t, -1, keepdims=True).astype(f32)
    C = features.shape[-1]
    if bg is None:
        bgc = np.broadcast_to(np.asarray(default_bg, f32), (*features.shape[:-2], len(default_bg)))
    else:
        bgc = bg.astype(f32)
    if not opts.hard_background:
        F = np.sum(w[..., None] * features, -2).astype(f32)
        A = opac if opts.blend_output else f32(1.0)
        feats = (A * F + (f32(1.0) - opac) * bgc).astype(f32)
    else:
        fx = np.concatenate([features[..., :-1, :], np.broadcast_to(bgc, (*features.shape[:-2], C))[..., None, :]], -2)
        F = np.sum(w[..., None] * fx, -2).astype(f32)
        feats = F
    ctx = dict(dens=dens, pre=pre, deltas=deltas, wd=wd, capped=capped, cs=cs, op=op, absorp=absorp, w=w, t=t,
               F=F, bgc=bgc, opac=opac, features=features, opts=opts)
    return feats, depths, opac, w, ctx


def raymarch_backward(ctx, g_feat, g_depth=None, g_alpha=None):
    """Reverse-mode of raymarch_forward -> (g_densities (R,P,1), g_features (R,P,C))."""
    o: RaymarchOpts = ctx["opts"]
    w, t, features, opac, bgc, F = ctx["w"], ctx["t"], ctx["features"], ctx["opac"], ctx["bgc"], ctx["F"]
    g_feat = g_feat.astype(f32)
    gD = np.zeros(t.shape[:-1] + (1,), f32) if g_depth is None else g_depth.astype(f32)
    gA = np.zeros(t.shape[:-1] + (1,), f32) if g_alpha is None else g_alpha.astype(f32)
    if not o.hard_background:
        A = opac if o.blend_output else f32(1.0)
        gF = (g_feat * A).astype(f32)
        g_op_last = gA + np.sum(-g_feat * np.broadcast_to(bgc, g_feat.shape), -1, keepdims=True)
        if o.blend_output:
            g_op_last = g_op_last + np.sum(g_feat * F, -1, keepdims=True)
        g_features = (w[..., None] * gF[..., None, :]).astype(f32)
        gw = np.sum(gF[..., None, :] * features, -1) + gD * t
    else:
        C = features.shape[-1]
        fx = np.concatenate([features[..., :-1, :], np.broadcast_to(bgc, (*features.shape[:-2], C))[..., None, :]], -2)
        g_features = (w[..., None] * g_feat[..., None, :]).astype(f32)
        g_features[..., -1, :] = 0.0
        gw = np.sum(g_feat[..., None, :] * fx, -1) + gD * t
        g_op_last = gA
    gw = gw.astype(f32)
    capped, absorp = ctx["capped"], ctx["absorp"]
    if o.weight_function == "product":
        g_capped, g_abs = gw * absorp, gw * capped
    else:
        eq = capped == absorp
        g_capped = np.where(eq, gw / 2, np.where(capped < absorp, gw, 0.0))
        g_abs = np.where(eq, gw / 2, np.where(absorp < capped, gw, 0.0))
    g_op = np.zeros_like(w)
    g_op[..., :-1] -= g_abs[..., 1:]
    g_op[..., -1:] += g_op_last
    g_cs = g_op * _cap_grad(ctx["cs"], o.capping_function)
    g_wd = np.flip(np.cumsum(np.flip(g_cs.astype(np.float64), -1), -1), -1).astype(f32)
    g_wd = g_wd + g_capped * _cap_grad(ctx["wd"], o.capping_function)
    g_s = (g_wd * ctx["deltas"]).astype(f32)
    g_dens = np.where(ctx["pre"] > 0, g_s, f32(0.0)).astype(f32) if o.density_relu else g_s
    return g_dens[..., None], g_features


# ============================================================================ importance sampling
def sample_pdf(bins: np.ndarray, weights: np.ndarray, n_samples: int, det: bool, u: Optional[np.ndarray] = None,
               eps: float = 1e-5) -> np.ndarray:
    """sample_pdf_python (renderers/utils.py:83-158). bins (R, nb+1), weights (R, nb)."""
    w = (weights + f32(eps)).astype(f32)
    if w.min() <= 0:
        raise ValueError("Negative weights provided.")
    pdf = (w / torch_sum_lastdim(w)).astype(f32)
    cdf = cumsum_acc64(pdf)
    cdf = np.concatenate([np.zeros_like(cdf[..., :1]), cdf], -1)
    if det:
        u = np.broadcast_to(torch_linspace(0.0, 1.0, n_samples), (*cdf.shape[:-1], n_samples)).astype(f32)
    else:
        assert u is not None, "random sample_pdf needs injected uniforms"
        u = u.reshape(*cdf.shape[:-1], n_samples).astype(f32)
    R = cdf.shape[0]
    inds = np.stack([np.searchsorted(cdf[r], u[r], side="right") for r in range(R)])
    below = np.maximum(inds - 1, 0)
    above = np.minimum(inds, cdf.shape[-1] - 1)
    cb = np.take_along_axis(cdf, below, -1)
    ca = np.take_along_axis(cdf, above, -1)
    bb = np.take_along_axis(bins, below, -1)
    ba = np.take_along_axis(bins, above, -1)
    denom = (ca - cb).astype(f32)
    denom = np.where(denom < f32(eps), f32(1.0), denom).astype(f32)
    tt = ((u - cb) / denom).astype(f32)
    return (bb + tt * (ba - bb)).astype(f32)


def lerp_half(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """torch.lerp(a, b, 0.5) on CPU: weight >= 0.5 branch, b - (b - a) * (1 - w)."""
    return (b - (b - a) * f32(0.5)).astype(f32)


def refine(lengths: np.ndarray, ray_weights: np.ndarray, n_pts: int, random_sampling: bool,
           u: Optional[np.ndarray] = None, add_input_samples: bool = True) -> np.ndarray:
    """RayPointRefiner.forward (renderers/utils.py:48-69): midpoints, sample_pdf(w[1:-1]), cat, sort."""
    lead = lengths.shape[:-1]
    P = lengths.shape[-1]
    z = lengths.reshape(-1, P).astype(f32)
    mids = lerp_half(z[:, 1:], z[:, :-1])
    s = sample_pdf(mids, ray_weights.reshape(-1, P)[:, 1:-1], n_pts, det=not random_sampling, u=u)
    zz = np.concatenate([z, s], -1) if add_input_samples else s
    return np.sort(zz, -1).reshape(*lead, -1).astype(f32)


# ============================================================================ metrics
def rgb_metrics(gt: np.ndarray, pred: np.ndarray) -> Dict[str, np.ndarray]:
    """pipelines/utils.py:189-196 (mse, huber scaling 0.03)."""
    B = gt.shape[0]
    diff = ((pred.reshape(B, -1) - gt.reshape(B, -1)) ** 2).astype(f32)
    mse = diff.mean(-1).astype(f32)
    s = f32(0.03)
    huber = ((np.sqrt(np.maximum(f32(1.0) + mse / (s * s), 0) + f32(1e-4)) - 1) * s).astype(f32)
    return {"rgb_mse": mse, "rgb_huber": huber}


def psnr_from_mse(mse: float) -> float:
    """runners/utils.py:270-283 mse2psnr."""
    return float(-10.0 * np.log10(max(mse, 1e-10)))


# ============================================================================ two-pass renderer
@dataclass
class RenderCfg:
    n_pts_coarse: int = 64
    n_pts_fine: int = 128
    near: float = 2.0
    far: float = 6.0
    density_noise_std: float = 0.0
    raymarch: RaymarchOpts = field(default_factory=lambda: RaymarchOpts(background_density_bias=1e-6))
    bg_color: Tuple[float, ...] = (0.0, 0.0, 0.0)
    append_coarse_samples_to_fine: bool = True


def render_two_pass(params_c, params_f, arch, cfg: RenderCfg, origins, directions, lengths, bg=None,
                    noise_c=None, noise_f=None, pdf_u=None, random_sampling=False, z_fine=None, relu_masks=None):
    """MultipassEmissionAbsorpsionRenderer._run_raymarcher recursion (renderer.py:84-117) for 2 passes.
    origins/directions (R,3), lengths (R,Pc). z_fine (optional): the refined depths to run the fine pass at instead
    of this refinement (e.g. the reference's own, recorded in the golden). relu_masks (optional): (coarse, fine)
    ReLU decisions for nerf_mlp_forward. Returns dict with both stages and caches."""
    R = lengths.shape[0]
    mc, mf = relu_masks if relu_masks is not None else (None, None)
    sc, cc, cache_c = nerf_mlp_forward(params_c, arch, origins, directions, lengths, relu_masks=mc)
    fc, dc, ac, wc, ctx_c = raymarch_forward(sc, cc, lengths, directions, cfg.raymarch,
                                             noise=None if noise_c is None else noise_c.reshape(R, -1),
                                             bg=bg, default_bg=cfg.bg_color)
    zf = refine(lengths, wc, cfg.n_pts_fine, random_sampling, u=pdf_u,
                add_input_samples=cfg.append_coarse_samples_to_fine) if z_fine is None else \
        np.asarray(z_fine, f32).reshape(R, -1)
    sf, cf, cache_f = nerf_mlp_forward(params_f, arch, origins, directions, zf, relu_masks=mf)
    ff, df, af, wf, ctx_f = raymarch_forward(sf, cf, zf, directions, cfg.raymarch,
                                             noise=None if noise_f is None else noise_f.reshape(R, -1),
                                             bg=bg, default_bg=cfg.bg_color)
    return dict(coarse=(fc, dc, ac, wc), fine=(ff, df, af, wf), z_fine=zf, cache_c=cache_c, cache_f=cache_f,
                ctx_c=ctx_c, ctx_f=ctx_f)


def train_step_grads(params_c, params_f, arch, cfg: RenderCfg, origins, directions, lengths, gt_rgb,
                     noise_c, noise_f, pdf_u, z_fine=None, relu_masks=None, abs_terms: bool = False,
                     loss_rays: Optional[int] = None):
    """One training step's objective and parameter gradients (nerf_pipeline.py:181-213, 284-305; apis.py:87-88):
    objective = mse(fine) + mse(coarse); noise_* already include density_noise_std. abs_terms=True adds each gradient
    element's sum of absolute term values (abs_fine / abs_coarse, nerf_mlp_backward). loss_rays: the number of rays the
    mean-squared error averages over when these rays are one chunk of a larger step (the gradients of a step are sums
    over its rays, so chunks' gradients add up; the objective is this chunk's own)."""
    R = lengths.shape[0]
    out = render_two_pass(params_c, params_f, arch, cfg, origins, directions, lengths, noise_c=noise_c,
                          noise_f=noise_f, pdf_u=pdf_u, random_sampling=True, z_fine=z_fine,
                          relu_masks=relu_masks)
    gt = gt_rgb.reshape(R, 3)
    mse_f = rgb_metrics(gt[None], out["fine"][0][None])["rgb_mse"]
    mse_c = rgb_metrics(gt[None], out["coarse"][0][None])["rgb_mse"]
    scale = f32(2.0 / ((R if loss_rays is None else int(loss_rays)) * 3))
    grads, absg = [], []
    for stage, params, cache, ctx in (("fine", params_f, out["cache_f"], out["ctx_f"]),
                                      ("coarse", params_c, out["cache_c"], out["ctx_c"])):
        g_feat = ((out[stage][0] - gt) * scale).astype(f32)
        g_dens, g_cols = raymarch_backward(ctx, g_feat)
        r = nerf_mlp_backward(params, arch, cache, g_dens, g_cols, abs_terms=abs_terms)
        grads.append(r[0] if abs_terms else r)
        absg.append(r[1] if abs_terms else None)
    res = dict(objective=float(mse_f[0] + mse_c[0]), loss_rgb_mse=mse_f, loss_prev_stage_rgb_mse=mse_c,
               grads_fine=grads[0], grads_coarse=grads[1], render=out)
    if abs_terms:
        res.update(abs_fine=absg[0], abs_coarse=absg[1])
    return res
