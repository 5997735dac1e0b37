"""Generate golden input/output vectors by running the REFERENCE implementation.

Run ONLY in the survey/build container, where /root/reference exists:

    python tests/golden/make_golden.py

It imports the reference (`yanerf.pipelines` from /root/reference) in-process
with the small stand-ins under tests/golden/_stubs for third-party modules the
image lacks (addict, yapf, imageio, omegaconf, cv2, torch._six). Every random
draw the reference makes (torch.multinomial / rand_like / randn_like / rand) is
recorded through a pass-through wrapper, so the fixtures hold the exact
uniforms/normals the reference consumed and our kernels can be driven with the
same values ("injected randomness" test mode).

Outputs (data only: inputs + expected outputs) go to tests/golden/*.npz. The
reference source never leaves /root/reference. Nothing in the GPU tests, bench
or smoke() runs this script.
"""
from __future__ import annotations

import os
import sys
import types
import zlib
from contextlib import contextmanager
from functools import partial
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REF = Path(os.environ.get("YANERF_REFERENCE", "/root/reference"))
sys.path.insert(0, str(HERE / "_stubs"))
sys.path.insert(0, str(REF))
sys.path.insert(0, str(HERE))

import torch  # noqa: E402

_six = types.ModuleType("torch._six")
_six.string_classes = (str, bytes)
sys.modules.setdefault("torch._six", _six)

from weights import LEGO_ARCH, SMALL_ARCH, checksum, load_trained_params, make_nerf_mlp_params  # noqa: E402
from scene import synthetic_pose  # noqa: E402

from yanerf.pipelines.builder import PIPELINES  # noqa: E402
from yanerf.pipelines.models import MODELS  # noqa: E402
from yanerf.pipelines.models.utils import HarmonicEmbedding  # noqa: E402
from yanerf.pipelines.ray_samplers import RAY_SAMPLERS  # noqa: E402
from yanerf.pipelines.renderers import RENDERERS  # noqa: E402
from yanerf.pipelines.renderers.multipass_emission_absorpsion_renderer import (  # noqa: E402
    EmissionAbsorptionRaymarcher,
)
from yanerf.pipelines.renderers.utils import RayPointRefiner, sample_pdf  # noqa: E402
from yanerf.pipelines.utils import EvaluationMode  # noqa: E402
from yanerf.utils.config import Config  # noqa: E402

torch.set_num_threads(8)


# ----------------------------------------------------------------------------- randomness capture
class Recorder:
    def __init__(self):
        self.log = []

    @contextmanager
    def capture(self):
        orig = {n: getattr(torch, n) for n in ("multinomial", "rand_like", "randn_like", "rand")}

        def wrap(name):
            f = orig[name]

            def g(*a, **k):
                out = f(*a, **k)
                self.log.append((name, out.detach().clone()))
                return out

            return g

        for n in orig:
            setattr(torch, n, wrap(n))
        try:
            yield self
        finally:
            for n, f in orig.items():
                setattr(torch, n, f)

    def take(self, name):
        return [t for (n, t) in self.log if n == name]


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def build_mlp(arch, seed):
    cfg = dict(type="NeRFMLP", **arch, harmonic_functions_xyz_append_intput=True,
               harmonic_functions_dir_append_intput=True, latent_dim=0, input_xyz=True, input_dir=True)
    model = MODELS.build(Config(dict(model=cfg)).model)
    params = make_nerf_mlp_params(arch, seed)
    sd = model.state_dict()
    assert set(sd.keys()) == set(params.keys()), (sorted(sd.keys()), sorted(params.keys()))
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    return model, params


# ----------------------------------------------------------------------------- cases
def gen_harmonic(out):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(257, 3, generator=g) * 3.0
    out["harmonic"] = dict(
        x=np32(x),
        xyz10=np32(HarmonicEmbedding(10, append_input=True)(x)),
        dir4=np32(HarmonicEmbedding(4, append_input=True)(x)),
        xyz8=np32(HarmonicEmbedding(8, append_input=True)(x)),
    )


def gen_raysampler(out):
    g = torch.Generator().manual_seed(1)
    for tag, cfg in (
        ("small", dict(type="RaySampler", image_width=10, image_height=6, n_rays_per_image_sampled_from_mask=4,
                       min_depth=0.5, max_depth=1.0, scene_extent=0.0, n_pts_per_ray_training=5,
                       n_pts_per_ray_evaluation=5, stratified_point_sampling_training=True,
                       stratified_point_sampling_evaluation=False)),
        ("lego", dict(type="RaySampler", image_width=800, image_height=800, n_rays_per_image_sampled_from_mask=64,
                      min_depth=2.0, max_depth=6.0, scene_extent=0.0, n_pts_per_ray_training=64,
                      n_pts_per_ray_evaluation=64, stratified_point_sampling_training=True,
                      stratified_point_sampling_evaluation=False)),
    ):
        rs = RAY_SAMPLERS.build(Config(dict(r=cfg)).r)
        poses = torch.randn(2, 3, 4, generator=g)
        focal = torch.tensor([500.0, 731.5])
        d = dict(poses=np32(poses), focal=np32(focal))
        # evaluation, configured grid (lego: override to 12x9 to keep the fixture small; quirk: principal point
        # still uses the configured W/H, reference ray_sampler.py:236-246, 302-303)
        kw = {} if tag == "small" else dict(image_height=9, image_width=12)
        rb = rs(poses, focal, EvaluationMode.EVALUATION, **kw)
        for k, v in rb._asdict().items():
            d[f"eval_{k}"] = np32(v)
        rb = rs(poses, focal, EvaluationMode.EVALUATION, image_height=3, image_width=6, min_depth=15.0, max_depth=30.0)
        for k, v in rb._asdict().items():
            d[f"evalov_{k}"] = np32(v)
        rec = Recorder()
        torch.manual_seed(5)
        with rec.capture():
            rb = rs(poses, focal, EvaluationMode.TRAINING)
        d["train_pixel_ids"] = rec.take("multinomial")[0].numpy().astype(np.int64)
        d["train_jitter_u"] = np32(rec.take("rand_like")[0])
        for k, v in rb._asdict().items():
            d[f"train_{k}"] = np32(v)
        out[f"raysampler_{tag}"] = d


def gen_mlp(out):
    for tag, arch, seed, n_rays, P in (("small", SMALL_ARCH, 1, 6, 16), ("lego", LEGO_ARCH, 7, 4, 64)):
        model, params = build_mlp(arch, seed)
        g = torch.Generator().manual_seed(2)
        o = torch.randn(2, n_rays // 2, 1, 3, generator=g) * 0.5 + torch.tensor([0.0, 0.0, 4.0])
        dvec = torch.randn(2, n_rays // 2, 1, 3, generator=g)
        dvec[..., 2] -= 1.5
        t = torch.sort(torch.rand(2, n_rays // 2, 1, P, generator=g) * 4.0 + 2.0, dim=-1)[0]
        res = model(o, dvec, t)
        sig, rgb = res["rays_densities"], res["rays_features"]
        gs = torch.randn(sig.shape, generator=g)
        gc = torch.randn(rgb.shape, generator=g)
        model.zero_grad()
        ((sig * gs).sum() + (rgb * gc).sum()).backward()
        d = dict(origins=np32(o), directions=np32(dvec), lengths=np32(t), sigma=np32(sig), rgb=np32(rgb),
                 g_sigma=np32(gs), g_rgb=np32(gc), seed=np.int64(seed), checksum=checksum(params))
        for name, p in model.named_parameters():
            gr = np32(p.grad)
            if gr.size <= 4096:
                d[f"grad:{name}"] = gr
            else:  # large weight grads: norm, sum and a fixed sample of entries
                rng = np.random.Generator(np.random.PCG64(zlib.crc32(name.encode())))
                idx = rng.choice(gr.size, size=512, replace=False)
                d[f"gradidx:{name}"] = idx.astype(np.int64)
                d[f"gradval:{name}"] = gr.reshape(-1)[idx]
                d[f"gradsum:{name}"] = np.array([gr.astype(np.float64).sum(), np.linalg.norm(gr.astype(np.float64))])
        out[f"mlp_{tag}"] = d


def gen_mlp_bf16ref(out):
    """The reference's Lego NeRFMLP on mlp_lego's inputs under torch.autocast("cpu", bfloat16) -- its own
    reduced-precision behaviour (bf16 Linear layers, fp32 elsewhere) -- with the same upstream gradients: outputs and
    parameter gradients on mlp_lego's entries. The bf16 mode's gates are bounded by this error against the fp32
    reference (tests/test_gpu_parity.py)."""
    g = np.load(HERE / "mlp_lego.npz")
    model, _ = build_mlp(LEGO_ARCH, int(g["seed"]))
    with torch.autocast("cpu", dtype=torch.bfloat16):
        res = model(torch.from_numpy(g["origins"]), torch.from_numpy(g["directions"]), torch.from_numpy(g["lengths"]))
    sig, rgb = res["rays_densities"].float(), res["rays_features"].float()
    model.zero_grad()
    ((sig * torch.from_numpy(g["g_sigma"])).sum() + (rgb * torch.from_numpy(g["g_rgb"])).sum()).backward()
    d = dict(sigma=np32(sig), rgb=np32(rgb))
    for name, p in model.named_parameters():
        gr = np32(p.grad).reshape(-1)
        if f"grad:{name}" in g.files:
            d[f"grad:{name}"] = gr.reshape(p.shape)
        else:
            d[f"gradval:{name}"] = gr[g[f"gradidx:{name}"]]
            d[f"gradsum:{name}"] = np.array([gr.astype(np.float64).sum(), np.linalg.norm(gr.astype(np.float64))])
    out["mlp_lego_bf16ref"] = d


def gen_raymarcher(out):
    g = torch.Generator().manual_seed(3)
    R, P = 37, 64
    t = torch.sort(torch.rand(R, P, generator=g) * 4.0 + 2.0, dim=-1)[0]
    dirs = torch.randn(R, 3, generator=g)
    sig = torch.randn(R, P, 1, generator=g) * 3.0
    sig[:5] -= 6.0  # mostly-empty rays
    sig[5:9, 20:30] += 40.0  # hard surfaces
    feats = torch.rand(R, P, 3, generator=g)
    bg = torch.rand(R, 3, generator=g)
    gf = torch.randn(R, 3, generator=g)
    gd = torch.randn(R, 1, generator=g)
    ga = torch.randn(R, 1, generator=g)
    cases = [
        ("blend0_bgdef", dict(blend_output=False), None, 0.0),
        ("blend1_bgray", dict(blend_output=True), bg, 0.0),
        ("blend0_noise", dict(blend_output=False), None, 0.2),
        ("cap1_min", dict(blend_output=True, capping_function="cap1", weight_function="minimum"), bg, 0.0),
        ("hardbg", dict(blend_output=False, hard_background=True), bg, 0.0),
    ]
    d = dict(lengths=np32(t), directions=np32(dirs), densities=np32(sig), features=np32(feats), bg=np32(bg),
             g_features=np32(gf), g_depths=np32(gd), g_alpha=np32(ga))
    for tag, kw, bgc, noise in cases:
        rm = EmissionAbsorptionRaymarcher(surface_thickness=1, bg_color=(0.25, 0.5, 0.75),
                                          background_density_bias=1e-6, **kw)
        s = sig.clone().requires_grad_(True)
        f = feats.clone().requires_grad_(True)
        rec = Recorder()
        torch.manual_seed(9)
        with rec.capture():
            feat, depth, alpha, w, _ = rm(s, f, {}, t, dirs, density_noise_std=noise, bg_color=bgc)
        ((feat * gf).sum() + (depth * gd).sum() + (alpha * ga).sum()).backward()
        if noise > 0:
            d[f"{tag}:noise_n"] = np32(rec.take("randn_like")[0])
        d[f"{tag}:features"] = np32(feat)
        d[f"{tag}:depths"] = np32(depth)
        d[f"{tag}:alpha"] = np32(alpha)
        d[f"{tag}:weights"] = np32(w)
        d[f"{tag}:g_densities"] = np32(s.grad)
        d[f"{tag}:g_feats"] = np32(f.grad)
    out["raymarcher"] = d


def gen_sample_pdf(out):
    g = torch.Generator().manual_seed(4)
    R, P = 29, 64
    z = torch.sort(torch.rand(R, P, generator=g) * 4.0 + 2.0, dim=-1)[0]
    w = torch.rand(R, P, generator=g) ** 4
    w[:3] = 0.0  # empty rays -> uniform pdf
    w[3:6] = 0.0
    w[3:6, 30] = 0.9  # single spike
    d = dict(z=np32(z), w=np32(w))
    bins = torch.lerp(z[..., 1:], z[..., :-1], 0.5)
    d["bins"] = np32(bins)
    d["det128"] = np32(sample_pdf(bins, w[..., 1:-1], 128, det=True))
    d["det64"] = np32(sample_pdf(bins, w[..., 1:-1], 64, det=True))
    rec = Recorder()
    with rec.capture():
        s = sample_pdf(bins, w[..., 1:-1], 128, det=False)
    d["rand128_u"] = np32(rec.take("rand")[0])
    d["rand128"] = np32(s)
    for tag, rnd in (("det", False), ("rand", True)):
        ref = RayPointRefiner(n_pts_per_ray=128, random_sampling=rnd, add_input_samples=True)
        rec = Recorder()
        with rec.capture():
            rb = ref(torch.zeros(R, 3), torch.ones(R, 3), z, torch.zeros(R, 2), w)
        if rnd:
            d["refine_rand_u"] = np32(rec.take("rand")[0])
        d[f"refine_{tag}"] = np32(rb.lengths)
    out["sample_pdf"] = d


def lego_pipeline_cfg(n_fine=128, noise=0.2, n_rays=4096, H=800, W=800, focal_img=800):
    cfg = Config.fromfile(str(REF / "configs/nerf/lego.yml"))
    p = cfg.pipeline
    p.renderer.n_pts_per_ray_fine_training = n_fine
    p.renderer.n_pts_per_ray_fine_evaluation = n_fine
    p.renderer.density_noise_std_train = noise
    p.ray_sampler.n_rays_per_image_sampled_from_mask = n_rays
    p.ray_sampler.image_height = H
    p.ray_sampler.image_width = W
    return p


def load_pipeline_weights(pipe, seeds):
    """seeds: one PCG64 seed per MLP (make_nerf_mlp_params), or the string "trained" (trained_weights.npz)."""
    params = load_trained_params() if isinstance(seeds, str) else [make_nerf_mlp_params(LEGO_ARCH, s) for s in seeds]
    for f, p in zip(pipe.implicit_functions, params):
        f._fn.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})


def seeds_field(seeds):
    return np.str_(seeds) if isinstance(seeds, str) else np.array(list(seeds))


def gen_render_eval(out):
    pcfg = lego_pipeline_cfg()
    pipe = PIPELINES.build(pcfg)
    load_pipeline_weights(pipe, (11, 12))
    pipe.eval()
    pose = torch.from_numpy(synthetic_pose(30.0, -30.0, 4.0))[None]
    focal = torch.tensor([1111.1111])
    Hs, Ws = 16, 16
    g = torch.Generator().manual_seed(6)
    img = torch.rand(1, Hs, Ws, 3, generator=g)
    with torch.no_grad():
        preds = pipe(poses=pose, focal_lengths=focal, image_rgb=img, image_height=Hs, image_width=Ws,
                     evaluation_mode=EvaluationMode.EVALUATION)
    d = dict(pose=np32(pose), focal=np32(focal), image_rgb=np32(img), H=np.int64(Hs), W=np.int64(Ws),
             seeds=np.array([11, 12]))
    for k, v in preds.items():
        if torch.is_tensor(v):
            d[k] = np32(v)
    # per-stage raw renderer outputs (both passes), through the renderer directly
    rb = pipe.ray_sampler(pose, focal, evaluation_mode=EvaluationMode.EVALUATION, image_height=Hs, image_width=Ws)
    with torch.no_grad():
        ro = pipe.renderer(*rb, bg_color=None, implicit_functions=pipe.implicit_functions,
                           evaluation_mode=EvaluationMode.EVALUATION)
    d["fine_features"], d["fine_depths"], d["fine_alpha"] = np32(ro.features), np32(ro.depths), np32(ro.alpha_masks)
    pv = ro.prev_stage
    d["coarse_features"], d["coarse_depths"], d["coarse_alpha"] = np32(pv.features), np32(pv.depths), np32(pv.alpha_masks)
    d["coarse_weights"] = np32(pv.aux["weights"])
    d["fine_weights"] = np32(ro.aux["weights"])
    out["render_eval_lego"] = d


def gen_train_step(out):
    n_rays = 48
    pcfg = lego_pipeline_cfg(n_rays=n_rays)
    pose = torch.from_numpy(synthetic_pose(-60.0, -20.0, 4.0))[None]
    focal = torch.tensor([1111.1111])
    g = torch.Generator().manual_seed(8)
    img = torch.rand(1, 800, 800, 3, generator=g)
    out["train_step_lego"] = record_train_step(pcfg, (21, 22), pose, focal, img, n_rays, torch_seed=10)


def record_train_step(pcfg, seeds, pose, focal, img, n_rays, torch_seed, min_depth=None, max_depth=None):
    """One reference training step (NeRFPipeline TRAINING forward + objective backward) with every random draw, the
    refiner's inputs / outputs, both MLPs' ReLU decisions, the losses, the rasterized MC outputs and the parameter
    gradients recorded."""
    pipe = PIPELINES.build(pcfg)
    load_pipeline_weights(pipe, seeds)
    pipe.train()
    rec = Recorder()
    # the refiner's input weights and output depths (RayPointRefiner.forward, renderers/utils.py:48-69; the fine pass
    # runs at these depths, multipass_emission_absorpsion_renderer.py:107-114): recorded through a pass-through wrapper
    refined = []
    orig_fwd = RayPointRefiner.forward

    def rec_fwd(self, origins, directions, lengths, xys, ray_weights):
        rb = orig_fwd(self, origins, directions, lengths, xys, ray_weights)
        refined.append((ray_weights.detach().clone(), rb.lengths.detach().clone()))
        return rb

    RayPointRefiner.forward = rec_fwd
    # the ReLU decisions of both MLPs (output > 0 of every ReLU module: the 8 trunk layers, nerf_mlp.py:256-260, and
    # the colour hidden layer, :72-83), per point, so a parity test can tell an fp32 tie at a kink from an error
    relu = {}
    hooks = []
    for k, f in enumerate(pipe.implicit_functions):
        mods = [(f"{k}:trunk{li}", layer[1]) for li, layer in enumerate(f._fn.xyz_encoder.mlp)]
        mods.append((f"{k}:color", f._fn.color_layer[1]))
        for key, mod in mods:
            hooks.append(mod.register_forward_hook(
                lambda m, i, o, key=key: relu.__setitem__(key, (o.detach() > 0).reshape(-1, o.shape[-1]).numpy())))
    torch.manual_seed(torch_seed)
    bounds = {} if min_depth is None else dict(min_depth=min_depth, max_depth=max_depth)
    try:
        with rec.capture():
            preds = pipe(poses=pose, focal_lengths=focal, image_rgb=img, evaluation_mode=EvaluationMode.TRAINING,
                         **bounds)
    finally:
        RayPointRefiner.forward = orig_fwd
        for h in hooks:
            h.remove()
    preds["objective"].mean().backward()
    ids = rec.take("multinomial")[0].numpy().astype(np.int64)
    assert len(refined) == 1
    d = dict(pose=np32(pose), focal=np32(focal), seeds=seeds_field(seeds), n_rays=np.int64(n_rays),
             H=np.int64(pcfg.ray_sampler.image_height), W=np.int64(pcfg.ray_sampler.image_width),
             pixel_ids=ids, gt_rgb=np32(img.reshape(1, -1, 3)[0, ids[0]]),
             jitter_u=np32(rec.take("rand_like")[0]),
             pdf_u=np32(rec.take("rand")[0]),
             coarse_weights=np32(refined[0][0]).reshape(n_rays, -1), z_fine=np32(refined[0][1]).reshape(n_rays, -1))
    noise = rec.take("randn_like")
    if noise:
        d["noise_coarse"], d["noise_fine"] = np32(noise[0]), np32(noise[1])
    if min_depth is not None:
        d["min_depth"], d["max_depth"] = np32(min_depth), np32(max_depth)
    for k in ("objective", "loss_rgb_mse", "loss_prev_stage_rgb_mse", "loss_rgb_huber"):
        d[k] = np32(preds[k])
    # the Monte-Carlo rays splatted onto full-size images (output_rasterized_mc: nerf_pipeline.py:196-201 ->
    # _rasterize_mc_samples -> scatter_rays_to_image, pipelines/utils.py:299-323), mostly zeros (compressed)
    for k in ("rendered_images", "rendered_depths", "rendered_alpha_masks"):
        d[k] = np32(preds[k])
    for k in range(len(pipe.implicit_functions)):  # bit-packed along the feature axis (np.packbits, big-endian)
        d[f"relu{k}:trunk"] = np.stack([np.packbits(relu[f"{k}:trunk{li}"], axis=-1) for li in range(8)])
        d[f"relu{k}:color"] = np.packbits(relu[f"{k}:color"], axis=-1)
    for i, f in enumerate(pipe.implicit_functions):
        for name, p in f._fn.named_parameters():
            gr = np32(p.grad)
            if gr.size <= 4096:
                d[f"grad{i}:{name}"] = gr
            else:
                d[f"gradsum{i}:{name}"] = np.array([gr.astype(np.float64).sum(), np.linalg.norm(gr.astype(np.float64))])
                rng = np.random.Generator(np.random.PCG64(len(name) * 1000 + i))
                idx = rng.choice(gr.size, size=256, replace=False)
                d[f"gradidx{i}:{name}"] = idx.astype(np.int64)
                d[f"gradval{i}:{name}"] = gr.reshape(-1)[idx]
    return d


# BASELINE configs[3]: the reference's own Fern config (fern.yml) at 64 + 64 and BASELINE's 64 + 128, with LLFF-style
# per-image depth bounds as (B, 1) tensors (llff_dataset.py items; ray_sampler.py:280-283 averages them with .item())
FERN_FOCAL, FERN_NEAR, FERN_FAR = 407.6, 1.3125, 7.25


def fern_pipeline_cfg(n_fine, n_rays=1024):
    cfg = Config.fromfile(str(REF / "configs/nerf/fern.yml"))
    p = cfg.pipeline
    p.renderer.n_pts_per_ray_fine_training = n_fine
    p.renderer.n_pts_per_ray_fine_evaluation = n_fine
    p.ray_sampler.n_rays_per_image_sampled_from_mask = n_rays
    return p


def record_eval_render(pipe, pose, focal, H, W, subset=None, **bounds):
    """The reference's two-pass EVALUATION render through its renderer, with the per-stage outputs: coarse features /
    depths / weights, the refined depths (RayPointRefiner, recorded through a pass-through wrapper) and the fine
    features / depths. subset: render only these rays (flat indices into the H x W grid) of the sampler's bundle."""
    refined = []
    orig_fwd = RayPointRefiner.forward

    def rec_fwd(self, origins, directions, lengths, xys, ray_weights):
        rb = orig_fwd(self, origins, directions, lengths, xys, ray_weights)
        refined.append(rb.lengths.detach().clone())
        return rb

    RayPointRefiner.forward = rec_fwd
    try:
        rb = pipe.ray_sampler(pose, focal, evaluation_mode=EvaluationMode.EVALUATION, image_height=H, image_width=W,
                              **bounds)
        if subset is not None:
            sel = torch.as_tensor(np.asarray(subset, np.int64))
            rb = type(rb)(*[x.reshape(x.shape[0], -1, *x.shape[3:])[:, sel] for x in rb])
        with torch.no_grad():
            ro = pipe.renderer(*rb, bg_color=None, implicit_functions=pipe.implicit_functions,
                               evaluation_mode=EvaluationMode.EVALUATION)
    finally:
        RayPointRefiner.forward = orig_fwd
    R = H * W if subset is None else len(subset)
    pv = ro.prev_stage
    return dict(lengths=np32(rb.lengths).reshape(R, -1), coarse_features=np32(pv.features).reshape(R, -1),
                coarse_depths=np32(pv.depths).reshape(R), coarse_weights=np32(pv.aux["weights"]).reshape(R, -1),
                z_fine=np32(refined[0]).reshape(R, -1), fine_features=np32(ro.features).reshape(R, -1),
                fine_depths=np32(ro.depths).reshape(R))


def gen_render_fern(out):
    from scene import forward_pose
    near, far = torch.tensor([[FERN_NEAR]]), torch.tensor([[FERN_FAR]])
    for n_fine in (64, 128):
        pipe = PIPELINES.build(fern_pipeline_cfg(n_fine))
        load_pipeline_weights(pipe, (41, 42))
        pipe.eval()
        pose = torch.from_numpy(forward_pose())[None]
        focal = torch.tensor([FERN_FOCAL])
        d = record_eval_render(pipe, pose, focal, 9, 12, min_depth=near, max_depth=far)
        d.update(pose=np32(pose), focal=np32(focal), H=np.int64(9), W=np.int64(12), seeds=np.array([41, 42]),
                 n_fine=np.int64(n_fine), min_depth=np32(near), max_depth=np32(far))
        out[f"render_fern_{n_fine}"] = d


def gen_train_step_fern(out):
    from scene import forward_pose
    near, far = torch.tensor([[FERN_NEAR]]), torch.tensor([[FERN_FAR]])
    for n_fine in (64, 128):
        n_rays = 64
        pose = torch.from_numpy(forward_pose(0.03))[None]
        focal = torch.tensor([FERN_FOCAL])
        g = torch.Generator().manual_seed(15 + n_fine)
        img = torch.rand(1, 378, 504, 3, generator=g)
        out[f"train_step_fern_{n_fine}"] = record_train_step(fern_pipeline_cfg(n_fine, n_rays), (51, 52), pose, focal,
                                                             img, n_rays, torch_seed=16 + n_fine, min_depth=near,
                                                             max_depth=far)


# ----------------------------------------------------------------------------- the HIP kernels' summation order
HIP_ORDER_INNER = 0  # how one v_mfma_f32_16x16x4_f32 combines its four products (profiles/r5_mfma_order.txt)


def _hip_order_lib():
    """tests/golden/mfma_order.c built with gcc (test infrastructure, this container only)."""
    import ctypes
    import subprocess
    so = Path("/tmp/yanerf_mfma_order.so")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", "-o", str(so), str(HERE / "mfma_order.c"), "-lm"],
                   check=True)
    lib = ctypes.CDLL(str(so))
    lib.hip_order_linear.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return lib


def _hip_linear(lib, x, w, b, bias_first):
    """y = x W^T + b in the fp32 HIP GEMMs' order (mfma_order.c): the chain over 16-wide K-blocks, 4 MFMA k-steps each."""
    K, N = w.shape[1], w.shape[0]
    x2 = np.ascontiguousarray(x.detach().reshape(-1, K).numpy(), np.float32)
    w2 = np.ascontiguousarray(w.detach().numpy(), np.float32)
    b2 = None if b is None else np.ascontiguousarray(b.detach().numpy(), np.float32)
    y = np.empty((x2.shape[0], N), np.float32)
    lib.hip_order_linear(x2.ctypes.data, x2.shape[0], K, w2.ctypes.data, N, None if b2 is None else b2.ctypes.data,
                         int(bias_first), HIP_ORDER_INNER, y.ctypes.data)
    return torch.from_numpy(y).reshape(*x.shape[:-1], N)


@contextmanager
def hip_order_model(model, lib, pe="torch"):
    """Evaluate one NeRFMLP (the reference's module) with every Linear in the HIP kernels' summation order: the trunk,
    intermediate and colour layers accumulate from the bias, the density and colour-output heads (16-row MFMA tiles)
    from zero with the bias added after (csrc/mlp.hip mlp_fwd_kernel); LinearWithRepeat is one K = 256 + 27 chain over
    [Y, dirPE] as the kernel's K = 288 colour GEMM. pe="cr": the harmonic embedding's sin / cos correctly rounded
    (float64, rounded once) instead of torch's vectorised ones (the fp32 kernels call the device libm sincosf)."""
    from yanerf.pipelines.models.utils import HarmonicEmbedding, LinearWithRepeat
    patched = []

    def lin_fwd(mod):
        head = mod.out_features <= 4
        return lambda x: _hip_linear(lib, x, mod.weight, mod.bias, not head)

    def lwr_fwd(mod):
        def f(inp):
            y, dpe = inp
            full = torch.cat([y, dpe.unsqueeze(-2).expand(*y.shape[:-1], dpe.shape[-1])], dim=-1)
            return _hip_linear(lib, full, mod.weight, mod.bias, True)
        return f

    def he_fwd(mod):
        def f(x):
            embed = (x[..., None] * mod._frequencies).view(*x.shape[:-1], -1)
            e64 = embed.double()
            sn, cs = e64.sin().float(), e64.cos().float()
            return torch.cat((sn, cs, x) if mod.append_input else (sn, cs), dim=-1)
        return f

    for mod in model.modules():
        if isinstance(mod, torch.nn.Linear):
            mod.forward = lin_fwd(mod)
        elif isinstance(mod, LinearWithRepeat):
            mod.forward = lwr_fwd(mod)
        elif isinstance(mod, HarmonicEmbedding) and pe == "cr":
            mod.forward = he_fwd(mod)
        else:
            continue
        patched.append(mod)
    try:
        yield
    finally:
        for mod in patched:
            del mod.forward


def hip_composite_weights(dens, lengths, dirs, background_opacity, density_bias):
    """The emission-absorption weights as csrc/render.hip composite_kernel computes them (fp32, contraction off, the
    capping exp correctly rounded, the running sum in double), for the reference's default options (exponential
    capping, product weights, density ReLU, surface thickness 1): renderer.py EmissionAbsorptionRaymarcher.forward."""
    f = np.float32
    sig = dens[..., 0].astype(f)
    z = lengths.astype(f)
    d = dirs.astype(f)
    dn = np.sqrt((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]).astype(f)
    delta = np.concatenate([z[..., 1:] - z[..., :-1], np.full(z.shape[:-1] + (1,), background_opacity, f)], -1)
    delta = (delta * dn[..., None]).astype(f)
    v = (delta * (np.maximum(sig, f(0)) + f(density_bias))).astype(f)
    exp_cr = lambda x: np.exp(x.astype(np.float64)).astype(f)  # noqa: E731
    capped = (f(1) - exp_cr(-v)).astype(f)
    cs = np.cumsum(v.astype(np.float64), axis=-1).astype(f)
    op = (f(1) - exp_cr(-cs)).astype(f)
    absorb = np.concatenate([np.ones(z.shape[:-1] + (1,), f), (f(1) - op[..., :-1]).astype(f)], -1)
    return (capped * absorb).astype(f)


@contextmanager
def hip_raymarcher():
    """The reference's raymarcher with its weights computed as the HIP composite kernel computes them
    (hip_composite_weights); depths and features follow from those weights as in renderer.py:218-238."""
    orig = EmissionAbsorptionRaymarcher.forward

    def fwd(self, rays_densities, rays_features, aux, ray_lengths, ray_directions, density_noise_std=0.0,
            bg_color=None):
        assert density_noise_std == 0.0 and self.surface_thickness == 1 and self.density_relu
        w = torch.from_numpy(hip_composite_weights(rays_densities.detach().numpy(), ray_lengths.detach().numpy(),
                                                   ray_directions.detach().numpy(), float(self.background_opacity),
                                                   float(self.background_density_bias)))
        depths = (w * ray_lengths)[..., None].sum(dim=-2)
        # opacity = the capped total (the last inclusive running sum)
        deltas = torch.cat((ray_lengths[..., 1:] - ray_lengths[..., :-1],
                            self.background_opacity * torch.ones_like(ray_lengths[..., :1])), dim=-1)
        deltas = deltas * ray_directions[..., None, :].norm(p=2, dim=-1)
        dens = torch.relu(rays_densities[..., 0]) + self.background_density_bias
        opacities = self._capping_function(torch.cumsum(deltas * dens, dim=-1))[..., -1:]
        if bg_color is None:
            bg_color = self._bg_color.view(*([1] * len(rays_features.shape[:-2])), -1).expand(*rays_features.shape[:-2], -1)
        features = (w[..., None] * rays_features).sum(dim=-2)
        alpha = opacities if self.blend_output else 1
        features = alpha * features + (1 - opacities) * bg_color
        return features, depths, opacities, w, aux

    EmissionAbsorptionRaymarcher.forward = fwd
    try:
        yield
    finally:
        EmissionAbsorptionRaymarcher.forward = orig


@contextmanager
def perturbed_refiner_weights(delta, rng):
    """RayPointRefiner (renderers/utils.py:48-69) fed the coarse weights moved by delta x U(-1, 1) per element (clamped
    at zero): coarse weights that differ from the reference's by the magnitude measured between an fp32 build and it."""
    orig = RayPointRefiner.forward

    def fwd(self, origins, directions, lengths, xys, ray_weights):
        u = torch.from_numpy(rng.uniform(-1.0, 1.0, size=tuple(ray_weights.shape)).astype(np.float32))
        return orig(self, origins, directions, lengths, xys, torch.clamp(ray_weights + delta * u, min=0.0))

    RayPointRefiner.forward = fwd
    try:
        yield
    finally:
        RayPointRefiner.forward = orig


STRIDED_800 = (np.arange(2048) * (800 * 800 // 2048) + 157).astype(np.int64)  # test_full_image_800_vs_oracle's rays

# measured max |coarse weight (this build) - coarse weight (reference)| on the gated renders, fp32 and fp32x3 builds,
# Lego 16 x 16, Fern 9 x 12, trained 25 x 25 (tools/dump_coarse_stage.py; profiles/r5_coarse_weight_deltas.json)
WEIGHT_DELTA = 1.8e-7


def gen_sensitivity(out):
    """How far the REFERENCE's own two-pass render moves under equally valid fp32 evaluations of its coarse stage: the
    Lego 16 x 16 evaluation render (render_eval_lego's config) and the Fern 9 x 12 renders (render_fern_*), each
    re-run (a) in float64 end to end (torch default dtype float64, the modules in double: the reference's algorithm
    without fp32 rounding), (b) with every result of torch.exp moved one ulp up or down (random signs: another correctly
    rounded exp, as in the capping function 1 - exp(-x)), (c) with every coarse parameter moved one ulp, (d) with the
    K-sums of every Linear layer split into 2 / 3 / 4 / 8 partial sums (another valid fp32 summation order). Per ray:
    the largest move of its refined depths and fine RGB over (b)-(d), and the float64 depths / RGB. sample_pdf's
    conditioning (renderers/utils.py:72-158: a pdf of ~1e-5 where the coarse weights hold no mass, at the `denom < eps`
    branch) turns such ulp-level differences of the coarse weights into moves of fine samples up to a bin width; the
    parity tests compare the set of rays whose refined depths differ between this build and the reference with the set
    of rays the reference itself moves this way (sensitive = float64 move or any (b)-(d) move above 2e-5)."""
    import torch.nn.functional as Fn
    from scene import forward_pose
    cases = [("lego", lego_pipeline_cfg(), (11, 12), torch.from_numpy(synthetic_pose(30.0, -30.0, 4.0))[None],
              torch.tensor([1111.1111]), 16, 16, {})]
    for n_fine in (64, 128):
        cases.append((f"fern_{n_fine}", fern_pipeline_cfg(n_fine), (41, 42), torch.from_numpy(forward_pose())[None],
                      torch.tensor([FERN_FOCAL]), 9, 12,
                      dict(min_depth=torch.tensor([[FERN_NEAR]]), max_depth=torch.tensor([[FERN_FAR]]))))
    cases.append(("trained", lego_pipeline_cfg(H=TRAINED_HW, W=TRAINED_HW), "trained", torch.from_numpy(TRAINED_POSE)[None],
                  torch.tensor([TRAINED_FOCAL], dtype=torch.float32), TRAINED_GRID, TRAINED_GRID, {}))
    # BASELINE configs[1]'s evaluation image at full size: the 2,048 strided rays of the 800 x 800 Lego camera that
    # tests/test_gpu_trainer.py::test_full_image_800_vs_oracle gates (base render stored with the trials)
    cases.append(("lego_800", lego_pipeline_cfg(), (11, 12), torch.from_numpy(synthetic_pose(30.0, -30.0, 4.0))[None],
                  torch.tensor([1111.1111]), 800, 800, dict(subset=STRIDED_800)))
    if os.environ.get("YANERF_SENSITIVITY_ONLY"):
        cases = [c for c in cases if c[0] == os.environ["YANERF_SENSITIVITY_ONLY"]]

    def ulp(a, rng):
        up = rng.integers(0, 2, size=a.shape).astype(bool)
        return np.where(up, np.nextafter(a, np.float32(np.inf)), np.nextafter(a, np.float32(-np.inf))).astype(np.float32)

    texp, flin = torch.exp, Fn.linear
    for name, pcfg, seeds, pose, focal, H, W, bounds in cases:
        pipe = PIPELINES.build(pcfg)
        load_pipeline_weights(pipe, seeds)
        pipe.eval()
        base = record_eval_render(pipe, pose, focal, H, W, **bounds)
        R = H * W if "subset" not in bounds else len(bounds["subset"])
        dz, drgb = np.zeros(R), np.zeros(R)

        def note(r):
            np.maximum(dz, np.abs(r["z_fine"].astype(np.float64) - base["z_fine"]).max(-1), out=dz)
            np.maximum(drgb, np.abs(r["fine_features"].astype(np.float64) - base["fine_features"]).max(-1), out=drgb)

        coarse = pipe.implicit_functions[0]._fn
        orig = {k: v.detach().clone() for k, v in coarse.state_dict().items()}
        for trial in range(8):  # (b) exp one ulp off
            rng = np.random.Generator(np.random.PCG64(1000 + trial))
            torch.exp = lambda x, *a, rng=rng, **k: torch.from_numpy(ulp(texp(x, *a, **k).numpy(), rng))
            try:
                note(record_eval_render(pipe, pose, focal, H, W, **bounds))
            finally:
                torch.exp = texp
        for trial in range(8):  # (c) coarse parameters one ulp off
            rng = np.random.Generator(np.random.PCG64(2000 + trial))
            coarse.load_state_dict({k: torch.from_numpy(ulp(v.numpy(), rng)) for k, v in orig.items()})
            note(record_eval_render(pipe, pose, focal, H, W, **bounds))
        coarse.load_state_dict(orig)
        for nsplit in (2, 3, 4, 8):  # (d) Linear K-sums in nsplit partial sums
            def lin(x, w, bias=None, nsplit=nsplit):
                cuts = np.linspace(0, w.shape[1], nsplit + 1).astype(int)
                y = None
                for a0, a1 in zip(cuts[:-1], cuts[1:]):
                    part = flin(x[..., a0:a1], w[:, a0:a1])
                    y = part if y is None else y + part
                return y if bias is None else y + bias
            Fn.linear = lin
            try:
                note(record_eval_render(pipe, pose, focal, H, W, **bounds))
            finally:
                Fn.linear = flin
        # (e) the coarse MLP in the fp32 HIP kernels' own summation order (the refined depths depend on it alone), with
        # torch's harmonic embedding and with correctly rounded sin / cos; (f) the coarse weights moved by WEIGHT_DELTA
        dz_e, dz_f = np.zeros(R), np.zeros(R)
        lib = _hip_order_lib()
        # the whole fp32 coarse stage as the HIP kernels evaluate it: correctly rounded embedding, the MFMA chain of
        # every Linear, the composite's arithmetic (its coarse weights equal this build's bit for bit: asserted in
        # test_gpu_parity.py::test_render_eval_lego, test_gpu_fern.py::test_fern_render_with_tensor_bounds_vs_reference and
        # test_gpu_trainer.py::test_trainer_render_matches_reference_render / test_full_image_800_vs_oracle); then the reference's own
        # RayPointRefiner / sample_pdf on them
        with hip_order_model(coarse, lib, pe="cr"), hip_raymarcher():
            r = record_eval_render(pipe, pose, focal, H, W, **bounds)
        hip_w = r["coarse_weights"]
        np.maximum(dz_e, np.abs(r["z_fine"].astype(np.float64) - base["z_fine"]).max(-1), out=dz_e)
        with hip_order_model(coarse, lib, pe="torch"):  # the MFMA order alone, torch's embedding and raymarcher
            r = record_eval_render(pipe, pose, focal, H, W, **bounds)
        np.maximum(dz_e, np.abs(r["z_fine"].astype(np.float64) - base["z_fine"]).max(-1), out=dz_e)
        for trial in range(8):
            rng = np.random.Generator(np.random.PCG64(3000 + trial))
            with perturbed_refiner_weights(WEIGHT_DELTA, rng):
                r = record_eval_render(pipe, pose, focal, H, W, **bounds)
            np.maximum(dz_f, np.abs(r["z_fine"].astype(np.float64) - base["z_fine"]).max(-1), out=dz_f)
        # (a) float64
        torch.set_default_dtype(torch.float64)
        pipe.double()
        try:
            r64 = record_eval_render(pipe, pose.double(), focal.double(), H, W,
                                     **{k: (v.double() if torch.is_tensor(v) else v) for k, v in bounds.items()})
        finally:
            torch.set_default_dtype(torch.float32)
            pipe.float()
        out[f"sensitivity_{name}"] = dict(
            trials=np.int64(20), max_z_move=dz.astype(np.float32), max_rgb_move=drgb.astype(np.float32),
            z_fine=base["z_fine"], fine_features=base["fine_features"], z_fine_f64=r64["z_fine"].astype(np.float64),
            fine_features_f64=r64["fine_features"].astype(np.float64), max_z_move_hip_order=dz_e.astype(np.float32),
            max_z_move_weights=dz_f.astype(np.float32), weight_delta=np.float32(WEIGHT_DELTA),
            hip_arithmetic_coarse_weights=hip_w,
            **({} if "subset" not in bounds else dict(subset=np.asarray(bounds["subset"], np.int64), pose=np32(pose),
                                                      focal=np32(focal), **{f"base_{k}": v for k, v in base.items()})))


# Parity at TRAINED weights: the Lego architecture trained 1,500 fused fp32 steps (tools/density_collapse_probe.py: seed
# 7, density-layer bias 1.0 at init, 4096 rays, 64 + 128, test PSNR 36.9 dB, profiles/r4_density_collapse_probe.jsonl)
# on the procedural scene of tools/synthetic_scene.py (100 x 100 views, camera radius 4, lego.yml's near / far),
# model tensors of its checkpoint saved as trained_weights.npz. Its density is peaked at the scene's surfaces, so
# sample_pdf is far better conditioned than at random init (the other goldens' weights). (With the reference's zero
# density bias, nerf_mlp.py:69-71, this scene's training collapses to the transparent solution for seeds 42 and 1.)
TRAINED_HW, TRAINED_GRID = 100, 25
TRAINED_POSE = synthetic_pose(45.0, -30.0, 4.0)
TRAINED_FOCAL = 0.5 * TRAINED_HW / np.tan(0.5 * 0.6911112070083618)  # synthetic_scene.CAMERA_ANGLE_X


def scene_view(theta, phi, hw):
    """The procedural scene's ground-truth RGB at one camera (tools/synthetic_scene.render_view, black background)."""
    sys.path.insert(0, str(HERE.parents[1] / "tools"))
    from synthetic_scene import pose_spherical, render_view
    return render_view(pose_spherical(theta, phi, 4.0), hw, hw)[..., :3]


def gen_render_trained(out):
    pipe = PIPELINES.build(lego_pipeline_cfg(H=TRAINED_HW, W=TRAINED_HW))
    load_pipeline_weights(pipe, "trained")
    pipe.eval()
    pose, focal = torch.from_numpy(TRAINED_POSE)[None], torch.tensor([TRAINED_FOCAL], dtype=torch.float32)
    d = record_eval_render(pipe, pose, focal, TRAINED_GRID, TRAINED_GRID)
    d.update(pose=np32(pose), focal=np32(focal), H=np.int64(TRAINED_GRID), W=np.int64(TRAINED_GRID),
             cfg_hw=np.int64(TRAINED_HW), seeds=seeds_field("trained"))
    out["render_trained"] = d


def gen_train_step_trained(out):
    n_rays = 64
    pcfg = lego_pipeline_cfg(n_rays=n_rays, H=TRAINED_HW, W=TRAINED_HW)
    pose = torch.from_numpy(synthetic_pose(-70.0, -25.0, 4.0))[None]
    focal = torch.tensor([TRAINED_FOCAL], dtype=torch.float32)
    img = torch.from_numpy(np.ascontiguousarray(scene_view(-70.0, -25.0, TRAINED_HW)))[None].float()
    out["train_step_trained"] = record_train_step(pcfg, "trained", pose, focal, img, n_rays, torch_seed=31)


@contextmanager
def replay_draws(log):
    """Feed a Recorder's draws back, in order, to the same torch calls (cast to the dtype the caller asks for: the float64
    re-run of a recorded fp32 trajectory consumes the same uniforms / normals / pixel ids)."""
    names = ("multinomial", "rand_like", "randn_like", "rand")
    orig = {n: getattr(torch, n) for n in names}
    it = iter(list(log))

    def make(name):
        def g(*a, **k):
            n_, v = next(it)
            assert n_ == name, (n_, name)
            if name in ("rand_like", "randn_like"):
                return v.to(a[0].dtype)
            if name == "rand":
                return v.to(k.get("dtype") or torch.get_default_dtype())
            return v.clone()
        return g

    for n in names:
        setattr(torch, n, make(n))
    try:
        yield
    finally:
        for n, f in orig.items():
            setattr(torch, n, f)


TRAJ_HW, TRAJ_RAYS, TRAJ_STEPS = 32, 256, 20


def _trajectory_setup():
    """gen_train_trajectory's fixed inputs: the runner config, pipeline config, focal, per-step poses / images, seeds."""
    cfg = Config.fromfile(str(REF / "configs/nerf/lego.yml"))
    pcfg = lego_pipeline_cfg(n_rays=TRAJ_RAYS, H=TRAJ_HW, W=TRAJ_HW)
    focal = torch.tensor([0.5 * TRAJ_HW / np.tan(0.5 * 0.6911112070083618)], dtype=torch.float32)
    views = [(-180.0 + 360.0 * k / TRAJ_STEPS, -30.0 + 10.0 * np.sin(k)) for k in range(TRAJ_STEPS)]
    poses = [torch.from_numpy(synthetic_pose(th, ph, 4.0))[None] for th, ph in views]
    images = [torch.from_numpy(np.ascontiguousarray(scene_view(th, ph, TRAJ_HW)))[None].float() for th, ph in views]
    return cfg.runner, pcfg, focal, poses, images, (61, 62)


def _trajectory_run(setup, dtype, draws=None, autocast=False):
    """The reference's registry pipeline trained TRAJ_STEPS steps by the reference runner's Adam and schedule (see
    gen_train_trajectory). draws: per-step Recorder logs to replay (None: draw and record). autocast: every step's
    forward under torch.autocast("cpu", bfloat16). Returns (pipeline, logs, losses [steps, 3], lrs)."""
    from yanerf.runners.utils import create_lr_scheduler, warmup_lr_scheduler
    runner, pcfg, focal, poses, images, seeds = setup
    torch.set_default_dtype(dtype)
    try:
        pipe = PIPELINES.build(pcfg)
        load_pipeline_weights(pipe, seeds)
        pipe.to(dtype)
        pipe.train()
        opt = torch.optim.Adam([{"params": pipe.parameters(), "init_lr": runner.init_lr}], lr=runner.init_lr,
                               weight_decay=runner.weight_decay)
        sched = create_lr_scheduler(opt, runner)
        torch.manual_seed(70)
        rec, logs, losses, lrs = Recorder(), [], [], []
        for it in range(TRAJ_STEPS):
            sched(iter=it)
            if runner["warmup_steps"] > 0 and it <= runner["warmup_steps"]:
                warmup_lr_scheduler(opt, it, runner["warmup_steps"], runner["warmup_lr"])
            lrs.append(opt.param_groups[0]["lr"])
            opt.zero_grad()
            kw = dict(poses=poses[it].to(dtype), focal_lengths=focal.to(dtype), image_rgb=images[it].to(dtype),
                      evaluation_mode=EvaluationMode.TRAINING)
            if draws is None:
                rec.log = []
                with rec.capture():
                    preds = pipe(**kw)
                logs.append(list(rec.log))
            elif autocast:
                with replay_draws(draws[it]), torch.autocast("cpu", dtype=torch.bfloat16):
                    preds = pipe(**kw)
            else:
                with replay_draws(draws[it]):
                    preds = pipe(**kw)
            preds["objective"].mean().backward()
            opt.step()
            losses.append([float(preds["objective"].mean()), float(preds["loss_rgb_mse"].mean()),
                           float(preds["loss_prev_stage_rgb_mse"].mean())])
        return pipe, logs, np.array(losses, np.float64), np.array(lrs, np.float64)
    finally:
        torch.set_default_dtype(torch.float32)


def _trajectory_params(d, prefix, pipe):
    """Parameters after the trajectory: whole tensors up to 4,096 elements, a fixed 256-entry sample of the others."""
    for i, f in enumerate(pipe.implicit_functions):
        for name, p in f._fn.named_parameters():
            v = p.detach().double().numpy()
            if v.size <= 4096:
                d[f"{prefix}{i}:{name}"] = v.astype(np.float32 if prefix == "param" else np.float64)
            else:
                idx = np.random.Generator(np.random.PCG64(len(name) * 1000 + i)).choice(v.size, 256, replace=False)
                if prefix == "param":
                    d[f"paramidx{i}:{name}"] = idx.astype(np.int64)
                d[f"{prefix}{i}:{name}"] = v.reshape(-1)[idx].astype(np.float32 if prefix == "param" else np.float64)


def gen_train_trajectory(out):
    """Multi-step training parity: the reference's registry pipeline (lego.yml: 64 + 128 samples, density noise 0.2) with
    the reference runner's optimizer and schedule (scripts/run.py:158-160: torch.optim.Adam over create_param_groups,
    runners/utils.py:148-151; runners/apis.py:66-89 per iteration: create_lr_scheduler's decay, warmup_lr_scheduler while
    passed_iter <= warmup_steps, zero_grad, objective.mean().backward(), optimizer.step()) for TRAJ_STEPS steps on
    TRAJ_HW x TRAJ_HW views of the procedural scene (one view per step), TRAJ_RAYS rays per step, from the seeded Lego
    weights (the reference's zero density bias). Every random draw of every step is recorded (pixel ids, stratified
    jitter, both density-noise draws, refinement uniforms), with the per-step losses and learning rates, and the
    parameters after the last step (whole tensors up to 4,096 elements, a fixed 256-entry sample of the larger ones).
    The same trajectory is then re-run by the reference in float64 on the recorded draws: the exact algorithm's
    parameters after the same steps, the yardstick both fp32 implementations are measured against."""
    setup = _trajectory_setup()
    _, _, focal, poses, images, seeds = setup
    pipe, logs, losses, lrs = _trajectory_run(setup, torch.float32)
    pipe64, _, losses64, _ = _trajectory_run(setup, torch.float64, logs)
    d = dict(seeds=np.array(seeds), n_rays=np.int64(TRAJ_RAYS), hw=np.int64(TRAJ_HW), steps=np.int64(TRAJ_STEPS),
             focal=np32(focal), poses=np.concatenate([np32(p) for p in poses]),
             images=np.concatenate([np32(i) for i in images]), losses=losses, losses_f64=losses64, lrs=lrs)
    for it, log in enumerate(logs):
        kinds = [n for n, _ in log]
        assert kinds == ["multinomial", "rand_like", "randn_like", "rand", "randn_like"], kinds
        d[f"pixel_ids:{it}"] = log[0][1].numpy().astype(np.int64)
        d[f"jitter_u:{it}"] = np32(log[1][1])
        d[f"noise_coarse:{it}"] = np32(log[2][1])
        d[f"pdf_u:{it}"] = np32(log[3][1])
        d[f"noise_fine:{it}"] = np32(log[4][1])
    _trajectory_params(d, "param", pipe)
    _trajectory_params(d, "param64_", pipe64)
    out["train_trajectory"] = d


def gen_train_trajectory_bf16ref(out):
    """The reference's own bf16 trajectory: gen_train_trajectory's 20 steps on the SAME recorded draws (read from the
    committed train_trajectory.npz), every forward under torch.autocast("cpu", bfloat16), the reference's own
    refinement of its bf16 coarse weights. Per-step losses and the parameters after the last step on the trajectory
    golden's entries: the bound of the bf16 mode's trajectory test (tests/test_gpu_trainer.py)."""
    g = np.load(HERE / "train_trajectory.npz")
    logs = []
    for it in range(TRAJ_STEPS):
        logs.append([("multinomial", torch.from_numpy(g[f"pixel_ids:{it}"])),
                     ("rand_like", torch.from_numpy(g[f"jitter_u:{it}"])),
                     ("randn_like", torch.from_numpy(g[f"noise_coarse:{it}"])),
                     ("rand", torch.from_numpy(g[f"pdf_u:{it}"])),
                     ("randn_like", torch.from_numpy(g[f"noise_fine:{it}"]))])
    pipe, _, losses, lrs = _trajectory_run(_trajectory_setup(), torch.float32, logs, autocast=True)
    assert np.array_equal(lrs, g["lrs"])
    d = dict(losses=losses)
    _trajectory_params(d, "param", pipe)
    d = {k: v for k, v in d.items() if not k.startswith("paramidx")}  # the trajectory golden's entries
    out["train_trajectory_bf16ref"] = d


def gen_zero_outputer(out):
    """Known-answer (reference tests/test_pipeline.py:67-151): zero density -> rendered == bg exactly."""
    pcfg = lego_pipeline_cfg(n_rays=4)
    pcfg.model = dict(type="ZeroOutputer")
    pcfg.renderer.blend_output = True
    pcfg.renderer.density_noise_std_train = 0.0
    pcfg.renderer.background_density_bias = 0.0  # as the reference test's renderer config
    pcfg.ray_sampler.image_height = 6
    pcfg.ray_sampler.image_width = 10
    pipe = PIPELINES.build(pcfg)
    g = torch.Generator().manual_seed(12)
    poses = torch.randn(3, 3, 4, generator=g)
    focal = torch.ones(3) * 500
    bg = torch.randn(3, 2, 4, 3, generator=g)
    preds = pipe(poses=poses, focal_lengths=focal, bg_image_rgb=bg, image_rgb=bg,
                 evaluation_mode=EvaluationMode.EVALUATION, image_width=4, image_height=2)
    assert torch.all(preds["rendered_images"] == bg), "reference known answer must hold"
    out["zero_outputer"] = dict(poses=np32(poses), focal=np32(focal), bg=np32(bg),
                                rendered_images=np32(preds["rendered_images"]), objective=np32(preds["objective"]))


def gen_init_checksums(out):
    """Seeded initialisation of the reference NeRFMLP (nerf_mlp.py:50-83, 244-261; _xavier_init :292-296)."""
    d = dict(seed=np.int64(1234))
    for tag, arch in (("lego", LEGO_ARCH), ("small", SMALL_ARCH)):
        cfg = dict(type="NeRFMLP", **arch, harmonic_functions_xyz_append_intput=True,
                   harmonic_functions_dir_append_intput=True, latent_dim=0, input_xyz=True, input_dir=True)
        torch.manual_seed(1234)
        m = MODELS.build(Config(dict(model=cfg)).model)
        names = list(m.state_dict().keys())
        d[f"{tag}_names"] = np.array(names)
        d[f"{tag}_sums"] = np.array([m.state_dict()[k].double().sum().item() for k in names])
    out["init_checksums"] = d


def gen_pipeline_state(out):
    """The reference NeRFPipeline's state_dict layout (the checkpoint format of scripts/run.py:168-175, 409-414:
    {"model": pipeline.state_dict(), ...}) for the Lego and Fern configs, and its seeded-initialisation checksums
    (torch.manual_seed(42) then PIPELINES.build, as run.py:70-73, 149)."""
    d = {}
    for tag, cfgfile in (("lego", "configs/nerf/lego.yml"), ("fern", "configs/nerf/fern.yml")):
        cfg = Config.fromfile(str(REF / cfgfile))
        torch.manual_seed(42)
        pipe = PIPELINES.build(cfg.pipeline)
        sd = pipe.state_dict()
        names = list(sd.keys())
        d[f"{tag}_names"] = np.array(names)
        d[f"{tag}_ndim"] = np.array([sd[k].dim() for k in names], np.int64)
        d[f"{tag}_shapes"] = np.array([list(sd[k].shape) + [0] * (2 - sd[k].dim()) for k in names], np.int64)
        d[f"{tag}_sums"] = np.array([sd[k].double().sum().item() for k in names])
    out["pipeline_state"] = d


@contextmanager
def pytest_raises_any():
    try:
        yield
    except (AttributeError, NameError, UnboundLocalError):
        return
    raise AssertionError("expected the reference RaySampler to fail on a mask")


def gen_raysampler_masked(out):
    """Masked / probability-weighted training ray sampling (ray_sampler.py:82-96, 178-227, 317-358) and LLFF-style
    per-image tensor depth bounds (:280-283): the multinomial weights the reference builds (captured as the inputs
    of torch.multinomial), the pixels it drew, its jitter and the resulting rays.

    The reference's RaySampler.forward cannot take a mask at all (ray_sampler.py:87-89 reads self.image_height, an
    attribute it never sets: AttributeError; with an explicit size the local is unbound), so the masked cases call its
    training _RaySampler directly with the mask resized as :90-96 intends (nearest, configured size)."""
    g = torch.Generator().manual_seed(3)
    base = dict(type="RaySampler", image_width=10, image_height=6, n_rays_per_image_sampled_from_mask=5,
                min_depth=0.5, max_depth=2.0, scene_extent=0.0, n_pts_per_ray_training=7, n_pts_per_ray_evaluation=7,
                stratified_point_sampling_training=True, stratified_point_sampling_evaluation=False)
    B, H, W = 2, 6, 10
    poses = torch.randn(B, 3, 4, generator=g)
    focal = torch.tensor([9.0, 11.5])
    mask = (torch.rand(B, 1, 3, 5, generator=g) > 0.4).float()  # nearest-resized to 6 x 10 by the sampler
    spm = torch.rand(B, H, W, generator=g) * (torch.rand(B, H, W, generator=g) > 0.3).float()
    spm4 = torch.rand(B, 2, H, W, generator=g)
    sparse = torch.zeros(B, 1, H, W)
    sparse[0, 0, 1, 2] = sparse[0, 0, 4, 7] = sparse[0, 0, 5, 9] = 1.0  # 3 pixels < 5 rays: with replacement
    sparse[1] = 1.0
    near = torch.tensor([[0.75], [1.25]])
    far = torch.tensor([[3.0], [4.5]])
    cases = {
        "mask": (dict(), dict(mask=mask)),
        "mask_prob": (dict(), dict(mask=mask, sampling_prob_mask=spm)),
        "prob_only": (dict(), dict(sampling_prob_mask=spm)),
        "mask_nrays_none": (dict(n_rays_per_image_sampled_from_mask=None), dict(mask=mask)),
        "layered": (dict(), dict(sampling_prob_mask=spm4, n_rays_per_image=[3, 4])),
        "fallback": (dict(), dict(mask=sparse)),
        "bounds": (dict(), dict(min_depth=near, max_depth=far)),
    }
    d = dict(poses=np32(poses), focal=np32(focal), mask=np32(mask), spm=np32(spm), spm4=np32(spm4), sparse=np32(sparse),
             near=np32(near), far=np32(far))
    for tag, (over, kw) in cases.items():
        rs = RAY_SAMPLERS.build(Config(dict(r=dict(base, **over))).r)
        kw = dict(kw)
        if "mask" in kw:
            with pytest_raises_any():
                rs(poses, focal, EvaluationMode.TRAINING, **kw)  # the reference's own entry point fails here
            kw["mask"] = torch.nn.functional.interpolate(kw["mask"], size=[H, W], mode="nearest")[:, 0]
            call = rs._raysamplers[EvaluationMode.TRAINING]
        else:
            call = partial(rs, evaluation_mode=EvaluationMode.TRAINING)
        calls = []
        orig = torch.multinomial

        def mn(inp, num, replacement=False, **k):
            r = orig(inp, num, replacement=replacement, **k)
            calls.append((inp.detach().clone(), bool(replacement), r.clone()))
            return r

        torch.multinomial = mn
        rec = Recorder()
        torch.manual_seed(17)
        try:
            with rec.capture():
                rb = call(poses, focal, **kw)
        finally:
            torch.multinomial = orig
        d[f"{tag}:n_calls"] = np.int64(len(calls))
        for i, (inp, repl, r) in enumerate(calls):
            d[f"{tag}:w{i}"] = np32(inp)
            d[f"{tag}:repl{i}"] = np.int64(repl)
        d[f"{tag}:jitter_u"] = np32(rec.take("rand_like")[0])
        for k, v in rb._asdict().items():
            d[f"{tag}:{k}"] = np32(v)
    out["raysampler_masked"] = d


def gen_lr_schedule(out):
    """The reference runner's per-iteration learning rate (runners/apis.py:66-68: the decay scheduler from
    runners/utils.py:89-109, then warmup_lr_scheduler while passed_iter <= warmup_steps) on a torch Adam whose group
    carries init_lr (create_param_groups, runners/utils.py:148-151), with scripts/run.py:152-156's linear scaling of
    init_lr / min_lr by the world size, for the Lego runner config and variants."""
    from yanerf.runners.utils import create_lr_scheduler, warmup_lr_scheduler
    base = Config.fromfile(str(REF / "configs/nerf/lego.yml")).runner
    its = np.unique(np.concatenate([np.arange(0, 1010), np.arange(1010, 260000, 997), [199999, 250000, 259999]]))
    d = dict(iters=its.astype(np.int64))
    variants = {
        "lego_w1": (dict(), 1),
        "lego_w8": (dict(), 8),
        "cosine_w2": (dict(lr_decay_type="cosine"), 2),
        "nowarm_w1": (dict(warmup_steps=0), 1),
        "shortwarm_cos_w1": (dict(lr_decay_type="cosine", warmup_steps=7, warmup_lr=2e-4, lr_decay_iters=50,
                                  num_iters=300), 1),
    }
    for tag, (over, world) in variants.items():
        cfg = Config(dict(runner=dict(base))).runner
        for k, v in over.items():
            cfg[k] = v
        if world > 1 and cfg.linear_scale:  # scripts/run.py:152-156
            cfg.init_lr = cfg.init_lr * world
            cfg.min_lr = cfg.min_lr * world
        p = torch.nn.Parameter(torch.zeros(1))
        opt = torch.optim.Adam([{"params": [p], "init_lr": cfg.init_lr}], lr=cfg.init_lr)
        sched = create_lr_scheduler(opt, cfg)
        lrs = []
        for it in its.tolist():
            sched(iter=it)
            if cfg["warmup_steps"] > 0 and it <= cfg["warmup_steps"]:
                warmup_lr_scheduler(opt, it, cfg["warmup_steps"], cfg["warmup_lr"])
            lrs.append(opt.param_groups[0]["lr"])
        d[f"{tag}:lr"] = np.array(lrs, np.float64)
        d[f"{tag}:world"] = np.int64(world)
        d[f"{tag}:cfg"] = np.array([f"{k}={v!r}" for k, v in over.items()])
    out["lr_schedule"] = d


ITER_RUNNER_CASES = {  # tag: (config file, runner overrides, train images, world size, batch size)
    "lego_w1": ("configs/nerf/lego.yml", {}, 100, 1, 1),
    "lego_w8": ("configs/nerf/lego.yml", {}, 100, 8, 1),
    "lego_w3": ("configs/nerf/lego.yml", {}, 100, 3, 1),
    "lego_cos_w2_b2": ("configs/nerf/lego.yml", {"lr_decay_type": "cosine"}, 100, 2, 2),
    "fern_w1": ("configs/nerf/fern.yml", {}, 17, 1, 1),
    "fern_w4": ("configs/nerf/fern.yml", {}, 17, 4, 1),
    "fern_w8": ("configs/nerf/fern.yml", {}, 17, 8, 1),
}
ITER_RUNNER_KEYS = ("num_iters", "num_iters_on_one_gpu", "num_epochs", "val_per_epoch", "save_per_epoch",
                    "lr_decay_iters", "val_per_iter", "save_per_iter")


def gen_iter_runner(out):
    """scripts/run.py:243-271 setup_iter_based_runner (the iteration -> epoch conversion that rescales every '*iters'
    key of the runner config before the scheduler is built, run.py:144), run by the reference itself on its product
    configs at several world sizes: the training DataLoader is the one create_loader builds (DistributedSampler over
    the train split, drop_last=True; runners/utils.py:112-145) over a dummy dataset of the split's size, and
    get_world_size is pinned to the world size. Then the per-iteration learning rate under the rescaled config with
    the linear world scaling (run.py:152-156), through the reference's create_lr_scheduler + warmup_lr_scheduler."""
    import importlib.util
    import logging

    from torch.utils.data import DistributedSampler

    from yanerf.runners.utils import create_loader, create_lr_scheduler, warmup_lr_scheduler
    spec = importlib.util.spec_from_file_location("ref_scripts_run", REF / "scripts" / "run.py")
    run = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(run)
    log = logging.getLogger("golden")
    its = np.unique(np.concatenate([np.arange(0, 1010), np.arange(1010, 40000, 37), np.arange(40000, 260000, 997)]))
    d = dict(iters=its.astype(np.int64), keys=np.array(ITER_RUNNER_KEYS))
    for tag, (cfgfile, over, n_train, world, bs) in ITER_RUNNER_CASES.items():
        cfg = Config.fromfile(str(REF / cfgfile))
        for k, v in over.items():
            cfg.runner[k] = v
        ds = list(range(n_train))
        sampler = DistributedSampler(ds, num_replicas=world, rank=0, shuffle=True) if world > 1 else None
        dl = create_loader(ds, sampler, batch_size=bs, num_workers=0, is_train=True)
        run.get_world_size = lambda w=world: w
        run.setup_iter_based_runner(cfg.runner, dl, log)
        d[f"{tag}:case"] = np.array([cfgfile, repr(over), str(n_train), str(world), str(bs)])
        d[f"{tag}:len_loader"] = np.int64(len(dl))
        d[f"{tag}:values"] = np.array([float(cfg.runner[k]) for k in ITER_RUNNER_KEYS], np.float64)
        r = cfg.runner
        if world > 1 and r.linear_scale:  # scripts/run.py:152-156
            r.init_lr, r.min_lr = r.init_lr * world, r.min_lr * world
        p = torch.nn.Parameter(torch.zeros(1))
        opt = torch.optim.Adam([{"params": [p], "init_lr": r.init_lr}], lr=r.init_lr)
        sched = create_lr_scheduler(opt, r)
        lrs = []
        for it in its.tolist():
            sched(iter=it)
            if r["warmup_steps"] > 0 and it <= r["warmup_steps"]:
                warmup_lr_scheduler(opt, it, r["warmup_steps"], r["warmup_lr"])
            lrs.append(opt.param_groups[0]["lr"])
        d[f"{tag}:lr"] = np.array(lrs, np.float64)
    out["iter_runner"] = d


# ----------------------------------------------------------------------------- BASELINE configs[1] at full size
FULL_RAYS = 4096  # lego.yml:77 n_rays_per_image_sampled_from_mask
FULL_TIE_REL = 2e-6  # ReLU tie candidates recorded: |pre-activation| <= FULL_TIE_REL * max |pre-activation| of the layer
FULL_SAMPLE = 256  # entries sampled per large gradient tensor (as record_train_step)


def relu_hash_coeffs(P: int, U: int) -> np.ndarray:
    """[P * U, 2] float64 integer coefficients of the per-ray ReLU-decision hash (relu_ray_hash): two independent
    sets, each in [1, 2^31). Test side: tests/test_gpu_fullsize.py builds the same arrays."""
    rng = np.random.Generator(np.random.PCG64(7000 + 1000 * P + U))
    return rng.integers(1, 2 ** 31, size=(P * U, 2), dtype=np.int64).astype(np.float64)


def relu_ray_hash(mask: np.ndarray, R: int, P: int) -> np.ndarray:
    """[R, 2] per-ray hashes of one layer's ReLU decisions mask [R * P, U]: sum over the ray's (point, unit) pairs with
    decision 1 of the pair's two coefficients. Every partial sum is an integer below 2^53, so the float64 matmul is
    exact in any summation order (the GPU test recomputes it with torch and compares for equality). One flipped
    decision changes both sums."""
    U = mask.shape[-1]
    return mask.reshape(R, P * U).astype(np.float64) @ relu_hash_coeffs(P, U)


def gen_train_step_lego_4096(out):
    """BASELINE configs[1]'s training step at its full size, through the reference: lego.yml's pipeline (4096 rays,
    64 + 128 samples, density noise 0.2, 800 x 800) on one synthetic camera, every random draw recorded (pixel ids,
    jitter, both noise draws, refinement uniforms), the coarse weights and refined depths, per-ray coarse / fine outputs,
    the objective and losses, and the parameter gradients (whole tensors up to 4,096 elements, a fixed 256-entry sample
    plus the sum / norm of the larger ones, as record_train_step). The ReLU decisions (786,432 fine points x 2,304 units)
    are too large to commit, so they are recorded as (a) two exact integer hashes per ray and layer (relu_ray_hash) and
    (b) every unit whose pre-activation lies within FULL_TIE_REL of its layer's largest, with the reference's decision
    there: a GPU test that finds the hashes of a ray different can rebuild the reference's decisions of that ray from
    its own plus these candidates, and must reproduce the hash (so the two differ only at fp32 ties).
    Then, on the same draws and the reference's refined depths:
      * the reference re-run in float64 (the exact algorithm's gradients: the EXACT_RATIO yardstick);
      * the reference under torch.autocast("cpu", bfloat16) (its own reduced-precision gradients: the bf16 gates'
        reference-derived bound);
      * the oracle under the reference's own ReLU decisions (O_ref of parity_gates.tie_budget_gate, in 512-ray chunks
        whose gradients add up) with each element's sum of |terms|, pinned here to the reference's gradients."""
    out["train_step_lego_4096"] = _full_step(128, (81, 82), (15.0, -35.0), 18, 19, relu_oracle=True)


def gen_train_step_lego256_4096(out):
    """BASELINE configs[4]'s training step (Lego, 64 + 256 samples: 320 fine points per ray, 1.31 M fine points) at its
    full 4096 rays through the reference, as gen_train_step_lego_4096 without the ReLU record and the oracle: the draws,
    depths, per-ray outputs, objective and gradients, and the float64 and bf16-autocast re-runs on the same draws and
    depths. The bf16 mode's weight gradients then run two rounds of splits (yanerf_mlp_dw_plan: 36 splits)."""
    out["train_step_lego256_4096"] = _full_step(256, (91, 92), (-40.0, -25.0), 28, 29, relu_oracle=False)


FERN_FULL_RAYS = 1024  # fern.yml's n_rays_per_image_sampled_from_mask (BASELINE configs[3])


def gen_train_step_fern_1024(out):
    """BASELINE configs[3]'s training step (Fern 504 x 378, 64 + 128 samples, per-image (1, 1) depth bounds, no density
    noise) at its full 1024 rays through the reference, as gen_train_step_lego256_4096: the draws (pixel ids, jitter,
    refinement uniforms), depths, per-ray outputs, objective and gradients, and the float64 and bf16-autocast re-runs on
    the same draws and depths."""
    out["train_step_fern_1024"] = _full_step(128, (53, 54), (0.05,), 37, 38, relu_oracle=False, scene="fern")


def _full_step(n_fine, seeds, view, img_seed, torch_seed, relu_oracle, scene="lego"):
    sys.path.insert(0, str(HERE.parents[1]))
    from oracle import nerf_oracle as O
    if scene == "lego":
        R, H, W = FULL_RAYS, 800, 800
        pcfg = lego_pipeline_cfg(n_fine=n_fine)
        pose = torch.from_numpy(synthetic_pose(view[0], view[1], 4.0))[None]
        focal = torch.tensor([1111.1111])
        bounds = {}
        draw_kinds = ["multinomial", "rand_like", "randn_like", "rand", "randn_like"]
    else:
        from scene import forward_pose
        R, H, W = FERN_FULL_RAYS, 378, 504
        pcfg = fern_pipeline_cfg(n_fine, R)
        pose = torch.from_numpy(forward_pose(view[0]))[None]
        focal = torch.tensor([FERN_FOCAL])
        bounds = dict(min_depth=torch.tensor([[FERN_NEAR]]), max_depth=torch.tensor([[FERN_FAR]]))
        draw_kinds = ["multinomial", "rand_like", "rand"]  # fern.yml: no density noise
    tag = f"train_step_{scene}_{R}"
    assert int(pcfg.ray_sampler.n_rays_per_image_sampled_from_mask) == R
    img = torch.rand(1, H, W, 3, generator=torch.Generator().manual_seed(img_seed))
    Pc, Pf = 64, 64 + n_fine

    def build(dtype=torch.float32):
        pipe = PIPELINES.build(pcfg)
        load_pipeline_weights(pipe, seeds)
        pipe.to(dtype)
        pipe.train()
        return pipe

    # ---- the fp32 step, every draw and the ReLU pre-activations recorded
    pipe = build()
    rec = Recorder()
    refined = []
    orig_ref = RayPointRefiner.forward

    def rec_fwd(self, origins, directions, lengths, xys, ray_weights):
        rb = orig_ref(self, origins, directions, lengths, xys, ray_weights)
        refined.append((ray_weights.detach().clone(), rb.lengths.detach().clone()))
        return rb

    masks, cands, hashes, stage_out = {}, {}, {}, []
    hooks = [pipe.renderer.register_forward_hook(lambda m, i, o: stage_out.append(o))]
    for k, f in enumerate(pipe.implicit_functions if relu_oracle else []):
        mods = [(li, layer[1]) for li, layer in enumerate(f._fn.xyz_encoder.mlp)] + [(8, f._fn.color_layer[1])]
        for li, mod in mods:
            def hook(m, inp, k=k, li=li):  # a PRE-hook: the reference's ReLUs are in place
                pre = inp[0].detach().reshape(-1, inp[0].shape[-1]).numpy().copy()
                P = Pc if k == 0 else Pf
                mk = pre > 0
                masks[(k, li)] = mk
                hashes[(k, li)] = relu_ray_hash(mk, R, P)
                a = np.abs(pre)
                idx = np.flatnonzero(a <= FULL_TIE_REL * a.max())
                cands[(k, li)] = (idx.astype(np.int64), mk.reshape(-1)[idx], (a.reshape(-1)[idx] / a.max()).astype(
                    np.float32))
            hooks.append(mod.register_forward_pre_hook(hook))
    RayPointRefiner.forward = rec_fwd
    torch.manual_seed(torch_seed)
    try:
        with rec.capture():
            preds = pipe(poses=pose, focal_lengths=focal, image_rgb=img, evaluation_mode=EvaluationMode.TRAINING,
                         **bounds)
    finally:
        RayPointRefiner.forward = orig_ref
        for h in hooks:
            h.remove()
    preds["objective"].mean().backward()
    kinds = [n for n, _ in rec.log]
    assert kinds == draw_kinds, kinds
    ids = rec.log[0][1].numpy().astype(np.int64)
    z_fine = np32(refined[0][1]).reshape(R, Pf)
    fine_o, coarse_o = stage_out[-1], stage_out[-1].prev_stage
    drawn = dict(jitter_u=np32(rec.log[1][1]), pdf_u=np32(rec.log[kinds.index("rand")][1]))
    if "randn_like" in kinds:
        drawn.update(noise_coarse=np32(rec.log[2][1]), noise_fine=np32(rec.log[4][1]))
    d = dict(pose=np32(pose), focal=np32(focal), seeds=np.array(seeds), n_rays=np.int64(R), H=np.int64(H),
             W=np.int64(W), pixel_ids=ids, gt_rgb=np32(img.reshape(1, -1, 3)[0, ids[0]]),
             **{k: np32(v) for k, v in bounds.items()}, **drawn,
             coarse_weights=np32(refined[0][0]).reshape(R, Pc), z_fine=z_fine,
             coarse_features=np32(coarse_o.features).reshape(R, 3), coarse_depths=np32(coarse_o.depths).reshape(R),
             fine_features=np32(fine_o.features).reshape(R, 3), fine_depths=np32(fine_o.depths).reshape(R),
             **({"tie_rel": np.float32(FULL_TIE_REL)} if relu_oracle else {}))
    for kk in ("objective", "loss_rgb_mse", "loss_prev_stage_rgb_mse"):
        d[kk] = np32(preds[kk])
    for (k, li), hsh in hashes.items():
        d[f"relu_hash{k}:{li}"] = hsh
        idx, dec, rel = cands[(k, li)]
        d[f"relu_cand_idx{k}:{li}"], d[f"relu_cand_dec{k}:{li}"], d[f"relu_cand_rel{k}:{li}"] = idx, dec, rel

    def sample_of(i, name, n):
        return np.random.Generator(np.random.PCG64(len(name) * 1000 + i)).choice(n, size=FULL_SAMPLE, replace=False)

    def put_grads(prefix, model_list):
        for i, f in enumerate(model_list):
            for name, p in f._fn.named_parameters():
                gr = p.grad.detach().double().numpy().reshape(-1)
                if gr.size <= 4096:
                    d[f"{prefix}{i}:{name}"] = gr.astype(np.float64 if prefix == "grad64_" else np.float32)
                else:
                    sel = sample_of(i, name, gr.size)
                    d[f"{prefix}idx{i}:{name}"] = sel.astype(np.int64)
                    d[f"{prefix}val{i}:{name}"] = gr[sel].astype(np.float64 if prefix == "grad64_" else np.float32)
                    d[f"{prefix}sum{i}:{name}"] = np.array([gr.sum(), np.linalg.norm(gr)])

    put_grads("grad", pipe.implicit_functions)  # grad / gradidx / gradval / gradsum: the golden_grad_items layout
    log = list(rec.log)
    del pipe, preds, stage_out, fine_o, coarse_o
    print(f"{tag}: fp32 step recorded", flush=True)

    def rerun(dtype, autocast=False):
        """The same step on the recorded draws, the refined depths replaced by the fp32 reference's."""
        torch.set_default_dtype(dtype)
        try:
            p2 = build(dtype)
            zf = torch.from_numpy(z_fine).to(dtype)

            def fixed(self, origins, directions, lengths, xys, ray_weights):
                rb = orig_ref(self, origins, directions, lengths, xys, ray_weights)  # consumes the pdf_u draw
                return rb._replace(lengths=zf.reshape(rb.lengths.shape))

            RayPointRefiner.forward = fixed
            try:
                bd = {k: v.to(dtype) for k, v in bounds.items()}
                with replay_draws(log):
                    if autocast:
                        with torch.autocast("cpu", dtype=torch.bfloat16):
                            pr = p2(poses=pose.to(dtype), focal_lengths=focal.to(dtype), image_rgb=img.to(dtype),
                                    evaluation_mode=EvaluationMode.TRAINING, **bd)
                    else:
                        pr = p2(poses=pose.to(dtype), focal_lengths=focal.to(dtype), image_rgb=img.to(dtype),
                                evaluation_mode=EvaluationMode.TRAINING, **bd)
            finally:
                RayPointRefiner.forward = orig_ref
            pr["objective"].mean().backward()
            return p2, float(pr["objective"].mean())
        finally:
            torch.set_default_dtype(torch.float32)

    p64, obj64 = rerun(torch.float64)
    put_grads("grad64_", p64.implicit_functions)
    d["objective_f64"] = np.float64(obj64)
    del p64
    print(f"{tag}: float64 re-run", flush=True)
    pbf, objbf = rerun(torch.float32, autocast=True)
    put_grads("grad_bf16ac", pbf.implicit_functions)
    d["objective_bf16ac"] = np.float64(objbf)
    del pbf
    print(f"{tag}: bf16 autocast re-run", flush=True)

    if not relu_oracle:
        return d
    # ---- the oracle under the reference's own ReLU decisions at its depths (O_ref), in 512-ray chunks
    arch = O.MLPArch.from_dict(LEGO_ARCH)
    pc, pf = make_nerf_mlp_params(LEGO_ARCH, seeds[0]), make_nerf_mlp_params(LEGO_ARCH, seeds[1])
    cfg = O.RenderCfg(n_pts_fine=n_fine, density_noise_std=0.2, raymarch=O.RaymarchOpts(background_density_bias=1e-6))
    o, dd, z, _ = O.sample_rays_train(d["pose"], d["focal"], 800, 800, 2.0, 6.0, Pc, ids, d["jitter_u"])
    o, dd, z = o.reshape(R, 3), dd.reshape(R, 3), z.reshape(R, Pc)
    nc = (d["noise_coarse"].reshape(R, Pc) * np.float32(0.2)).astype(np.float32)
    nf = (d["noise_fine"].reshape(R, Pf) * np.float32(0.2)).astype(np.float32)
    acc = {}
    C = 512
    for r0 in range(0, R, C):
        sl = slice(r0, r0 + C)

        def mk(k, P):
            rows = slice(r0 * P, (r0 + C) * P)
            return dict(trunk=[masks[(k, li)][rows] for li in range(8)], color=masks[(k, 8)][rows])

        res = O.train_step_grads(pc, pf, arch, cfg, o[sl], dd[sl], z[sl], d["gt_rgb"][sl], nc[sl], nf[sl],
                                 d["pdf_u"].reshape(R, -1)[sl], z_fine=z_fine[sl], relu_masks=(mk(0, Pc), mk(1, Pf)),
                                 abs_terms=True, loss_rays=R)
        for key in ("grads_coarse", "grads_fine", "abs_coarse", "abs_fine"):
            for name, v in res[key].items():
                a = np.asarray(v, np.float64)
                acc[(key, name)] = a if (key, name) not in acc else acc[(key, name)] + a
        print(f"train_step_lego_4096: oracle rays {r0}..{r0 + C}", flush=True)
    pin = 0.0
    for i, key in ((0, "coarse"), (1, "fine")):
        for name in pc:
            g_or, ab = acc[(f"grads_{key}", name)].reshape(-1), acc[(f"abs_{key}", name)].reshape(-1)
            if f"grad{i}:{name}" in d:
                ref, sel = d[f"grad{i}:{name}"].astype(np.float64), slice(None)
            else:
                ref, sel = d[f"gradval{i}:{name}"].astype(np.float64), d[f"gradidx{i}:{name}"]
            d[f"oref{i}:{name}"], d[f"oabs{i}:{name}"] = g_or[sel].astype(np.float64), ab[sel].astype(np.float64)
            err = np.abs(g_or[sel] - ref)
            M = max(np.abs(ref).max(), 1e-30)
            assert (err <= 2e-5 * M + 2e-5 * ab[sel]).all(), (i, name, float(err.max() / M))
            pin = max(pin, float(err.max() / M))
    d["oracle_pin_max"] = np.float64(pin)
    print(f"train_step_lego_4096: oracle pinned to the reference at {pin:.3e} x max", flush=True)
    return d


GENERATORS = (gen_harmonic, gen_raysampler, gen_mlp, gen_raymarcher, gen_sample_pdf, gen_render_eval,
              gen_train_step, gen_zero_outputer, gen_init_checksums, gen_pipeline_state, gen_lr_schedule,
              gen_raysampler_masked, gen_iter_runner, gen_render_fern, gen_train_step_fern, gen_sensitivity,
              gen_render_trained, gen_train_step_trained, gen_train_trajectory, gen_train_step_lego_4096,
              gen_mlp_bf16ref, gen_train_trajectory_bf16ref, gen_train_step_lego256_4096, gen_train_step_fern_1024)


def main():
    """`make_golden.py [name ...]` regenerates only the named generators (e.g. gen_pipeline_state)."""
    out = {}
    want = set(sys.argv[1:])
    for f in GENERATORS:
        if want and f.__name__ not in want:
            continue
        f(out)
        print("generated", f.__name__)
    for name, d in out.items():
        path = HERE / f"{name}.npz"
        np.savez_compressed(path, **d)
        print(f"{path.name}: {path.stat().st_size / 1024:.1f} KiB")


if __name__ == "__main__":
    main()
