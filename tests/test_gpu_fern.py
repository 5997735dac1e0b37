"""BASELINE configs[3] (Fern / LLFF, forward-facing) on the HIP path, and masked / probability-weighted training
sampling.

* The Fern product config (504 x 378, 64 + 64 samples) and BASELINE's 64 + 128 variant with LLFF-style PER-IMAGE
  tensor depth bounds (llff_dataset.py:139-155 items; ray_sampler.py:280-283 averages them): the registry pipeline's
  two-pass evaluation render and the fused training step (NeRFTrainer.step(near=tensor, far=tensor), injected draws)
  against the CPU oracle -- objective and every parameter gradient of both MLPs.
* Masked / sampling_prob_mask training rays (ray_sampler.py:82-96, 178-227, 317-358) against golden vectors from the
  reference's _RaySampler (tests/golden/raysampler_masked.npz), and the sampling semantics on the device.

There is no NDC ray parameterisation in the reference: "Fern NDC" runs the reference's own Fern config.
"""
import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O
from parity_gates import (STRICT_GRAD, TIE_REL, grad_err, hip_relu_masks, loose_grad_gate, oracle_fine_at, relu_ties,
                          split_gate, write_report)
from weights import LEGO_ARCH, make_nerf_mlp_params

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
FOCAL = 407.6
NEAR, FAR = 1.3125, 7.25  # per-image LLFF-style bounds (bd_factor-rescaled scale)


def t(x, dtype=torch.float32):
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=DEV)


def n(x):
    return x.detach().float().cpu().numpy()


def fern_cfg(n_fine):
    import yanerf_boot
    from yanerf_amd.utils.config import Config
    cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/fern.yml"))
    cfg.pipeline.renderer.n_pts_per_ray_fine_training = n_fine
    cfg.pipeline.renderer.n_pts_per_ray_fine_evaluation = n_fine
    return cfg


def forward_pose(shift=0.0):
    pose = np.eye(4, dtype=np.float32)[:3].copy()  # forward-facing camera looking down -z... (LLFF convention)
    pose[:, 3] = [0.1 + shift, -0.05, 4.0]
    return pose


@pytest.mark.parametrize("n_fine", [64, 128])
def test_fern_render_with_tensor_bounds_vs_oracle(n_fine):
    from yanerf_amd.pipelines import PIPELINES
    from yanerf_amd.pipelines.utils import EvaluationMode
    cfg = fern_cfg(n_fine).pipeline
    pipe = PIPELINES.build(cfg).to(DEV)
    params = [make_nerf_mlp_params(LEGO_ARCH, s) for s in (41, 42)]
    for f, p in zip(pipe.implicit_functions, params):
        f._fn.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
    pipe.eval()
    pose = forward_pose()
    H, W = 9, 12
    # depths here reach FAR = 7.25 (Lego: 6): the depth gate is 1.5e-4 (2e-5 of the far bound, Lego's relative gate)
    near_t, far_t = torch.tensor([[NEAR]], device=DEV), torch.tensor([[FAR]], device=DEV)
    with torch.no_grad():
        rb = pipe.ray_sampler(t(pose[None]), t([FOCAL]), evaluation_mode=EvaluationMode.EVALUATION, image_height=H,
                              image_width=W, min_depth=near_t, max_depth=far_t)
        ro = pipe.renderer(*rb, bg_color=None, implicit_functions=pipe.implicit_functions,
                           evaluation_mode=EvaluationMode.EVALUATION)
    o, d, z, _ = O.sample_rays_eval(pose[None], np.array([FOCAL], np.float32), 504, 378, NEAR, FAR, 64, H=H, W=W)
    np.testing.assert_allclose(n(rb.lengths).reshape(-1), z.reshape(-1), atol=1e-6, rtol=1e-7)
    R = H * W
    ref = O.render_two_pass(params[0], params[1], O.MLPArch.from_dict(LEGO_ARCH),
                            O.RenderCfg(n_pts_fine=n_fine, raymarch=O.RaymarchOpts(background_density_bias=1e-6)),
                            o.reshape(R, 3), d.reshape(R, 3), z.reshape(R, 64))
    np.testing.assert_allclose(n(ro.prev_stage.features).reshape(R, 3), ref["coarse"][0], atol=1e-5, rtol=0)
    np.testing.assert_allclose(n(ro.prev_stage.depths).reshape(R), ref["coarse"][1].reshape(R), atol=1e-4, rtol=0)
    from yanerf_amd import ops
    z_gpu = n(ops.refine(rb.lengths.reshape(R, 64), ro.prev_stage.aux["weights"].reshape(R, 64), n_fine, det=True))
    fine_at = oracle_fine_at(O, params[1], O.MLPArch.from_dict(LEGO_ARCH), o, d,
                             O.RaymarchOpts(background_density_bias=1e-6))
    split_gate(n(ro.features).reshape(R, 3), ref["fine"][0], z_gpu, ref["z_fine"], n(ro.depths).reshape(R),
               ref["fine"][1].reshape(R), fine_at=fine_at, strict_depth=1.5e-4, tag=f"fern 64+{n_fine}",
               coarse=(O, n(rb.lengths), n(ro.prev_stage.aux["weights"]), n_fine))
    assert np.abs(ref["fine"][0]).max() > 1e-3


@pytest.mark.parametrize("depths", ["reference", "own"])
@pytest.mark.parametrize("n_fine", [64, 128])
@pytest.mark.parametrize("precision", ["fp32", "fp32x3"])
def test_fern_trainer_step_vs_oracle(precision, n_fine, depths):
    """The fused training step on the Fern config with per-image tensor bounds and injected draws, against the oracle's
    training step (objective = mse(fine) + mse(coarse), gradients of both MLPs; no density noise in fern.yml).
    The coarse MLP's gradients are strict (1e-4 * max) always; with depths="reference" the oracle's refined depths are
    injected and the fine MLP's gradients are strict too; with depths="own" our refined depths must be the oracle's
    refinement of our coarse weights (<= 2e-5) and the fine gradients keep the end-to-end statistical gate."""
    from yanerf_amd import ops
    from yanerf_amd.train import NeRFTrainer
    cfg = fern_cfg(n_fine)
    R, Pc = 64, 64
    tr = NeRFTrainer(cfg.pipeline, precision=precision, device=DEV, n_rays=R, runner_cfg=cfg.runner)
    seeds = (51, 52)
    sd = {}
    for i, s in enumerate(seeds):
        for k, v in make_nerf_mlp_params(LEGO_ARCH, s).items():
            sd[f"implicit_functions.{i}._fn.{k}"] = torch.from_numpy(v)
    tr.load_pipeline_state_dict(sd)
    rng = np.random.default_rng(5)
    H, W = 378, 504
    ids = rng.choice(H * W, R, replace=False).astype(np.int64)[None]
    ju = rng.random((1, R, Pc)).astype(np.float32)
    pu = rng.random((R, n_fine)).astype(np.float32)
    img = rng.random((1, H, W, 3)).astype(np.float32)
    pose = forward_pose(0.03)
    o, d, z, xy = O.sample_rays_train(pose[None], np.array([FOCAL], np.float32), W, H, NEAR, FAR, Pc, ids, ju)
    gt = img.reshape(-1, 3)[ids[0]]
    pc, pf = (make_nerf_mlp_params(LEGO_ARCH, s) for s in seeds)
    rcfg = O.RenderCfg(n_pts_fine=n_fine, near=NEAR, far=FAR, raymarch=O.RaymarchOpts(background_density_bias=1e-6))
    ref = O.train_step_grads(pc, pf, O.MLPArch.from_dict(LEGO_ARCH), rcfg, o.reshape(R, 3), d.reshape(R, 3),
                             z.reshape(R, Pc), gt, None, None, pu)
    draws = dict(pixel_ids=t(ids, torch.int64), jitter_u=t(ju), pdf_u=t(pu))
    if depths == "reference":
        draws["z_fine"] = t(ref["render"]["z_fine"])
    with ops.injected_randomness(**draws):
        out = tr.step(t(pose[None]), t([FOCAL]), t(img), near=torch.tensor([NEAR], device=DEV),
                      far=torch.tensor([FAR], device=DEV))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(n(tr.xys), xy.reshape(R, 2))
    obj = float((out["sq_fine"].sum() + out["sq_coarse"].sum()) / (R * 3))
    np.testing.assert_allclose(obj, ref["objective"], rtol=1e-5, atol=1e-7)
    report = dict(precision=precision, depths=depths, n_fine=n_fine,
                  coarse_weights_max_err=float(np.abs(n(tr.passes[0].w) - ref["render"]["coarse"][3]).max()),
                  rays_with_other_depths=int((np.abs(n(tr.zf) - ref["render"]["z_fine"]).max(-1) > 2e-5).sum()))
    assert report["coarse_weights_max_err"] <= 1e-5, report
    if depths == "own":
        z_or = O.refine(n(tr.zc), n(tr.passes[0].w), n_fine, random_sampling=True, u=pu)
        report["max_depth_err_vs_oracle_refine_of_our_weights"] = float(np.abs(n(tr.zf) - z_or).max())
        assert report["max_depth_err_vs_oracle_refine_of_our_weights"] <= 2e-5, report
    # strict, every element: the oracle at OUR refined depths under the ReLU decisions the HIP forward took; those
    # decisions equal the oracle's own signs except at fp32 ties (parity_gates.relu_ties)
    masks = [hip_relu_masks(tr.passes[k].saved, R * tr.passes[k].P) for k in range(2)]
    ora = O.train_step_grads(pc, pf, O.MLPArch.from_dict(LEGO_ARCH), rcfg, o.reshape(R, 3), d.reshape(R, 3),
                             z.reshape(R, Pc), gt, None, None, pu, z_fine=n(tr.zf), relu_masks=tuple(masks))
    worst = {0: 0.0, 1: 0.0}
    for i, (m, grads) in enumerate(((tr.models[0], ora["grads_coarse"]), (tr.models[1], ora["grads_fine"]))):
        for name, p in m.named_parameters():
            e = grad_err(n(p.grad), np.asarray(grads[name]).reshape(tuple(p.shape)))
            worst[i] = max(worst[i], e)
            assert e <= STRICT_GRAD, (i, name, e)
    ties = [relu_ties(masks[k], dict(trunk=[zz > 0 for zz in c.layer_pre], color=c.c0_pre > 0), c)
            for k, c in ((0, ora["render"]["cache_c"]), (1, ora["render"]["cache_f"]))]
    assert max(tt[1] for tt in ties) <= TIE_REL, ties
    # the direct comparison with the oracle's unmasked step at its own depths (end-to-end gate, reported)
    loose = 0.0
    for i, (m, grads) in enumerate(((tr.models[0], ref["grads_coarse"]), (tr.models[1], ref["grads_fine"]))):
        for name, p in m.named_parameters():
            loose = max(loose, loose_grad_gate(n(p.grad), np.asarray(grads[name]).reshape(tuple(p.shape)), name))
    report.update(coarse_grad_max_rel_err_vs_oracle_same_relu=worst[0],
                  fine_grad_max_rel_err_vs_oracle_same_relu=worst[1], relu_ties_coarse=ties[0][0],
                  relu_ties_fine=ties[1][0], relu_tie_max_rel_preact=max(ties[0][1], ties[1][1]),
                  grad_worst_rel_l2_vs_oracle_end_to_end=loose)
    print(f"fern trainer step vs oracle: {report}")
    write_report("train_step", f"fern 64+{n_fine} {precision} depths={depths}", report)
    assert loose < 2e-2


# ------------------------------------------------------------------------------------------- masked sampling
CASES = ["mask", "mask_prob", "prob_only", "mask_nrays_none", "layered", "fallback", "bounds"]


def _masked_sampler(tag):
    from yanerf_amd.pipelines.ray_samplers import RAY_SAMPLERS
    cfg = dict(type="RaySampler", image_width=10, image_height=6, n_rays_per_image_sampled_from_mask=5,
               min_depth=0.5, max_depth=2.0, scene_extent=0.0, n_pts_per_ray_training=7, n_pts_per_ray_evaluation=7,
               stratified_point_sampling_training=True, stratified_point_sampling_evaluation=False)
    if tag == "mask_nrays_none":
        cfg["n_rays_per_image_sampled_from_mask"] = None
    return RAY_SAMPLERS.build(cfg).to(DEV)


def _case_kwargs(g, tag):
    return {"mask": dict(mask=t(g["mask"])), "mask_prob": dict(mask=t(g["mask"]), sampling_prob_mask=t(g["spm"])),
            "prob_only": dict(sampling_prob_mask=t(g["spm"])), "mask_nrays_none": dict(mask=t(g["mask"])),
            "layered": dict(sampling_prob_mask=t(g["spm4"]), n_rays_per_image=[3, 4]),
            "fallback": dict(mask=t(g["sparse"])),
            "bounds": dict(min_depth=t(g["near"]), max_depth=t(g["far"]))}[tag]


@pytest.mark.parametrize("tag", CASES)
def test_masked_sampling_vs_reference(golden, tag):
    """Injected pixel draws (the reference's multinomial result) through our RaySampler with the raw mask: the rays
    equal the reference's (xys exact, directions / depths <= 1e-6)."""
    from yanerf_amd import ops
    from yanerf_amd.pipelines.utils import EvaluationMode
    g = golden("raysampler_masked")
    rs = _masked_sampler(tag)
    xy = g[f"{tag}:xys"]
    ids = (xy[..., 0] + 10 * xy[..., 1]).reshape(2, -1).astype(np.int64)
    with ops.injected_randomness(pixel_ids=t(ids, torch.int64), jitter_u=t(g[f"{tag}:jitter_u"])):
        rb = rs(t(g["poses"]), t(g["focal"]), EvaluationMode.TRAINING, **_case_kwargs(g, tag))
    np.testing.assert_array_equal(n(rb.xys).reshape(xy.shape), xy)
    np.testing.assert_allclose(n(rb.directions).reshape(-1), g[f"{tag}:directions"].reshape(-1), atol=1e-6, rtol=1e-6)
    np.testing.assert_allclose(n(rb.lengths).reshape(-1), g[f"{tag}:lengths"].reshape(-1), atol=1e-6, rtol=1e-6)
    np.testing.assert_array_equal(n(rb.origins).reshape(-1), g[f"{tag}:origins"].reshape(-1))


@pytest.mark.parametrize("tag", ["mask", "mask_prob", "prob_only", "mask_nrays_none", "layered", "fallback"])
def test_masked_sampling_semantics_on_device(golden, tag):
    """Without injection (torch.multinomial on the device): every drawn pixel has a positive weight, the count is the
    reference's, and draws are distinct wherever a row has enough positive weights (_safe_multinomial)."""
    from yanerf_amd.pipelines.ray_samplers.ray_sampler import RaySampler
    from yanerf_amd.pipelines.utils import EvaluationMode
    g = golden("raysampler_masked")
    rs = _masked_sampler(tag)
    kw = _case_kwargs(g, tag)
    torch.manual_seed(0)
    rb = rs(t(g["poses"]), t(g["focal"]), EvaluationMode.TRAINING, **kw)
    xy = n(rb.xys).reshape(2, -1, 2)
    assert xy.shape == g[f"{tag}:xys"].reshape(2, -1, 2).shape
    mask = kw.get("mask")
    if mask is not None:
        mask = torch.nn.functional.interpolate(mask, size=[6, 10], mode="nearest")[:, 0]
    num = [3, 4] if tag == "layered" else 5
    if tag == "mask_nrays_none":
        num = int(mask.sum(dim=(1, 2)).min().item())
    w, num = RaySampler._sampling_weights(2, 6, 10, num, mask, kw.get("sampling_prob_mask"), DEV)
    w = n(w)
    ids = (xy[..., 0] + 10 * xy[..., 1]).astype(np.int64)
    for b in range(2):
        if w.ndim == 3:
            off = 0
            for layer, k in enumerate(num):
                sel = ids[b, off:off + k]
                assert (w[b, layer, sel] > 0).all()
                assert len(set(sel.tolist())) == k
                off += k
        else:
            assert (w[b, ids[b]] > 0).all()
            if (w[b] > 0).sum() >= ids.shape[1]:
                assert len(set(ids[b].tolist())) == ids.shape[1]


def test_llff_step_with_device_bounds_is_sync_free():
    """NeRFTrainer.step fed LLFF's per-image bounds as DEVICE tensors (what DeviceImageSet holds) never synchronises
    with the host: the bounds are averaged on the device and read by the raygen kernel (the reference reads them with
    .item(), ray_sampler.py:280-283). Checked under torch.cuda.set_sync_debug_mode("error"); the step's rays equal
    those of a trainer given the same bounds as floats, bit for bit."""
    from yanerf_amd.train import NeRFTrainer
    cfg = fern_cfg(64)
    trs = [NeRFTrainer(cfg.pipeline, precision="fp32", device=DEV, n_rays=256, runner_cfg=cfg.runner, seed=9)
           for _ in range(2)]
    img = torch.rand(1, 378, 504, 3, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
    pose, focal = t(forward_pose(0.02)[None]), t([FOCAL])
    near, far = torch.tensor([[NEAR]], device=DEV), torch.tensor([[FAR]], device=DEV)
    trs[0].step(pose, focal, img, near=near, far=far)  # first call: allocator / library warm-up
    trs[1].step(pose, focal, img, near=NEAR, far=FAR)
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        for _ in range(2):
            trs[0].step(pose, focal, img, near=near, far=far)
    finally:
        torch.cuda.set_sync_debug_mode(0)
    for _ in range(2):
        trs[1].step(pose, focal, img, near=NEAR, far=FAR)
    torch.cuda.synchronize()
    for name in ("zc", "zf", "o", "d", "xys"):
        assert torch.equal(getattr(trs[0], name), getattr(trs[1], name)), name
    assert torch.equal(trs[0].flat.data, trs[1].flat.data)
