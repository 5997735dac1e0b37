"""Training converges on the HIP path, in every precision mode.

1. The reference's own integration test (tests/test_runner.py:42-104): the small test MLP pipeline
   (tests/configs/pipelines/nerf_pipeline_cfg_with_mlp.py, models/nerf_mlp.yml, ray_sampler.yml,
   renderers/multipass_emission_absorption_renderer.yml), a 2x2 image seen from 3 identical cameras, 50 Adam
   iterations with the runner.yml schedule (warm-up 3 its from 1e-5, cosine to 5e-5, init 1e-3), batch 2, then an
   evaluation pass whose objective must be < 0.01 (:104). Run through the registry NeRFPipeline + torch autograd +
   torch.optim.Adam, i.e. the drop-in path scripts/run.py uses.
2. The fused trainer (yanerf_amd.train.NeRFTrainer, the bench's step) on the Lego architecture fitting a smooth
   synthetic 32x32 target: the loss must fall by a fixed factor in every precision (bf16 included), which pins
   the whole training step (raygen, both MLP passes, compositing, refinement, backward, Adam) end to end.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"

SMALL_PIPELINE = dict(
    type="NeRFPipeline",
    model=dict(type="NeRFMLP", n_layers=5, input_skips=[2], n_harmonic_functions_xyz=8,
               harmonic_functions_xyz_append_intput=True, n_hidden_neurons_xyz=64, n_harmonic_functions_dir=4,
               harmonic_functions_dir_append_intput=True, n_hidden_neurons_dir=32, latent_dim=0, input_xyz=True,
               input_dir=True, color_dim=3),
    ray_sampler=dict(type="RaySampler", image_width=10, image_height=6, n_rays_per_image_sampled_from_mask=4,
                     min_depth=0.5, max_depth=1.0, scene_extent=0.0, n_pts_per_ray_training=5,
                     n_pts_per_ray_evaluation=5, stratified_point_sampling_training=True,
                     stratified_point_sampling_evaluation=False),
    renderer=dict(type="MultipassEmissionAbsorpsionRenderer", n_pts_per_ray_fine_training=5,
                  n_pts_per_ray_fine_evaluation=5, append_coarse_samples_to_fine=True, density_noise_std_train=1.0,
                  bg_color=[0.0, 0.0, 0.0], blend_output=False),
    chunk_size_grid=30, num_passes=2,
    loss_weights={"loss_rgb_mse": 1.0, "loss_prev_stage_rgb_mse": 1.0},
    output_rasterized_mc=True, feature_extractor=dict(type="IdentityMapper"))
RUNNER = dict(init_lr=1.0e-3, warmup_steps=3, warmup_lr=1.0e-5, lr_decay_type="cosine", min_lr=5.0e-5,
              lr_decay_rate=0.9, lr_decay_iters=10, num_iters=50)


@pytest.mark.parametrize("precision", ["fp32", "fp32x3", "bf16"])
def test_reference_runner_convergence(precision):
    import copy

    import yanerf_boot  # noqa: F401
    from yanerf_amd.pipelines import PIPELINES
    from yanerf_amd.pipelines.utils import EvaluationMode
    from yanerf_amd.lr_schedule import apply_schedule, create_lr_scheduler
    torch.manual_seed(0)
    np.random.seed(0)
    cfg = copy.deepcopy(SMALL_PIPELINE)
    cfg["model"]["precision"] = precision
    H = W = 2
    cfg["ray_sampler"]["image_height"], cfg["ray_sampler"]["image_width"] = H, W
    pipe = PIPELINES.build(cfg).to(DEV)
    B = 3
    pose = torch.cat([torch.eye(3), torch.tensor([[0.0], [0.0], [-1.0]])], dim=-1)
    poses = pose[None].expand(B, 3, 4).contiguous().to(DEV)
    focal = torch.ones(B, device=DEV)
    img = (torch.randn(H, W, 3).abs() * 255).to(torch.uint8).float() / 255.0  # test_runner.py:72-75
    images = img[None].expand(B, -1, -1, -1).contiguous().to(DEV)
    # one param group carrying init_lr, as the reference's create_param_groups builds it (runners/utils.py:148-151)
    opt = torch.optim.Adam([{"params": pipe.parameters(), "init_lr": RUNNER["init_lr"]}], lr=RUNNER["init_lr"])
    sched = create_lr_scheduler(opt, RUNNER)
    pipe.train()
    order = np.arange(B)
    it = 0
    while it < RUNNER["num_iters"]:  # batch 2, drop_last (runners/utils.py:129-131): one batch per epoch
        np.random.shuffle(order)
        idx = torch.as_tensor(order[:2], device=DEV)
        apply_schedule(opt, sched, RUNNER, it)  # runners/apis.py:66-68
        preds = pipe(poses=poses[idx], focal_lengths=focal[idx], image_rgb=images[idx],
                     evaluation_mode=EvaluationMode.TRAINING)
        opt.zero_grad(set_to_none=True)
        preds["objective"].mean().backward()
        opt.step()
        it += 1
    pipe.eval()
    with torch.no_grad():
        objs = [pipe(poses=poses[s:s + 2], focal_lengths=focal[s:s + 2], image_rgb=images[s:s + 2],
                     evaluation_mode=EvaluationMode.EVALUATION)["objective"].mean().item() for s in (0, 2)]
    obj = float(np.mean(objs))
    print(f"{precision}: eval objective after 50 its {obj:.5f}")
    assert obj < 0.01, obj  # test_runner.py:104


def _target(H, W):
    y, x = np.mgrid[0:H, 0:W].astype(np.float32)
    img = np.stack([0.5 + 0.4 * np.sin(x / 5.0), 0.5 + 0.4 * np.cos(y / 7.0), 0.5 + 0.3 * np.sin((x + y) / 9.0)], -1)
    return torch.from_numpy(img[None]).to(DEV)


@pytest.mark.parametrize("precision", ["fp32", "fp32x3", "bf16", "bf16s"])
def test_fused_trainer_converges(precision):
    import yanerf_boot  # noqa: F401
    from yanerf_amd.train import NeRFTrainer
    from yanerf_amd.utils.config import Config
    from scene import synthetic_pose
    cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml")).pipeline
    H = W = 32
    cfg.ray_sampler.image_height = H
    cfg.ray_sampler.image_width = W
    image = _target(H, W)
    pose = torch.from_numpy(synthetic_pose(30.0, -30.0, 4.0)).float()[None, :3, :4].contiguous().to(DEV)
    focal = torch.tensor([0.5 * W / math.tan(0.5 * 0.6911112)], device=DEV)
    tr = NeRFTrainer(cfg, precision=precision, device=DEV, n_rays=512, lr=5e-4, seed=3)
    losses = []
    for _ in range(300):
        out = tr.step(pose, focal, image)
        losses.append(float(NeRFTrainer.objective(out)))
    first, last = np.mean(losses[:10]), np.mean(losses[-20:])
    print(f"{precision}: fused-trainer loss {first:.4f} -> {last:.4f}")
    assert np.isfinite(losses).all()
    assert last < 0.02 * first, (first, last)  # measured ~1e-3 of the first loss in every mode


def test_trained_activations_stay_below_fp8_clamp(tmp_path):
    """The bf16 mode stores the post-ReLU activations H_0..H_7 and C for the weight gradients as fp8 e4m3 WITHOUT a
    scale, clamped at 448 (a value above it would give a wrong weight gradient). This pins the assumption
    on trained weights: the fused bf16 trainer fits the procedural nerf_synthetic-format scene (tools/synthetic_scene,
    Lego config, 1,500 steps), then the oracle evaluates its fp32 master weights on the rays of a test view and every
    trunk / colour-hidden activation must stay below 448 / 8 (a margin of 8x). The maxima go to the parity report."""
    import sys
    from pathlib import Path

    import yanerf_boot  # noqa: F401
    from oracle import nerf_oracle as O
    from parity_gates import write_report
    from weights import LEGO_ARCH
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root / "tools"))
    from synthetic_scene import write_scene
    from yanerf_amd.datasets import BlenderDataset, DeviceImageSet
    from yanerf_amd.train import NeRFTrainer
    from yanerf_amd.utils.config import Config

    data = write_scene(tmp_path / "scene", 64, 20, 2, device=DEV)
    train = DeviceImageSet(BlenderDataset(str(data), "train"), DEV)
    cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml"))
    pcfg = cfg.pipeline
    pcfg.ray_sampler.image_height, pcfg.ray_sampler.image_width = train.H, train.W
    runner = dict(cfg.runner)
    steps = 1500
    runner["warmup_steps"], runner["lr_decay_iters"] = steps // 10, steps * 1.25
    tr = NeRFTrainer(pcfg, precision="bf16", device=DEV, runner_cfg=runner, seed=7)
    it, epoch = 0, 0
    while it < steps:
        for i in train.epoch_order(epoch, seed=7):
            if it >= steps:
                break
            pose, focal, img, _, _ = train.item(i)
            tr.step(pose, focal, img)
            it += 1
        epoch += 1
    torch.cuda.synchronize()
    arch = O.MLPArch.from_dict(LEGO_ARCH)
    pose, focal, _, _, _ = train.item(0)
    pose_np = pose.reshape(1, 3, 4).cpu().numpy()
    o, d, z, _ = O.sample_rays_eval(pose_np, focal.reshape(1).cpu().numpy(), train.W, train.H, tr.near, tr.far, 64)
    o, d, z = o.reshape(-1, 3), d.reshape(-1, 3), z.reshape(-1, 64)
    rows = np.arange(0, o.shape[0], 16)  # 256 rays of the view
    maxima = {}
    for k, model in enumerate(tr.models):
        params = {n: p.detach().cpu().numpy() for n, p in model.state_dict().items()}
        _, _, cache = O.nerf_mlp_forward(params, arch, o[rows], d[rows], z[rows])
        maxima[("coarse", "fine")[k]] = [float(h.max()) for h in cache.layer_out] + [float(cache.c0.max())]
    write_report("activation_range", "bf16 trained 1500 steps, procedural scene", {"max_post_relu": maxima,
                                                                                   "fp8_clamp": 448.0})
    worst = max(max(v) for v in maxima.values())
    assert np.isfinite(worst) and worst < 448.0 / 8, maxima
