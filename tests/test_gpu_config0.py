"""BASELINE configs[0] on the GPU: the reference's plumbing run (scripts/run.py with lego.yml on a 64x64 crop,
64 coarse samples; the reference ran it with --device cpu) through the drop-in path on the HIP kernels.

scripts/run.py's training loop (runners/apis.py:55-89) is restated in a few lines: a nerf_synthetic-format scene
(procedural, 64x64, written by tools/synthetic_scene.py) read through BlenderDataset and a DataLoader, the registry
NeRFPipeline built from lego.yml, torch.optim.Adam with the runner's schedule applied every iteration (decay, then
warm-up), `objective.backward()`; then the evaluation pass (apis.py:150-203: EVALUATION mode, PSNR of the mean MSE)
and the reference checkpoint format written and read back (run.py:169-178, 409-422). The build has no CPU path (the
kernels are the product), so this is configs[0]'s plumbing on the MI355X rather than on the host."""
import math
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
ROOT = Path(__file__).resolve().parents[1]


def test_config0_plumbing_run_py_loop(tmp_path):
    sys.path.insert(0, str(ROOT / "tools"))
    import yanerf_boot
    from synthetic_scene import write_scene
    from yanerf_amd import checkpoint
    from yanerf_amd.datasets import BlenderDataset
    from yanerf_amd.lr_schedule import apply_schedule, create_lr_scheduler
    from yanerf_amd.pipelines import PIPELINES
    from yanerf_amd.pipelines.utils import EvaluationMode
    from yanerf_amd.utils.config import Config

    data = write_scene(tmp_path / "scene", size=64, n_train=6, n_test=2, device=DEV)
    cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml"))
    pcfg = cfg.pipeline
    pcfg.ray_sampler.image_height = pcfg.ray_sampler.image_width = 64
    pcfg.ray_sampler.n_pts_per_ray_training = pcfg.ray_sampler.n_pts_per_ray_evaluation = 64
    pcfg.ray_sampler.n_rays_per_image_sampled_from_mask = 1024
    runner = dict(cfg.runner)
    runner.update(warmup_steps=3, lr_decay_iters=40, num_iters=30)
    torch.manual_seed(0)
    pipe = PIPELINES.build(pcfg).to(DEV)
    opt = torch.optim.Adam(pipe.parameters(), lr=float(runner["init_lr"]))
    for grp in opt.param_groups:
        grp["init_lr"] = float(runner["init_lr"])  # runners/utils.py:148-151
    sched = create_lr_scheduler(opt, runner)
    train = BlenderDataset(str(data), "train")
    loader = torch.utils.data.DataLoader(train, batch_size=1, shuffle=True,
                                         generator=torch.Generator().manual_seed(0))
    losses = []
    it = 0
    pipe.train()
    while it < runner["num_iters"]:
        for pose, focal, image in loader:
            if it >= runner["num_iters"]:
                break
            apply_schedule(opt, sched, runner, it)
            preds = pipe(poses=pose.to(DEV), focal_lengths=focal.to(DEV), image_rgb=image.to(DEV),
                         evaluation_mode=EvaluationMode.TRAINING)
            opt.zero_grad(set_to_none=True)
            preds["objective"].mean().backward()
            opt.step()
            losses.append(float(preds["objective"].detach().mean()))
            it += 1
    assert all(math.isfinite(v) for v in losses)
    assert sum(losses[-5:]) / 5 < 0.8 * sum(losses[:5]) / 5, losses

    def evaluate(model):
        model.eval()
        mse = []
        with torch.no_grad():
            for pose, focal, image in torch.utils.data.DataLoader(BlenderDataset(str(data), "test", test_skip=1),
                                                                  batch_size=1):
                out = model(poses=pose.to(DEV), focal_lengths=focal.to(DEV), image_rgb=image.to(DEV),
                            evaluation_mode=EvaluationMode.EVALUATION)
                mse.append(out["loss_rgb_mse"].mean())
        return torch.stack(mse)

    mse = evaluate(pipe)
    psnr = -10.0 * math.log10(float(mse.mean()))
    assert 5.0 < psnr < 60.0, psnr
    path = checkpoint.save_checkpoint(str(tmp_path), pipe, opt, epoch=0)
    assert Path(path).name == "ckpts_0000.pth"
    pipe2 = PIPELINES.build(pcfg).to(DEV)
    opt2 = torch.optim.Adam(pipe2.parameters(), lr=1.0)
    assert checkpoint.load_checkpoint(path, pipe2, opt2, map_location=DEV) == 1
    assert opt2.param_groups[0]["init_lr"] == float(runner["init_lr"])
    assert torch.equal(evaluate(pipe2), mse)
