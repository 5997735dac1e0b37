"""The reference runner's learning-rate schedule (runners/utils.py:65-109 applied per iteration by runners/apis.py:66-68,
linear world-size scaling of scripts/run.py:152-156), against golden values produced by the reference's own functions
(tests/golden/make_golden.py: gen_lr_schedule). CPU only."""
import numpy as np
import pytest
import torch

import yanerf_boot
from yanerf_amd import checkpoint
from yanerf_amd.lr_schedule import apply_schedule, create_lr_scheduler, lr_at, scaled_lrs
from yanerf_amd.utils.config import Config

VARIANTS = {
    "lego_w1": dict(),
    "lego_w8": dict(),
    "cosine_w2": dict(lr_decay_type="cosine"),
    "nowarm_w1": dict(warmup_steps=0),
    "shortwarm_cos_w1": dict(lr_decay_type="cosine", warmup_steps=7, warmup_lr=2e-4, lr_decay_iters=50, num_iters=300),
}


def _runner(over):
    r = dict(Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml")).runner)
    r.update(over)
    return r


@pytest.mark.parametrize("tag", list(VARIANTS))
def test_lr_at_matches_reference(golden, tag):
    g = golden("lr_schedule")
    world = int(g[f"{tag}:world"])
    runner = _runner(VARIANTS[tag])
    got = np.array([lr_at(runner, int(it), world) for it in g["iters"]])
    np.testing.assert_array_equal(got, g[f"{tag}:lr"])  # same float arithmetic, bit-equal


@pytest.mark.parametrize("tag", list(VARIANTS))
def test_optimizer_schedule_matches_reference(golden, tag):
    """The optimizer-level restatement (param_group['init_lr'] -> param_group['lr']) on a torch Adam."""
    g = golden("lr_schedule")
    world = int(g[f"{tag}:world"])
    runner = _runner(VARIANTS[tag])
    init, mn = scaled_lrs(runner, world)
    runner = dict(runner, init_lr=init, min_lr=mn)  # run.py:152-156 rewrites the config before the scheduler
    opt = torch.optim.Adam([{"params": [torch.nn.Parameter(torch.zeros(1))], "init_lr": init}], lr=init)
    sched = create_lr_scheduler(opt, runner)
    got = []
    for it in g["iters"].tolist():
        apply_schedule(opt, sched, runner, it)
        got.append(opt.param_groups[0]["lr"])
    np.testing.assert_array_equal(np.array(got), g[f"{tag}:lr"])


def test_warmup_boundary_and_order():
    """Warm-up applies while passed_iter <= warmup_steps (inclusive) and overrides the decay; not at all when
    warmup_steps == 0; unknown decay types raise like the reference."""
    r = _runner({})
    assert lr_at(r, 0) == r["warmup_lr"]
    assert lr_at(r, r["warmup_steps"]) == min(r["init_lr"], r["warmup_lr"] + (r["init_lr"] - r["warmup_lr"]))
    assert lr_at(r, r["warmup_steps"] + 1) == max(r["min_lr"], r["init_lr"] * r["lr_decay_rate"] **
                                                  ((r["warmup_steps"] + 1) / r["lr_decay_iters"]))
    assert lr_at(dict(r, warmup_steps=0), 0) == r["init_lr"]
    with pytest.raises(ValueError):
        lr_at(dict(r, lr_decay_type="linear"), 5)
    assert scaled_lrs(r, 8) == (r["init_lr"] * 8, r["min_lr"] * 8)
    assert scaled_lrs(dict(r, linear_scale=False), 8) == (r["init_lr"], r["min_lr"])


def test_trainer_optimizer_state_resumes_under_reference_scheduler():
    """A NeRFTrainer checkpoint's optimizer state carries `init_lr`, so the reference runner's schedulers (which read
    param_group['init_lr'] every iteration) keep working after torch's load_state_dict replaces the group."""
    params = [torch.nn.Parameter(torch.randn(3, 2)), torch.nn.Parameter(torch.randn(4))]
    n = sum(p.numel() for p in params)
    osd = checkpoint.adam_state_from_flat(params, torch.rand(n), torch.rand(n), 7, lr=1.5e-4, betas=(0.9, 0.999),
                                          eps=1e-8, weight_decay=0.0, init_lr=5e-4)
    opt = torch.optim.Adam([{"params": params, "init_lr": 1.0}], lr=1.0)
    opt.load_state_dict(osd)
    assert opt.param_groups[0]["init_lr"] == 5e-4
    r = _runner({})
    sched = create_lr_scheduler(opt, r)
    apply_schedule(opt, sched, r, 2000)
    assert opt.param_groups[0]["lr"] == lr_at(r, 2000)
