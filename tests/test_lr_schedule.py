"""The reference runner's learning-rate schedule (runners/utils.py:65-109 applied per iteration by runners/apis.py:66-68,
linear world-size scaling of scripts/run.py:152-156), against golden values produced by the reference's own functions
(tests/golden/make_golden.py: gen_lr_schedule). CPU only."""
import ast

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


ITER_CASES = ["lego_w1", "lego_w8", "lego_w3", "lego_cos_w2_b2", "fern_w1", "fern_w4", "fern_w8"]


@pytest.mark.parametrize("tag", ITER_CASES)
def test_setup_iter_based_runner_matches_reference(golden, tag):
    """scripts/run.py:243-271 run by the reference on its product configs (tests/golden/make_golden.py:
    gen_iter_runner): the training loader's length, every rescaled '*iters' / epoch key (including the reference's own
    rescale of num_iters_on_one_gpu, which lands one above num_iters for Fern at 8 ranks), and the per-iteration
    learning rate of the rescaled, world-scaled schedule -- all bit-equal."""
    from yanerf_amd.lr_schedule import setup_iter_based_runner, train_loader_len
    g = golden("iter_runner")
    cfgfile, over, n_train, world, bs = (str(x) for x in g[f"{tag}:case"])
    n_train, world, bs = int(n_train), int(world), int(bs)
    runner = dict(Config.fromfile(str(yanerf_boot.PKG_DIR / cfgfile)).runner)
    runner.update(ast.literal_eval(over))  # the case's overrides (a dict literal written by the generator)
    n_loader = train_loader_len(n_train, world, bs)
    assert n_loader == int(g[f"{tag}:len_loader"])
    r = setup_iter_based_runner(runner, n_loader, world, bs)
    got = np.array([float(r[k]) for k in g["keys"]])
    np.testing.assert_array_equal(got, g[f"{tag}:values"])
    lrs = np.array([lr_at(r, int(it), world) for it in g["iters"]])
    np.testing.assert_array_equal(lrs, g[f"{tag}:lr"])


def test_lr_at_uses_restored_init_lr():
    """A resumed optimizer's param_group['init_lr'] drives the reference's schedulers (min_lr stays the config's)."""
    r = _runner({})
    opt = torch.optim.Adam([{"params": [torch.nn.Parameter(torch.zeros(1))], "init_lr": 7e-4}], lr=7e-4)
    sched = create_lr_scheduler(opt, r)
    for it in (0, 500, 1000, 1001, 5000, 123456):
        apply_schedule(opt, sched, r, it)
        assert lr_at(r, it, 1, init_lr=7e-4) == opt.param_groups[0]["lr"]


def test_trajectory_golden_learning_rates(golden):
    """The 20-step reference trajectory (train_trajectory.npz, make_golden.gen_train_trajectory) ran the lego.yml
    schedule through the reference runner's own functions; the fused trainer's lr_at gives the same rate every step."""
    g = golden("train_trajectory")
    runner = _runner({})
    got = np.array([lr_at(runner, k, 1) for k in range(int(g["steps"]))])
    np.testing.assert_array_equal(got, g["lrs"])
