"""Learning-rate schedule of the reference runner, for the fused trainer and for torch optimizers.

Reference: runners/utils.py:65-109 (warmup_lr_scheduler, cosine_lr_scheduler, step_lr_scheduler,
create_lr_scheduler), applied once per iteration before the forward in runners/apis.py:66-68:

    scheduler(iter=passed_iter)                                   # decay, from param_group["init_lr"]
    if warmup_steps > 0 and passed_iter <= warmup_steps:          # then warm-up (overrides the decay)
        warmup_lr_scheduler(optimizer, passed_iter, warmup_steps, warmup_lr)

`passed_iter` counts from 0 (apis.py:42, 117). Before any of that, scripts/run.py:144 converts the iteration-based
runner config to epochs (`setup_iter_based_runner`, run.py:243-271): num_iters becomes a whole number of epochs of the
rank's training loader, and every other '*iters' key (lr_decay_iters) is rescaled by the same factor -- at 8 ranks on
Lego's 100 training images num_iters 200000 -> 25012 and lr_decay_iters 250000 -> 31265. With torch.distributed and
`linear_scale`, init_lr and min_lr (not warmup_lr) are then multiplied by the world size before the optimizer is built
(run.py:152-156).

The optimizer-level functions below write `param_group["lr"]` from `param_group["init_lr"]` exactly as the reference
does, so an optimizer restored from a NeRFTrainer checkpoint (checkpoint.adam_state_from_flat stores `init_lr`) keeps
working under the reference runner. `lr_at` is the same arithmetic as a pure function of the iteration.
"""
from __future__ import annotations

import math
from functools import partial
from typing import Mapping


def _get(cfg, key, default=None):
    if isinstance(cfg, Mapping):
        return cfg.get(key, default)
    return getattr(cfg, key, default)


def warmup_lr_scheduler(optimizer, step, max_step, warmup_lr):
    """runners/utils.py:65-70."""
    for g in optimizer.param_groups:
        init_lr = g["init_lr"]
        g["lr"] = min(init_lr, warmup_lr + (init_lr - warmup_lr) * step / max_step)


def cosine_lr_scheduler(optimizer, iter, lr_decay_iters, min_lr, num_iters):  # noqa: A002 (reference name)
    """runners/utils.py:73-79 (the reference divides the cosine phase by num_iters a second time; kept)."""
    for g in optimizer.param_groups:
        g["lr"] = (g["init_lr"] - min_lr) * 0.5 * (1.0 + math.cos(math.pi * (iter / lr_decay_iters) / num_iters)) \
            + min_lr


def step_lr_scheduler(optimizer, iter, lr_decay_iters, min_lr, lr_decay_rate):  # noqa: A002
    """runners/utils.py:82-86."""
    for g in optimizer.param_groups:
        g["lr"] = max(min_lr, g["init_lr"] * (lr_decay_rate ** (iter / lr_decay_iters)))


def create_lr_scheduler(optimizer, runner_cfg):
    """runners/utils.py:89-109: a callable `sched(iter=...)`; ValueError for an unknown lr_decay_type."""
    kind = _get(runner_cfg, "lr_decay_type")
    if kind == "exponential":
        return partial(step_lr_scheduler, optimizer=optimizer, lr_decay_iters=_get(runner_cfg, "lr_decay_iters"),
                       min_lr=_get(runner_cfg, "min_lr"), lr_decay_rate=_get(runner_cfg, "lr_decay_rate"))
    if kind == "cosine":
        return partial(cosine_lr_scheduler, optimizer=optimizer, lr_decay_iters=_get(runner_cfg, "lr_decay_iters"),
                       min_lr=_get(runner_cfg, "min_lr"), num_iters=_get(runner_cfg, "num_iters"))
    raise ValueError(f"unknown lr_decay_type {kind!r}")


def apply_schedule(optimizer, scheduler, runner_cfg, passed_iter: int) -> None:
    """The per-iteration order of runners/apis.py:66-68: decay, then warm-up while passed_iter <= warmup_steps."""
    scheduler(iter=passed_iter)
    warm = int(_get(runner_cfg, "warmup_steps", 0) or 0)
    if warm > 0 and passed_iter <= warm:
        warmup_lr_scheduler(optimizer, passed_iter, warm, float(_get(runner_cfg, "warmup_lr")))


def train_loader_len(n_train: int, world_size: int = 1, batch_size: int = 1) -> int:
    """len() of the reference's training DataLoader (runners/utils.py:112-145): a DistributedSampler under
    torch.distributed (ceil(N / world) samples per rank, padded), batches of batch_size with drop_last=True."""
    n = math.ceil(n_train / world_size) if world_size > 1 else int(n_train)
    return n // int(batch_size)


def setup_iter_based_runner(runner_cfg, len_loader: int, world_size: int = 1, batch_size: int = 1) -> dict:
    """scripts/run.py:243-271 on a copy of the runner config (key order kept: the reference rescales the keys in
    iteration order, and `num_iters_on_one_gpu`, appended by the function itself, is rescaled too -- after the
    original keys, so the factor they see is the unmodified one)."""
    r = dict(runner_cfg)
    iters_per_epoch = int(len_loader) * int(world_size) * int(batch_size)
    r["num_iters_on_one_gpu"] = r["num_iters"]
    r["num_epochs"] = math.ceil(r["num_iters"] / iters_per_epoch)
    r["num_iters"] = r["num_epochs"] * int(len_loader)
    r["val_per_epoch"] = max(1, math.floor(r["val_per_iter"] / iters_per_epoch))
    r["save_per_epoch"] = max(1, math.floor(r["save_per_iter"] / iters_per_epoch))
    for key in list(r.keys()):
        if key != "num_iters" and "iters" in key:
            r[key] = math.ceil(r[key] * (r["num_iters"] / r["num_iters_on_one_gpu"]))
    return r


def scaled_lrs(runner_cfg, world_size: int = 1):
    """(init_lr, min_lr) after the linear world-size scaling of scripts/run.py:152-156 (only under
    torch.distributed, i.e. world_size > 1, and only when runner.linear_scale is set)."""
    init, mn = float(_get(runner_cfg, "init_lr")), float(_get(runner_cfg, "min_lr", 0.0) or 0.0)
    if world_size > 1 and bool(_get(runner_cfg, "linear_scale", False)):
        init, mn = init * world_size, mn * world_size
    return init, mn


def lr_at(runner_cfg, it: int, world_size: int = 1, init_lr=None) -> float:
    """The learning rate the reference runner uses at iteration `it` (0-based), as a pure function: the decay
    schedule from init_lr, then the warm-up override while it <= warmup_steps (warmup_steps > 0). `runner_cfg` is the
    config after setup_iter_based_runner. `init_lr` overrides the (world-scaled) config value, as a resumed
    optimizer's param_group["init_lr"] does for the reference's schedulers (run.py:169-178; min_lr stays the config's)."""
    init, mn = scaled_lrs(runner_cfg, world_size)
    if init_lr is not None:
        init = float(init_lr)
    kind = _get(runner_cfg, "lr_decay_type")
    decay_iters = _get(runner_cfg, "lr_decay_iters")
    if kind == "exponential":
        lr = max(mn, init * (_get(runner_cfg, "lr_decay_rate") ** (it / decay_iters)))
    elif kind == "cosine":
        lr = (init - mn) * 0.5 * (1.0 + math.cos(math.pi * (it / decay_iters) / _get(runner_cfg, "num_iters"))) + mn
    else:
        raise ValueError(f"unknown lr_decay_type {kind!r}")
    warm = int(_get(runner_cfg, "warmup_steps", 0) or 0)
    if warm > 0 and it <= warm:
        wl = float(_get(runner_cfg, "warmup_lr"))
        lr = min(init, wl + (init - wl) * it / warm)
    return lr
