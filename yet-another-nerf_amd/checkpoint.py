"""Checkpoints in the reference's format (scripts/run.py:168-178 load, :409-414 save):

    {"model": NeRFPipeline.state_dict(), "optimizer": torch.optim.Adam.state_dict(), "epoch": int}

The registry `NeRFPipeline` here has the reference's module tree, so its state_dict IS the reference layout
(tests/test_host.py pins the 48 keys, shapes and seeded initialisation against the reference). The fused trainer
(`train.NeRFTrainer`) keeps its two NeRFMLPs in one flat parameter buffer with flat Adam moments; this module
converts both ways, so a checkpoint written by the reference resumes in the fused trainer and vice versa.

Loading uses `torch.load(..., weights_only=True)`: a checkpoint is data (tensors, numbers, dicts), never code.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch

PREFIX = "implicit_functions.{i}._fn."


def save_checkpoint(path: str, model, optimizer=None, epoch: int = 0) -> str:
    """Write `{"model", "optimizer", "epoch"}` (run.py:409-414). `model` is a NeRFPipeline (any nn.Module) or a
    NeRFTrainer; `optimizer` a torch optimizer (ignored for a trainer, which carries its own Adam state). If
    `path` is a directory the file is `<path>/ckpts/ckpts_<epoch:04d>.pth`, as the reference names it."""
    if os.path.isdir(path):
        os.makedirs(os.path.join(path, "ckpts"), exist_ok=True)
        path = os.path.join(path, "ckpts", f"ckpts_{epoch:04d}.pth")
    if hasattr(model, "pipeline_state_dict"):
        obj = {"model": model.pipeline_state_dict(), "optimizer": model.optimizer_state_dict(), "epoch": int(epoch)}
    else:
        obj = {"model": model.state_dict(), "optimizer": optimizer.state_dict() if optimizer is not None else {},
               "epoch": int(epoch)}
    torch.save(obj, path)
    return path


def load_checkpoint(path: str, model, optimizer=None, map_location="cpu") -> int:
    """Load a reference-format checkpoint into a NeRFPipeline (+ optional torch optimizer) or a NeRFTrainer.
    Returns the epoch to resume from (`checkpoint["epoch"] + 1`, run.py:176)."""
    ck = torch.load(path, map_location=map_location, weights_only=True)
    if hasattr(model, "load_pipeline_state_dict"):
        model.load_pipeline_state_dict(ck["model"])
        if ck.get("optimizer"):
            model.load_optimizer_state_dict(ck["optimizer"])
    else:
        model.load_state_dict(ck["model"])
        if optimizer is not None and ck.get("optimizer"):
            optimizer.load_state_dict(ck["optimizer"])
    return int(ck["epoch"]) + 1


def split_pipeline_state(sd: Dict[str, torch.Tensor], n_models: int = 2):
    """{"implicit_functions.{i}._fn.<key>": t} -> [ {<key>: t} for each model ]."""
    out = [dict() for _ in range(n_models)]
    for k, v in sd.items():
        for i in range(n_models):
            p = PREFIX.format(i=i)
            if k.startswith(p):
                out[i][k[len(p):]] = v
                break
        else:
            raise KeyError(f"unexpected key in pipeline state_dict: {k}")
    return out


def adam_state_from_flat(params, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, step: int, lr: float,
                         betas, eps: float, weight_decay: float, init_lr: Optional[float] = None) -> Dict:
    """torch.optim.Adam.state_dict() for `params` (in order) from flat moment buffers. The param group carries the
    reference's `init_lr` key (runners/utils.py:148-151), which its lr schedulers read every iteration (:65-86):
    torch's Optimizer.load_state_dict replaces the whole group with the saved one, so without it a reference run
    resumed from this checkpoint would fail on its first scheduler call."""
    state, off = {}, 0
    for i, p in enumerate(params):
        n = p.numel()
        state[i] = {"step": torch.tensor(float(step)),
                    "exp_avg": exp_avg[off:off + n].view_as(p).detach().cpu().clone(),
                    "exp_avg_sq": exp_avg_sq[off:off + n].view_as(p).detach().cpu().clone()}
        off += n
    group = {"lr": float(lr), "init_lr": float(lr if init_lr is None else init_lr),
             "betas": tuple(float(b) for b in betas), "eps": float(eps),
             "weight_decay": float(weight_decay), "amsgrad": False, "maximize": False, "foreach": None,
             "capturable": False, "differentiable": False, "fused": None, "params": list(range(len(params)))}
    return {"state": state if step > 0 else {}, "param_groups": [group]}


def adam_state_to_flat(osd: Dict, params, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor) -> Optional[int]:
    """Copy a torch Adam state_dict's moments into flat buffers; returns its step (None if it holds no state)."""
    st = osd.get("state", {})
    if not st:
        exp_avg.zero_()
        exp_avg_sq.zero_()
        return 0
    off, step = 0, None
    for i, p in enumerate(params):
        n = p.numel()
        s = st[i] if i in st else st[str(i)]
        exp_avg[off:off + n].copy_(s["exp_avg"].reshape(-1))
        exp_avg_sq[off:off + n].copy_(s["exp_avg_sq"].reshape(-1))
        step = int(float(s["step"]))
        off += n
    return step
