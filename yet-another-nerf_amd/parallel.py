"""Data parallelism over torch.distributed, one process per GPU (RCCL = the "nccl" backend on ROCm).

Reference: DDP over NCCL (scripts/run.py:162-166; runners/utils.py:216-238), one image / 4096 rays per rank
per step, gradient all-reduce (average) every step and an all_gather of per-image metrics in evaluation
(apis.py:173-177). Here the two MLPs' 1,191,688 fp32 gradients live in ONE flat buffer, so a step issues a
single all-reduce of 4.77 MB (one bucket, well under the point where xGMI ring bandwidth matters: ~55 us on one
153 GB/s link at 8 ranks) instead of DDP's hook-driven per-bucket calls.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


def env_rank_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def init_distributed(backend: Optional[str] = None) -> tuple:
    """Initialise the default process group from torchrun's env (MASTER_ADDR=127.0.0.1 on one node).
    Returns (rank, world_size, local_rank). world_size 1 -> no process group."""
    rank, world, local = env_rank_world()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend=backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend=backend)
    return rank, world, local


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def allreduce_mean_(flat: torch.Tensor) -> torch.Tensor:
    """In-place average of a flat gradient buffer over all ranks (DDP semantics: sum / world)."""
    if is_dist():
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat.div_(dist.get_world_size())
    return flat


def broadcast_(flat: torch.Tensor, src: int = 0) -> torch.Tensor:
    """Make every rank start from rank `src`'s parameters (DDP does this at wrap time)."""
    if is_dist():
        dist.broadcast(flat, src=src)
    return flat


def allgather_cat(x: torch.Tensor) -> torch.Tensor:
    """concat_all_gather of per-image metrics (runners/utils.py:257-267)."""
    if not is_dist():
        return x
    out = [torch.empty_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(out, x.contiguous())
    return torch.cat(out, dim=0)


def max_over_ranks(value: float, device=None) -> float:
    if not is_dist():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier() -> None:
    if is_dist():
        dist.barrier()


def shard_range(n: int, rank: int, world: int) -> range:
    """Contiguous shard of n independent units (images or rays) for `rank`."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return range(lo, hi)


class FlatParams:
    """One flat fp32 storage for a set of parameters (+ a matching flat grad buffer); the modules' parameters
    become views into it, so state_dict/checkpoints are unchanged while all-reduce and the optimizer touch one
    contiguous buffer."""

    def __init__(self, params: Sequence[torch.nn.Parameter]):
        self.params: List[torch.nn.Parameter] = list(params)
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.data = torch.empty(n, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        off = 0
        self.views = []
        for p in self.params:
            k = p.numel()
            self.data[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.data[off:off + k].view_as(p)
            p.grad = self.grad[off:off + k].view_as(p)
            self.views.append((off, k))
            off += k
        self.numel = n

    def grad_views(self) -> List[torch.Tensor]:
        return [p.grad for p in self.params]
