"""Data parallelism over torch.distributed, one process per GPU (RCCL = the "nccl" backend on ROCm).

Reference: DDP over NCCL (scripts/run.py:162-166; runners/utils.py:216-238), one image / 4096 rays per rank
per step, gradient all-reduce (average) every step and an all_gather of per-image metrics in evaluation
(apis.py:173-177). Here the two MLPs' 1,191,688 fp32 gradients live in ONE flat buffer, and NeRFTrainer.step
exchanges it in two buckets, one per model (2.38 MB each): the coarse bucket's all-reduce is started asynchronously
right after the coarse MLP backward and runs on the collective stream while the fine MLP backward computes; only the
fine bucket's all-reduce is exposed (~55 us for all 4.77 MB on one 153 GB/s xGMI link at 8 ranks by a ring estimate).
`grad_exchange="single"` (or YANERF_GRAD_EXCHANGE=single) is the one-call fallback: both backwards, then one
all-reduce of the whole buffer. The per-element sums are the same either way.
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
    # YANERF_PG_AT_WORLD1=1: a process group even at world size 1, so one card runs the N-rank step schedule with its
    # collectives (bench.py's rehearsal of the exchange overlap against the plain N=1 line)
    want = world > 1 or os.environ.get("YANERF_PG_AT_WORLD1") == "1"
    if want and not dist.is_initialized():
        # YANERF_DIST_BACKEND=gloo: a rehearsal of the N-rank code path with several ranks on one card (RCCL needs one
        # card per rank); the measured runs use the default, RCCL
        backend = backend or os.environ.get("YANERF_DIST_BACKEND") or None
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            local = device_index(local)
            torch.cuda.set_device(local)
            dist.init_process_group(backend=backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend=backend)
    return rank, world, local


def device_index(local_rank: int) -> int:
    """The card of a local rank: one card per rank; ranks beyond the visible cards (a one-card rehearsal of an
    N-rank run) share them round-robin."""
    n = torch.cuda.device_count()
    return local_rank % n if n > 0 else local_rank


def is_dist() -> bool:
    """A process group is up (any size: a world-1 group over RCCL runs the N-rank code path, collectives included)."""
    return dist.is_available() and dist.is_initialized()


def allreduce_mean_(flat: torch.Tensor) -> torch.Tensor:
    """In-place average of a flat gradient buffer over all ranks (DDP semantics: sum / world)."""
    if is_dist():
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat.div_(dist.get_world_size())
    return flat


def allreduce_sum_(flat: torch.Tensor) -> torch.Tensor:
    """In-place sum of a flat buffer over all ranks (the caller divides by the world size: NeRFTrainer does it inside
    its Adam launch)."""
    if is_dist():
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    return flat


def allreduce_sum_async(t: torch.Tensor):
    """Start a sum all-reduce of `t` in place and return its handle (None without a process group). Under RCCL the
    collective runs on the process group's own stream after the work already queued on the current stream, so
    kernels queued afterwards overlap it; `finish_allreduce` makes the current stream wait for it."""
    if not is_dist():
        return None
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)


def finish_allreduce(handle) -> None:
    if handle is not None:
        handle.wait()


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
    _all_gather(out, x.contiguous())
    return torch.cat(out, dim=0)


def _all_gather(parts: List[torch.Tensor], x: torch.Tensor) -> None:
    """all_gather that also runs under gloo with device tensors (CPU round trip; RCCL gathers in place)."""
    if x.is_cuda and dist.get_backend() == "gloo":
        host = [torch.empty_like(p, device="cpu") for p in parts]
        dist.all_gather(host, x.cpu())
        for p, h in zip(parts, host):
            p.copy_(h)
    else:
        dist.all_gather(parts, x)


def max_over_ranks(value: float, device=None) -> float:
    if not is_dist():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allgather_floats(value: float, device=None) -> List[float]:
    """Every rank's `value`, in rank order (one all_gather of a float64; [value] without a process group)."""
    if not is_dist():
        return [float(value)]
    t = torch.tensor([value], dtype=torch.float64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    _all_gather(parts, t)
    return [float(x.item()) for x in parts]


def barrier() -> None:
    if is_dist():
        dist.barrier()


def shard_range(n: int, rank: int, world: int) -> range:
    """Contiguous shard of n independent units (images or rays) for `rank`."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return range(lo, hi)


def world_rank() -> tuple:
    """(world_size, rank) of the default group, (1, 0) without one."""
    if is_dist():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def eval_order(n: int, rank: int, world: int) -> List[int]:
    """The evaluation split of one rank: DistributedSampler(shuffle=False, drop_last=False) (runners/utils.py:
    112-131) pads the index list to a multiple of the world size by repeating it from the head, then rank r takes
    every world-th index from r. Gathering one item from every rank per iteration and concatenating the iterations
    (apis.py:173-177) restores dataset order; the padding is cut off by the final [: len(dataset)] (apis.py:201)."""
    total = -(-n // world) * world
    order = list(range(n))
    pad = total - n
    order = order + (order * -(-pad // n))[:pad] if n else []
    return order[rank:total:world]


def gather_rows(local: torch.Tensor, n_total: int) -> torch.Tensor:
    """Assemble a tensor sharded by `shard_range(n_total, rank, world)` along dim 0 on every rank: each shard is
    padded to the largest shard's length, all-gathered, and the padding dropped. One collective per call."""
    world, _ = world_rank()
    if world == 1:
        return local
    cap = -(-n_total // world)
    buf = local.new_zeros((cap,) + tuple(local.shape[1:]))
    buf[: local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    _all_gather(parts, buf)
    return torch.cat([parts[k][: len(shard_range(n_total, k, world))] for k in range(world)], dim=0)


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
