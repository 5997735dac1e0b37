"""Sharded evaluation on the HIP path with more than one rank: two gloo ranks share cuda:0 (the round-end GPU box has
one card; the RCCL path runs the same code with one card per rank). Each rank renders its block of image rows
(NeRFTrainer.render(shard=True)) and its DistributedSampler split of the test views (NeRFTrainer.evaluate); the
gathered image and the metrics must equal the single-rank results exactly (rays are independent and the per-image
MSEs are averaged in dataset order)."""
import os
import queue
import socket
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from mp_util import _as_tensors, _by_value

pytestmark = pytest.mark.gpu

H, W, N_VIEWS = 13, 20, 5  # odd row count and a view count that is not a multiple of the world size


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    import yanerf_boot
    from scene import synthetic_pose
    from yanerf_amd.datasets import DeviceImageSet
    from yanerf_amd.train import NeRFTrainer
    from yanerf_amd.utils.config import Config
    cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml")).pipeline
    tr = NeRFTrainer(cfg, precision="fp32", device="cuda:0", n_rays=256, seed=4)
    g = torch.Generator().manual_seed(7)
    items = []
    for k in range(N_VIEWS):
        pose = torch.eye(4)
        pose[:3, :4] = torch.from_numpy(synthetic_pose(-150.0 + 60.0 * k, -30.0, 4.0)).float()[:3, :4]
        items.append((pose, torch.tensor([1111.111]), torch.rand(H, W, 3, generator=g)))
    views = DeviceImageSet(items, "cuda:0")
    return tr, views


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests" / "golden")]
    import yanerf_boot  # noqa: F401  (registers the yanerf_amd package)
    from yanerf_amd import parallel
    parallel.init_distributed(backend="gloo")
    torch.cuda.set_device(0)
    tr, views = _setup()
    pose, focal, _, _, _ = views.item(1)
    f, c, d = tr.render(pose, focal, H, W, chunk=97, shard=True)
    ev = tr.evaluate(views)
    torch.cuda.synchronize()
    q.put(_by_value((rank, f.cpu(), c.cpu(), d.cpu(), ev)))
    parallel.barrier()
    torch.distributed.destroy_process_group()


def test_sharded_render_and_evaluate_two_ranks():
    tr, views = _setup()
    pose, focal, _, _, _ = views.item(1)
    f0, c0, d0 = (x.cpu() for x in tr.render(pose, focal, H, W))
    ev0 = tr.evaluate(views)
    torch.cuda.synchronize()
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        deadline = time.monotonic() + 150
        while len(res) < world and time.monotonic() < deadline:
            try:
                res.append(_as_tensors(q.get(timeout=2)))
            except queue.Empty:
                assert all(p.is_alive() or p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        res.sort(key=lambda x: x[0])
        assert len(res) == world
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    for _, f, c, d, ev in res:
        assert f.shape == (H, W, 3) and d.shape == (H, W)
        assert torch.equal(f, f0) and torch.equal(c, c0) and torch.equal(d, d0)
        for k, v in ev0.items():
            assert np.float64(ev[k]) == np.float64(v), (k, ev[k], v)


# ------------------------------------------------------------------------------------------- training exchange
def _spawn(target, world, extra=()):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + tuple(extra)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        deadline = time.monotonic() + 150
        while len(res) < world and time.monotonic() < deadline:
            try:
                res.append(_as_tensors(q.get(timeout=2)))
            except queue.Empty:
                assert all(p.is_alive() or p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        res.sort(key=lambda x: x[0])
        assert len(res) == world
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return res


def _init_worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests" / "golden")]
    import yanerf_boot  # noqa: F401
    from yanerf_amd import parallel
    parallel.init_distributed(backend="gloo")
    torch.cuda.set_device(0)


def _trainer_worker(rank, world, port, q):
    """Three fused training steps per rank on rank-specific images; records each step's local (pre-exchange)
    gradient, the exchanged gradient, the parameters and the sampled pixels."""
    _init_worker(rank, world, port)
    from scene import synthetic_pose
    from yanerf_amd import parallel
    from yanerf_amd.train import NeRFTrainer
    from yanerf_amd.utils.config import Config
    import yanerf_boot
    cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml"))
    # the two-bucket exchange explicitly (at 256 rays grad_exchange="auto" would pick the single all-reduce)
    tr = NeRFTrainer(cfg.pipeline, precision="fp32", device="cuda:0", n_rays=256, runner_cfg=cfg.runner, seed=42,
                     grad_exchange="bucketed")
    local = []
    orig = parallel.allreduce_sum_async

    def spy(bucket):  # the exchange's buckets (coarse slice, then fine slice) before the reduction
        local.append(bucket.detach().cpu().clone())
        return orig(bucket)

    parallel.allreduce_sum_async = spy
    g = torch.Generator().manual_seed(100 + rank)
    img = torch.rand(1, 800, 800, 3, generator=g).to("cuda:0")
    out = []
    for k in range(3):
        pose = torch.from_numpy(synthetic_pose(20.0 * k + 90.0 * rank, -30.0, 4.0)).float()[None].to("cuda:0")
        tr.step(pose, torch.tensor([1111.111], device="cuda:0"), img)
        torch.cuda.synchronize()
        assert len(local) == 2 * (k + 1)  # two buckets per step, one per model, in flat-buffer order
        out.append(dict(local=torch.cat(local[-2:]), reduced=tr.flat.grad.detach().cpu().clone(),
                        params=tr.flat.data.detach().cpu().clone(), xys=tr.xys.detach().cpu().clone(), lr=tr.lr))
    parallel.allreduce_sum_async = orig
    q.put(_by_value((rank, out)))
    parallel.barrier()
    torch.distributed.destroy_process_group()


def test_trainer_gradient_exchange_two_ranks():
    """configs[2]'s exchange on the fused path (scripts/run.py:162-166 DDP semantics): per step, the exchanged gradient
    is the mean of the ranks' local gradients (bit for bit), the parameters stay identical on every rank, the ranks
    sample different pixels (Philox keyed by seed + rank, run.py:70-71), and the learning rate is the linearly scaled
    schedule (run.py:152-156). The exchange runs as two buckets (coarse model, then fine model), the coarse one
    overlapped with the fine MLP's backward."""
    from yanerf_amd.lr_schedule import lr_at
    from yanerf_amd.utils.config import Config
    import yanerf_boot
    runner = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml")).runner
    res = _spawn(_trainer_worker, 2)
    (_, a), (_, b) = res
    for k in range(3):
        mean = (a[k]["local"] + b[k]["local"]) / 2
        assert torch.equal(a[k]["reduced"], mean) and torch.equal(b[k]["reduced"], mean), k
        assert not torch.equal(a[k]["local"], b[k]["local"])
        assert torch.equal(a[k]["params"], b[k]["params"]), k
        assert not torch.equal(a[k]["xys"], b[k]["xys"])
        assert a[k]["lr"] == lr_at(runner, k, world_size=2) == b[k]["lr"]


def _exchange_worker(rank, world, port, q, precision):
    """Three fused training steps per rank under each gradient exchange ("bucketed": one all-reduce per model, the
    coarse one overlapped with the fine backward; "single": one all-reduce of the whole flat gradient after both
    backwards), from the same seed and rank-specific images; records the parameters and Adam moments after the steps."""
    _init_worker(rank, world, port)
    from scene import synthetic_pose
    from yanerf_amd import parallel
    from yanerf_amd.train import NeRFTrainer
    from yanerf_amd.utils.config import Config
    import yanerf_boot
    cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml"))
    g = torch.Generator().manual_seed(200 + rank)
    img = torch.rand(1, 800, 800, 3, generator=g).to("cuda:0")
    out = {}
    # (bf16 defaults to the "early" schedule: the coarse backward and its bucket's all-reduce on the side stream beside
    # the fine forward; "bucketed_serial" is the same exchange with the serial backward)
    for name, exch, overlap in (("bucketed", "bucketed", None), ("single", "single", None),
                                ("bucketed_serial", "bucketed", False)):
        tr = NeRFTrainer(cfg.pipeline, precision=precision, device="cuda:0", n_rays=256, runner_cfg=cfg.runner,
                         seed=42, grad_exchange=exch, overlap=overlap)
        for k in range(3):
            pose = torch.from_numpy(synthetic_pose(25.0 * k + 90.0 * rank, -30.0, 4.0)).float()[None].to("cuda:0")
            tr.step(pose, torch.tensor([1111.111], device="cuda:0"), img)
        torch.cuda.synchronize()
        out[name] = dict(params=tr.flat.data.detach().cpu().clone(), m=tr.exp_avg.detach().cpu().clone(),
                         v=tr.exp_avg_sq.detach().cpu().clone(), overlap=tr.overlap)
        del tr
    q.put(_by_value((rank, out)))
    parallel.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_bucketed_and_single_exchange_give_identical_parameters(precision):
    """configs[2]'s exchange (scripts/run.py:162-166 DDP semantics) in both of the trainer's schedules: after three
    steps on two ranks the bucketed (overlapped) and the single all-reduce give bit-identical parameters and Adam
    moments, on both ranks, in fp32 and bf16 -- the bucketing changes when the sums run, not what they sum. bf16 runs
    its default "early" schedule at world 2 (coarse backward + coarse bucket on the side stream beside the fine forward),
    checked against the serial bucketed schedule as well."""
    res = _spawn(_exchange_worker, 2, extra=(precision,))
    (_, a), (_, b) = res
    assert a["bucketed"]["overlap"] == ("early" if precision == "bf16" else False)
    for key in ("params", "m", "v"):
        for other in ("single", "bucketed_serial"):
            assert torch.equal(a["bucketed"][key], a[other][key]), (key, other)
            assert torch.equal(b["bucketed"][key], b[other][key]), (key, other)
        assert torch.equal(a["bucketed"][key], b["bucketed"][key]), key


def _rccl_world1_worker(rank, world, port, q):
    """RCCL on the hardware at world size 1 (the box has one card; RCCL refuses two ranks on one device): the
    communicator set up as parallel.init_distributed does for "nccl" (device_id bound), then the trainer's bucket
    pattern -- an async all-reduce started right after a kernel that produced the bucket, a second kernel queued behind
    it on the compute stream, the wait, the divide -- checked for stream ordering: the collective must see the first
    kernel's output and the second kernel must not be blocked on, or corrupted by, the collective."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group(backend="nccl", device_id=torch.device("cuda", 0))
    out = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    g = torch.Generator(device="cuda:0").manual_seed(1)
    a = torch.randn(4096, 4096, device="cuda:0", generator=g)
    bucket = torch.empty(595_844, device="cuda:0")
    ref = None
    for it in range(3):
        torch.mul(a.view(-1)[it:it + 595_844], 2.0 + it, out=bucket)  # the producer kernel of the bucket
        ref = bucket.clone()
        h = dist.all_reduce(bucket, op=dist.ReduceOp.SUM, async_op=True)
        c = a @ a  # compute queued behind the collective's start (the fine backward's place)
        h.wait()
        bucket.div_(dist.get_world_size())
        torch.cuda.synchronize()
        out[f"equal_{it}"] = bool(torch.equal(bucket, ref))
        out[f"compute_ok_{it}"] = bool(torch.isfinite(c).all())
    q.put(_by_value((0, out)))
    dist.destroy_process_group()


def test_rccl_world1_bucket_ordering():
    """The "nccl" (RCCL) backend actually runs on the MI355X box at world size 1: process-group init with a bound
    device and the trainer's async-bucket / wait / divide ordering against kernels on the compute stream. (Multi-rank
    RCCL over xGMI needs a multi-card box: the driver's N-GPU bench runs it.)"""
    (_, out), = _spawn(_rccl_world1_worker, 1)
    assert out["backend"] == "nccl" and out["world"] == 1
    for it in range(3):
        assert out[f"equal_{it}"] and out[f"compute_ok_{it}"], out


def _ddp_worker(rank, world, port, q, golden_dir):
    """The drop-in path as scripts/run.py:162-166 runs it: the registry NeRFPipeline wrapped in
    DistributedDataParallel(find_unused_parameters=True); one step on rank-specific data with injected draws, and the
    same step without DDP for the local gradient."""
    _init_worker(rank, world, port)
    from yanerf_amd import ops
    from yanerf_amd.pipelines import PIPELINES
    from yanerf_amd.pipelines.utils import EvaluationMode
    from yanerf_amd.utils.config import Config
    import yanerf_boot
    cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml")).pipeline
    cfg.ray_sampler.n_rays_per_image_sampled_from_mask = 64
    torch.manual_seed(42)  # the same initial weights on every rank (DDP also broadcasts rank 0's)
    pipe = PIPELINES.build(cfg).to("cuda:0")
    ddp = torch.nn.parallel.DistributedDataParallel(pipe, find_unused_parameters=True)
    g = torch.Generator().manual_seed(10 + rank)
    R, Pc, Pn = 64, 64, 128
    draws = dict(pixel_ids=torch.randperm(800 * 800, generator=g)[:R][None].to("cuda:0"),
                 jitter_u=torch.rand(1, R, Pc, generator=g).to("cuda:0"),
                 noise=[torch.randn(R, Pc, generator=g).to("cuda:0"), torch.randn(R, Pc + Pn, generator=g).to("cuda:0")],
                 pdf_u=torch.rand(R, Pn, generator=g).to("cuda:0"))
    from scene import synthetic_pose
    pose = torch.from_numpy(synthetic_pose(45.0 * rank, -30.0, 4.0)).float()[None].to("cuda:0")
    focal = torch.tensor([1111.111], device="cuda:0")
    img = torch.rand(1, 800, 800, 3, generator=g).to("cuda:0")
    ddp.train()

    def run(model):
        model.zero_grad(set_to_none=True)
        with ops.injected_randomness(**{k: (list(v) if isinstance(v, list) else v) for k, v in draws.items()}):
            preds = model(poses=pose, focal_lengths=focal, image_rgb=img, evaluation_mode=EvaluationMode.TRAINING)
        preds["objective"].mean().backward()
        torch.cuda.synchronize()
        return torch.cat([p.grad.detach().reshape(-1).cpu() if p.grad is not None else torch.zeros(p.numel())
                          for p in pipe.parameters()])

    reduced = run(ddp)
    local = run(pipe)
    q.put(_by_value((rank, local, reduced)))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_ddp_registry_pipeline_two_ranks():
    res = _spawn(_ddp_worker, 2, extra=("",))
    (_, la, ra), (_, lb, rb) = res
    mean = (la + lb) / 2
    assert not torch.equal(la, lb)
    assert torch.equal(ra, rb)
    np.testing.assert_allclose(ra.numpy(), mean.numpy(), rtol=0, atol=1e-7 * float(mean.abs().max()))


@pytest.mark.gpu
def test_bench_two_ranks_one_card_reports_distributed_fields():
    """The real bench (fused training step, RCCL replaced by gloo because two ranks share the one card of a test box)
    under torch.distributed.run with 2 ranks: the N-rank line has the process group's backend and world size, both
    ranks' ms/step and the exposed gradient exchange (HIP events around the wait), and value = both ranks' rays / the
    max-over-ranks time. Not a measurement (the ranks share one GPU). Launched as the driver launches it: the plain
    `python bench.py --gpus 2`, which starts its two ranks itself (no torch.distributed.run on the command line)."""
    import json

    from test_parallel import _run_bench_plain
    r = _run_bench_plain(["--gpus", "2", "--steps", "3", "--warmup", "1", "--psnr-steps", "0", "--secondary", "none",
                          "--no-extras", "--no-cpu-baseline", "--rays", "1024"], timeout=600,
                         env={"YANERF_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0 prints ONE JSON line
    d = json.loads(lines[0])
    info = d["distributed"]
    assert d["n_gpus"] == 2 and info["backend"] == "gloo" and info["world_size"] == 2
    assert len(info["ms_per_step_per_rank"]) == 2 and all(v > 0 for v in info["ms_per_step_per_rank"])
    assert info["allreduce_exposed_ms_max"] >= 0.0
    np.testing.assert_allclose(d["value"], 2 * 1024 * 3 / (d["ms_per_step"] * 3 / 1e3), rtol=1e-3)
