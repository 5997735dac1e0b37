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
    q.put((rank, f.cpu(), c.cpu(), d.cpu(), ev))
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
                res.append(q.get(timeout=2))
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
