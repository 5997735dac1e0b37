"""Data-parallel plumbing over torch.distributed with the gloo backend on CPU, world_size 2 (the GPU runs use
the same code over RCCL): flat-buffer gradient all-reduce (DDP mean), parameter broadcast, metric all_gather,
max-over-ranks timing, ray/image sharding."""
import os
import socket

import torch
import torch.multiprocessing as mp
from mp_util import _as_tensors, _by_value

import yanerf_boot  # noqa: F401


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from yanerf_amd import parallel
    r, w, _ = parallel.init_distributed(backend="gloo")
    assert (r, w) == (rank, world)
    torch.manual_seed(100 + rank)  # different init per rank
    lin = [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(7))]
    fp = parallel.FlatParams(lin)
    parallel.broadcast_(fp.data)
    fp.grad.copy_(torch.arange(fp.numel, dtype=torch.float32) * (rank + 1))
    parallel.allreduce_mean_(fp.grad)
    # the trainer's bucketed exchange: two async sums on slices of one flat buffer, then the mean
    b = torch.arange(12, dtype=torch.float32) * (rank + 1)
    h0 = parallel.allreduce_sum_async(b[:5])
    h1 = parallel.allreduce_sum_async(b[5:])
    parallel.finish_allreduce(h0)
    parallel.finish_allreduce(h1)
    b.div_(world)
    m = parallel.allgather_cat(torch.tensor([float(rank)]))
    mx = parallel.max_over_ranks(float(rank) + 0.5)
    shards = [list(parallel.shard_range(10, k, world)) for k in range(world)]
    q.put(_by_value((rank, fp.data.clone(), lin[0].grad.clone(), m, mx, shards, b)))
    parallel.barrier()
    torch.distributed.destroy_process_group()


def test_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([_as_tensors(q.get(timeout=120)) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, d0, g0, m0, x0, s0, b0), (_, d1, g1, m1, x1, s1, b1) = res
    assert torch.equal(b0, torch.arange(12, dtype=torch.float32) * 1.5) and torch.equal(b0, b1)
    assert torch.equal(d0, d1)  # broadcast from rank 0
    expect = torch.arange(15, dtype=torch.float32).view(5, 3) * 1.5  # mean of x1 and x2
    assert torch.allclose(g0, expect) and torch.allclose(g1, expect)
    assert torch.equal(m0, torch.tensor([0.0, 1.0])) and x0 == x1 == 1.5
    assert sorted(sum(s0, [])) == list(range(10))


def _eval_worker(rank, world, port, q):
    """Sharded evaluation plumbing: DistributedSampler split + per-iteration all_gather restores dataset order and
    drops the padding (apis.py:173-177, 201); row shards of an image reassemble it exactly."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from yanerf_amd import parallel
    parallel.init_distributed(backend="gloo")
    n = 7  # not a multiple of the world size: the reference's sampler pads with the head of the list
    per_image = torch.arange(n, dtype=torch.float32) * 0.5 + 1.0
    got = [parallel.allgather_cat(per_image[i].view(1, 1)) for i in parallel.eval_order(n, rank, world)]
    gathered = torch.cat(got, dim=0)[:n].view(-1)
    H, W = 11, 5
    img = torch.arange(H * W * 3, dtype=torch.float32).view(H, W, 3)
    rows = parallel.shard_range(H, rank, world)
    full = parallel.gather_rows(img[rows.start:rows.stop].clone(), H)
    q.put(_by_value((rank, gathered, full, parallel.world_rank())))
    parallel.barrier()
    torch.distributed.destroy_process_group()


def test_gloo_world3_sharded_eval():
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_eval_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([_as_tensors(q.get(timeout=120)) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = torch.arange(7, dtype=torch.float32) * 0.5 + 1.0
    img = torch.arange(11 * 5 * 3, dtype=torch.float32).view(11, 5, 3)
    for rank, gathered, full, wr in res:
        assert wr == (3, rank)
        assert torch.equal(gathered, expect)
        assert torch.equal(full, img)


def test_eval_order_matches_distributed_sampler():
    from torch.utils.data import DistributedSampler

    from yanerf_amd import parallel
    for n in (1, 5, 8, 13):
        for world in (1, 2, 3, 8):
            for rank in range(world):
                ref = list(DistributedSampler(range(n), num_replicas=world, rank=rank, shuffle=False))
                assert parallel.eval_order(n, rank, world) == ref


def _run_bench_dist(extra, nproc=2, timeout=300, env=None):
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(root / "bench.py"),
           "--gpus", str(nproc)] + extra
    e = dict(os.environ, **(env or {}))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0 prints ONE JSON line
    return json.loads(lines[0])


def test_bench_distributed_fields_gloo_world2():
    """bench.py under torch.distributed.run with two CPU ranks over gloo (--dist-selftest: the N-rank plumbing, no
    GPU work): the line carries the backend and world size the process group reports, every rank's ms/step and the
    exposed exchange time, and the two-bucket exchange averages the ranks' gradients."""
    d = _run_bench_dist(["--steps", "3", "--dist-selftest"])
    info = d["distributed"]
    assert d["n_gpus"] == 2 and info["backend"] == "gloo" and info["world_size"] == 2
    assert len(info["ms_per_step_per_rank"]) == 2 and info["ms_per_step_min"] <= info["ms_per_step_max"]
    assert len(info["allreduce_exposed_ms_per_rank"]) == 2 and info["allreduce_exposed_ms_max"] >= 0
    assert info["grad_exchange"] == "bucketed" and info["grad_bytes"] == 4 * 1_191_688
    assert info["selftest_grad_ok"]


def _run_bench_plain(extra, timeout=300, env=None):
    """`python bench.py EXTRA` with no launcher (and no launcher variables in the environment)."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = dict({k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}, **(env or {}))
    r = subprocess.run([sys.executable, str(root / "bench.py")] + extra, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd="/tmp")
    return r


def test_bench_gpus_n_starts_its_own_ranks():
    """`python bench.py --gpus 2` with NO launcher starts two ranks itself (a child torch.distributed.run, before any
    GPU call) and rank 0's line reports the two-rank group: an N-GPU invocation never degrades to a world-1 line
    (reference launch: scripts/run.py:162-166)."""
    import json
    r = _run_bench_plain(["--gpus", "2", "--steps", "2", "--dist-selftest"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["distributed"]["world_size"] == 2 and d["distributed"]["selftest_grad_ok"]


def test_bench_world_size_mismatch_fails():
    """A launcher that started another number of ranks than --gpus asks for is an error, not a warning."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--dist-selftest"],
                       capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
