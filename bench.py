#!/usr/bin/env python
"""Benchmark: NeRF training-step throughput (rays/s) on Lego 800x800, 64 coarse + 128 fine samples
(BASELINE.json configs[1]; configs[2] at N GPUs), MI355X HIP path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--precision fp32|bf16|fp32x3] [--rays 4096]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

`python bench.py --gpus N` with N > 1 and no launcher (no WORLD_SIZE in the environment) starts the N ranks itself:
before anything touches the GPU it runs the second form above as a CHILD process (never an exec) and exits with its
status, so an N-GPU invocation never degrades to a world-1 line (reference launch: scripts/run.py:162-166,
runners/utils.py:216-238). Under a launcher, a WORLD_SIZE that differs from --gpus is an error (exit 2).

A step = one rank's training step on one synthetic 800x800 image (4096 rays, 64 + (64+128) points per ray):
raygen -> coarse MLP -> composite -> refine -> fine MLP -> composite -> loss -> backward (both MLPs) ->
RCCL gradient all-reduce (two buckets, the coarse one overlapped with the fine MLP backward) -> Adam. Inputs (target image, poses) are resident in HBM before timing; weights are
random-init of the Lego architecture; targets are synthetic (no dataset in this environment). Weak scaling:
every rank runs its own 4096-ray step, value = total rays of all ranks / max-over-ranks time.

Rank 0 prints ONE JSON line (contract in the task statement), with `roofline` for the dominant kernel by time
(the fine pass's three MLP kernels, each timed alone with HIP events on its launch stream; `roofline_kernels` has all
three) and `cpu_baseline` (the CPU oracle's training step on a bounded sample, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv) -> int:
    """`--gpus N` (N > 1) without a launcher: run this script under torch.distributed.run with N local ranks as a
    child process and return its exit status (non-zero when any rank fails to start or dies: torch.distributed.run
    tears the group down then). Called before torch is imported, so this process never initialises the GPU."""
    import subprocess
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    n = pre.parse_known_args(argv)[0].gpus
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve()), *argv]
    print(f"[bench] --gpus {n} without a launcher: starting {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def _needs_launch(argv) -> bool:
    if "WORLD_SIZE" in os.environ:
        return False
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    return pre.parse_known_args(argv)[0].gpus > 1


if __name__ == "__main__" and _needs_launch(sys.argv[1:]):
    sys.exit(launch_ranks(sys.argv[1:]))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import yanerf_boot  # noqa: E402,F401
from yanerf_amd import parallel  # noqa: E402
from yanerf_amd.train import NeRFTrainer  # noqa: E402
from yanerf_amd.utils.config import Config  # noqa: E402

METRIC = "rays/sec (train step) + PSNR, Lego 800×800 64c+128f, 1/2/4/8 MI355X"
MAC_PER_POINT = 589_952  # 63*256 + 4*256^2 + 319*256 + 2*256^2 + 256^2 + 256 + 256*128 + 128*3
MAC_PER_RAY_PASS = 27 * 128  # LinearWithRepeat direction term, once per ray per pass
# MI355X dense matrix peaks (MI355X_MICROARCH.md); fp32x3 runs six bf16 MFMAs per fp32 product, so its ceiling
# for fp32 work is the bf16 peak / 6
PEAK_TFLOPS = {"fp32": 157.3, "bf16": 2500.0, "fp32x3": 2500.0 / 6, "bf16s": 2500.0}
PEAK_FP8_TFLOPS = 5000.0  # block-scaled fp8 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4, e4m3): 2x the bf16 rate, dense
# The bf16 mode's weight-gradient kernel runs its fp8 x fp8 tiles (fp8 saved activations x fp8 gradient rows) on the
# block-scaled fp8 MFMA and the rest (the bf16 PE / dirPE columns, the bf16 dU rows) on the bf16 MFMA. Algorithmic
# dW MACs per point by instruction (csrc/mlp.hip dw_tile_pm / use_f8mma): fp8 = 7 trunk layers' 256 x 256 H columns +
# intermediate 256 x 256 + colour layer 128 x 256 (Y); bf16 = layer 0's and the skip layer's 256 x 63 PE columns +
# colour 128 x 27 (dirPE) + density 1 x 256 + colour output 3 x 128.
DW_MAC_FP8 = 7 * 256 * 256 + 256 * 256 + 128 * 256
DW_MAC_BF16 = 2 * 256 * 63 + 128 * 27 + 256 + 3 * 128


def bf16_dw_instruction_peak() -> float:
    """The MFMA peak the bf16 mode's dW kernel can reach with the instructions it issues (TFLOP/s): its FLOPs over
    the ideal time of the fp8 part at the fp8 rate plus the bf16 part at the bf16 rate."""
    tot = DW_MAC_FP8 + DW_MAC_BF16
    return tot / (DW_MAC_FP8 / PEAK_FP8_TFLOPS + DW_MAC_BF16 / PEAK_TFLOPS["bf16"])


def synthetic_pose(theta, phi, radius=4.0):
    """Camera on a sphere, Blender c2w convention + the reference's flip diag(1,-1,-1,1)
    (blender_dataset.py:58-60, 69)."""
    def tr(t):
        return np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, t], [0, 0, 0, 1]], np.float64)

    def rphi(p):
        c, s = math.cos(p), math.sin(p)
        return np.array([[1, 0, 0, 0], [0, c, -s, 0], [0, s, c, 0], [0, 0, 0, 1]], np.float64)

    def rth(t):
        c, s = math.cos(t), math.sin(t)
        return np.array([[c, 0, -s, 0], [0, 1, 0, 0], [s, 0, c, 0], [0, 0, 0, 1]], np.float64)

    c2w = rth(math.radians(theta)) @ rphi(math.radians(phi)) @ tr(radius)
    c2w = np.array([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], np.float64) @ c2w
    return (c2w @ np.diag([1.0, -1.0, -1.0, 1.0]))[:3, :4].astype(np.float32)


# algorithmic MACs per point of the input-gradient walk (mlp_bwd_dx_kernel): every layer's input gradient except layer
# 0's (the embedding carries no gradient): trunk l1..l7 over their 256 hidden inputs, intermediate 256x256, density
# 256, colour layer over its 256 feature inputs, output 3x128
MAC_PER_POINT_DX = 8 * 256 * 256 + 256 + 128 * 256 + 3 * 128
# HBM-bound kernel ceilings are not used here: the three MLP kernels are priced against the MFMA peak of their mode


def kernel_flops(kind: str, R: int, P: int) -> float:
    """Algorithmic FLOPs of one launch of an MLP kernel over R rays x P points."""
    if kind == "dx":
        return 2.0 * MAC_PER_POINT_DX * R * P
    return 2.0 * (MAC_PER_POINT * R * P + MAC_PER_RAY_PASS * R)  # forward and weight gradients


def pmc_traffic(kind: str, precision: str):
    """HBM bytes per fine launch from the committed PMC summary (tools/pmc_summary.py over separate FETCH_SIZE /
    WRITE_SIZE passes), reported only when that file was collected on the kernel sources this run loaded (its build id
    equals the library's); a stale file gives traffic null and says so in traffic_source."""
    from yanerf_amd import _C
    pmc = ROOT / "profiles" / f"pmc_mlp_{kind}_{precision}.json"
    src = {"file": str(pmc.relative_to(ROOT)), "build_id": None, "library_build_id": _C.lib().yanerf_build_id().decode()}
    if not pmc.exists():
        src["status"] = "missing"
        return None, src
    try:
        d = json.loads(pmc.read_text())
    except Exception:
        src["status"] = "unreadable"
        return None, src
    src["build_id"] = d.get("build_id")
    if src["build_id"] != src["library_build_id"]:
        src["status"] = "stale (collected on other kernel sources)"
        return None, src
    src["status"] = "current"
    return d.get("hbm_bytes_per_launch"), src


def kernel_rooflines(tr, poses, focal, image, precision: str, steps: int = 4, live=None):
    """Per-kernel HIP-event timings of the fine pass's three MLP kernels (forward, dX walk, dW), each alone on the
    stream. `live` = the event timings taken inside the timed steps (the forwards always; in the serial-backward modes,
    fp32 and fp32x3, the dX and dW launches too): a kernel timed there is priced on that average ("timing": "timed
    steps"). The others come from a few steps in the trainer's probe mode after the timed region, which serialises the
    backward (dX, dW, slab reduce per pass; coarse after fine), so no kernel shares the GPU while it is timed
    ("timing": "probe steps"). Returns {kernel: roofline dict}, the dominant kernel by time, the probe-step timings."""
    tr.kernel_probes = True
    names = ["mlp_fwd_1", "mlp_dx_1", "mlp_dw_1", "mlp_reduce_1", "mlp_fwd_0", "mlp_dx_0", "mlp_dw_0", "mlp_reduce_0"]
    tr.enable_probes(names)
    for i in range(steps):
        tr.step(poses[i % len(poses)][None], focal, image)
    torch.cuda.synchronize()
    ms = tr.probe_ms()
    tr.kernel_probes = False
    tr.events = None
    R, Pf = tr.R, tr.Pf
    peak = PEAK_TFLOPS[precision]
    out = {}
    live = live or {}
    for kind, kname in (("fwd", "mlp_fwd_kernel"), ("dx", "mlp_bwd_dx_kernel"), ("dw", "mlp_dw_kernel")):
        how = "timed steps" if f"mlp_{kind}_1" in live else "probe steps"
        t_ms = live.get(f"mlp_{kind}_1", ms.get(f"mlp_{kind}_1", float("nan")))
        fl = kernel_flops(kind, R, Pf)
        ach = fl / (t_ms * 1e-3) / 1e12
        traffic, source = pmc_traffic(kind, precision)
        out[kind] = {"bound": "mfma", "kernel": f"{kname} (fine pass)", "achieved": round(ach, 2), "peak": peak,
                     "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": traffic, "traffic_source": source,
                     "flops_per_launch": fl, "avg_launch_ms": round(t_ms, 4), "timing": how}
        if precision == "bf16" and kind == "dw":
            # priced against the peak of the MFMAs it issues (94 % of its FLOPs on the 2x-rate fp8 MFMA), with the
            # bf16-peak figure above kept beside it
            pk = bf16_dw_instruction_peak()
            out[kind].update({"peak_bf16": peak, "frac_bf16_peak": round(ach / peak, 4), "peak": round(pk, 1),
                              "frac": round(ach / pk, 4), "peak_basis": (
                                  "instruction-matched: fp8 x fp8 tiles on v_mfma_scale_f32_32x32x64_f8f6f4 (5 PF "
                                  "dense), bf16 tiles on the bf16 MFMA (2.5 PF), weighted by their algorithmic FLOPs")})
    dom = max(out, key=lambda k: out[k]["avg_launch_ms"])
    serial_ms = {k: round(v, 4) for k, v in ms.items()}
    return out, dom, serial_ms


def train_flops_per_ray(pc: int, pf: int) -> float:
    fwd = 2.0 * (MAC_PER_POINT * (pc + pf) + 2 * MAC_PER_RAY_PASS)
    return 3.0 * fwd  # forward + input-gradient chain + weight gradients


def cpu_baseline(precision_cfg, n_pts_c: int, n_pts_f_new: int, budget_s: float = 12.0):
    """The CPU oracle (numpy restatement, tests' checker) timed on a bounded sample of the same workload."""
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    from oracle import nerf_oracle as O  # noqa: E402  (cpu_baseline leg only)
    from weights import LEGO_ARCH, make_nerf_mlp_params  # noqa: E402
    threads = int(os.environ.get("YANERF_CPU_THREADS", min(16, os.cpu_count() or 1)))
    try:
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(threads)
    except Exception:  # pragma: no cover
        limiter = None
    arch = O.MLPArch.from_dict(LEGO_ARCH)
    pc, pf = make_nerf_mlp_params(LEGO_ARCH, 1), make_nerf_mlp_params(LEGO_ARCH, 2)
    cfg = O.RenderCfg(n_pts_coarse=n_pts_c, n_pts_fine=n_pts_f_new, density_noise_std=0.2,
                      raymarch=O.RaymarchOpts(background_density_bias=1e-6))
    rng = np.random.default_rng(0)
    R = 256
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        o = np.tile([[0.0, 0.0, 4.0]], (R, 1)).astype(np.float32)
        d = (rng.standard_normal((R, 3)) * 0.3 + [0, 0, -1]).astype(np.float32)
        z = O.jiggle_within_stratas(np.broadcast_to(O.torch_linspace(2, 6, n_pts_c), (R, n_pts_c)).copy(),
                                    rng.random((R, n_pts_c)).astype(np.float32))
        O.train_step_grads(pc, pf, arch, cfg, o, d, z, rng.random((R, 3)).astype(np.float32),
                           (rng.standard_normal((R, n_pts_c)) * 0.2).astype(np.float32),
                           (rng.standard_normal((R, n_pts_c + n_pts_f_new)) * 0.2).astype(np.float32),
                           rng.random((R, n_pts_f_new)).astype(np.float32))
        done += R
    dt = time.perf_counter() - t0
    if limiter is not None:
        limiter.unregister()
    return {"value": round(done / dt, 2), "unit": "rays/s", "cores": threads, "kind": "port",
            "what": "oracle/nerf_oracle.py: this repo's numpy restatement of the reference's training step, NOT the "
                    "reference itself (which cannot run on the GPU box)",
            "sample": f"{done} rays of the Lego 64+{n_pts_f_new} training step (fwd+bwd both MLPs, no optimizer) "
                      f"in batches of {R}, numpy fp32 oracle, {dt:.1f} s"}


# The reference's own CPU path (scripts/run.py --device cpu, torch 2.10 CPU, Lego 64 + 128, 4096 rays), timed in the
# build container on 8 Xeon cores: 330-390 train rays/s. It is not re-timed here (the
# reference does not exist on the GPU box); stated beside the port so the ratio against the reference is visible.
REFERENCE_CPU = {"value": 360.0, "range": [330.0, 390.0], "unit": "rays/s", "cores": 8, "kind": "reference",
                 "where": "build container, SURVEY.md §6 (not the GPU box)",
                 "sample": "reference scripts/run.py --device cpu training steps, Lego 64+128, 4096 rays"}


def extras(pcfg, cfg, dev, poses, focal, image, precision, others=()):
    """Secondary timings (not the headline): (1) full 800x800 evaluation render through the registry
    NeRFPipeline (no_grad, the reference's 131072-point chunking), (2) one training step through the drop-in
    path: registry NeRFPipeline + torch autograd + torch.optim.Adam, i.e. what scripts/run.py would run."""
    import copy

    from yanerf_amd.pipelines import PIPELINES
    from yanerf_amd.pipelines.utils import EvaluationMode
    out = {}
    c = copy.deepcopy(pcfg)
    c.model.precision = precision
    pipe = PIPELINES.build(c).to(dev)
    pipe.eval()
    H = W = 800
    with torch.no_grad():
        pipe(poses=poses[:1], focal_lengths=focal, image_height=64, image_width=64,
             evaluation_mode=EvaluationMode.EVALUATION)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pred = pipe(poses=poses[1:2], focal_lengths=focal, image_rgb=image, evaluation_mode=EvaluationMode.EVALUATION)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    out["eval_render"] = {"rays_per_s": round(H * W / dt, 1), "s_per_image": round(dt, 3),
                          "psnr_vs_synthetic": round(-10 * math.log10(float(pred["loss_rgb_mse"].mean())), 3),
                          "chunk_size_grid": int(c.chunk_size_grid), "precision": precision}
    # the same full-image evaluation on the fused inference path (NeRFTrainer.render: 65,536-ray chunks, no autograd,
    # no per-chunk Python pipeline): 10 chunks per image instead of 313
    tr = NeRFTrainer(pcfg, precision=precision, device=dev, n_rays=256)
    tr.render(poses[:1], focal, 64, 64)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.render(poses[1:2], focal, H, W)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out["eval_render_fused"] = {"rays_per_s": round(H * W / dt, 1), "s_per_image": round(dt, 3),
                                "chunk_rays": 65536, "precision": precision}
    # the same render as one HIP-graph launch per image (NeRFTrainer.render_graph, bitwise equal)
    tr.render_graph(poses[:1], focal, H, W)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.render_graph(poses[1:2], focal, H, W)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out["eval_render_graph"] = {"rays_per_s": round(H * W / dt, 1), "s_per_image": round(dt, 3),
                                "launches_per_image": 1, "precision": precision}
    del tr
    # the fused evaluation render in every precision mode, with its whole-image MFMA utilisation (inference FLOPs:
    # 2 x (589,952 MAC/point x (Pc + Pc + Pf) points + 3,456 MAC/ray/pass x 2) per ray)
    Pc = int(pcfg.ray_sampler.n_pts_per_ray_evaluation)
    Pn = int(pcfg.renderer.n_pts_per_ray_fine_evaluation)
    inf_flops_ray = 2.0 * (MAC_PER_POINT * (Pc + Pc + Pn) + 2 * MAC_PER_RAY_PASS)
    out["eval_render_fused_by_precision"] = {}
    for p in (precision,) + tuple(others):
        tr = NeRFTrainer(pcfg, precision=p, device=dev, n_rays=256)
        tr.render(poses[:1], focal, 64, 64)
        torch.cuda.synchronize()
        best = float("inf")
        for rep in range(2):
            t0 = time.perf_counter()
            tr.render(poses[2 + rep:3 + rep], focal, H, W)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        rps = H * W / best
        out["eval_render_fused_by_precision"][p] = {
            "rays_per_s": round(rps, 1), "s_per_image": round(best, 4),
            "mfma_tflops": round(rps * inf_flops_ray / 1e12, 1),
            "mfma_frac": round(rps * inf_flops_ray / 1e12 / PEAK_TFLOPS[p], 4)}
        del tr
    pipe.train()
    opt = torch.optim.Adam(pipe.parameters(), lr=float(cfg.runner.init_lr))
    steps = 5
    for i in range(steps + 2):
        if i == 2:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        preds = pipe(poses=poses[i:i + 1], focal_lengths=focal, image_rgb=image,
                     evaluation_mode=EvaluationMode.TRAINING)
        opt.zero_grad(set_to_none=True)
        preds["objective"].mean().backward()
        opt.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    R = int(c.ray_sampler.n_rays_per_image_sampled_from_mask)
    out["dropin_train"] = {"rays_per_s": round(R / dt, 1), "ms_per_step": round(1e3 * dt, 3), "precision": precision,
                           "path": "registry NeRFPipeline + autograd + torch.optim.Adam"}
    # BASELINE configs[4] on one GPU: bf16, 64 coarse + 256 fine samples (64 + 320 = 384 points per ray), the same
    # fused training step (4096 rays), with its whole-step MFMA utilisation and the fine forward's roofline -- in both
    # bf16 storage modes: "bf16" (bf16 MFMA, fp8 e4m3 saved activations / gradient rows, dW on the fp8 MFMA; the
    # top-level fields) and "bf16s" (bf16 storage throughout, dW on the bf16 MFMA: the precision configs[4] names)
    import copy as _copy
    c4 = _copy.deepcopy(pcfg)
    c4.renderer.n_pts_per_ray_fine_training = 256
    c4.renderer.n_pts_per_ray_fine_evaluation = 256

    def lego256(prec):
        tr = NeRFTrainer(c4, precision=prec, device=dev)
        for i in range(3):
            tr.step(poses[i:i + 1], focal, image)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        steps4 = 10
        for i in range(steps4):
            tr.step(poses[(3 + i) % len(poses)][None], focal, image)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps4
        R4, Pc4, Pf4 = tr.R, tr.Pc, tr.Pf
        # the fine forward timed alone on the GPU: a few steps in the trainer's probe mode (serial backward; bf16's
        # default "early" schedule runs the coarse backward beside the fine forward in the steps timed above)
        tr.kernel_probes = True
        tr.enable_probes(["mlp_fwd_1"])
        for i in range(3):
            tr.step(poses[(13 + i) % len(poses)][None], focal, image)
        torch.cuda.synchronize()
        f4ms = tr.probe_ms().get("mlp_fwd_1", float("nan"))
        del tr
        fwd4 = 2.0 * (MAC_PER_POINT * R4 * Pf4 + MAC_PER_RAY_PASS * R4)
        return {"rays_per_s": round(R4 / dt, 1), "ms_per_step": round(1e3 * dt, 3), "pts_per_ray": Pc4 + Pf4,
                "step_mfma_frac": round(train_flops_per_ray(Pc4, Pf4) * R4 / dt / 1e12 / PEAK_TFLOPS["bf16"], 4),
                "fine_fwd_ms": round(f4ms, 4),
                "fine_fwd_mfma_frac": round(fwd4 / (f4ms * 1e-3) / 1e12 / PEAK_TFLOPS["bf16"], 4),
                "dtype": DTYPES[prec]}

    out["lego256_bf16_train"] = {
        "config": "BASELINE configs[4] at 1 GPU: 64 coarse + 256 fine (64 + 320 fine-pass points), bf16",
        **lego256("bf16"), "bf16s": lego256("bf16s")}
    # SURVEY §8(d)'s large-batch roofline variant: the same Lego 64 + 128 step at 16,384 and 65,536 rays per step (the
    # per-step fixed costs -- packs, ray generation, composites, refinement, reduces, Adam, launch gaps -- amortised
    # over 4-16x the MLP work), bf16's default schedule; fp32 at 16,384 rays
    out["lego_large_batch_train"] = {"config": "Lego 800x800, 64 + 128, one GPU, synthetic target"}
    for p, R_big in (("bf16", 16384), ("bf16", 65536), ("fp32", 16384)):
        tr = NeRFTrainer(pcfg, precision=p, device=dev, n_rays=R_big)
        for i in range(2):
            tr.step(poses[i:i + 1], focal, image)
        torch.cuda.synchronize()
        nst = 6
        t0 = time.perf_counter()
        for i in range(nst):
            tr.step(poses[(2 + i) % len(poses)][None], focal, image)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / nst
        out["lego_large_batch_train"][f"{p}_{R_big}"] = {
            "rays_per_step": R_big, "rays_per_s": round(R_big / dt, 1), "ms_per_step": round(1e3 * dt, 3),
            "step_mfma_frac": round(train_flops_per_ray(tr.Pc, tr.Pf) * R_big / dt / 1e12 / PEAK_TFLOPS[p], 4)}
        del tr
        torch.cuda.empty_cache()
    # the fused step captured as a HIP graph (NeRFTrainer.capture_step / replay_step: bit-equal to the eager step,
    # tests/test_gpu_trainer.py::test_graph_replayed_steps_equal_eager_steps), eager vs replayed ms per step
    out["graph_step"] = {}
    for p in dict.fromkeys(("bf16", precision)):
        tr = NeRFTrainer(pcfg, precision=p, device=dev, runner_cfg=cfg.runner, train_set_size=LEGO_TRAIN_IMAGES)
        for i in range(3):
            tr.step(poses[i:i + 1], focal, image)
        nst = 20
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(nst):
            tr.step(poses[(3 + i) % len(poses)][None], focal, image)
        torch.cuda.synchronize()
        eager_ms = 1e3 * (time.perf_counter() - t0) / nst
        # GRAPH_STEPS consecutive steps per graph (capture_step(n_steps=...)): each replay copies its poses in one
        # copy and launches one graph for all of them
        K = GRAPH_STEPS
        tr.capture_step(poses[0:K], focal, image, n_steps=K)
        tr.replay_step(poses[K:2 * K], focal)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(nst // K):
            tr.replay_step(poses[(K * i) % len(poses):(K * i) % len(poses) + K], focal)
        torch.cuda.synchronize()
        graph_ms = 1e3 * (time.perf_counter() - t0) / (K * (nst // K))
        out["graph_step"][p] = {"eager_ms_per_step": round(eager_ms, 4), "graph_ms_per_step": round(graph_ms, 4),
                                "graph_steps_per_launch": K,
                                "graph_rays_per_s": round(tr.R / graph_ms * 1e3, 1),
                                "step_mfma_frac_graph": round(train_flops_per_ray(tr.Pc, tr.Pf) * tr.R / (graph_ms * 1e-3)
                                                              / 1e12 / PEAK_TFLOPS[p], 4)}
        del tr
    # BASELINE configs[3] on one GPU: the Fern config (504 x 378, 1024 rays per step) at BASELINE's 64 + 128 samples,
    # LLFF-style per-image depth bounds (a [1, 2] tensor, averaged as ray_sampler.py:280-283 does), synthetic target.
    # Reference CPU path on 8 cores: 341 rays/s
    fcfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/fern.yml")).pipeline
    fcfg.renderer.n_pts_per_ray_fine_training = 128
    fcfg.renderer.n_pts_per_ray_fine_evaluation = 128
    fimg = torch.rand(1, 378, 504, 3, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    ffocal = torch.tensor([407.56], device=dev)
    bounds = torch.tensor([[1.3, 5.9]])  # host tensor (LLFF's bounds come from the loader on the host): no device sync
    out["fern_64_128_train"] = {"config": "BASELINE configs[3] at 1 GPU: Fern 504x378, 64 + 128, 1024 rays, "
                                          "per-image bounds", "reference_cpu_rays_per_s": 341.0}
    for p in ("fp32", "bf16"):
        tr = NeRFTrainer(fcfg, precision=p, device=dev)
        for i in range(3):
            tr.step(poses[i:i + 1], ffocal, fimg, near=bounds[:, :1], far=bounds[:, 1:])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        nst = 20
        for i in range(nst):
            tr.step(poses[(3 + i) % len(poses)][None], ffocal, fimg, near=bounds[:, :1], far=bounds[:, 1:])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / nst
        out["fern_64_128_train"][p] = {
            "rays_per_s": round(tr.R / dt, 1), "ms_per_step": round(1e3 * dt, 3),
            "step_mfma_frac": round(train_flops_per_ray(tr.Pc, tr.Pf) * tr.R / dt / 1e12 / PEAK_TFLOPS[p], 4)}
        # the same steps replayed as a HIP graph of GRAPH_STEPS steps per launch (a 1024-ray step is short, so the
        # launch and input copies weigh more); the captured steps read their per-image bounds from a static device
        # buffer (replay_step(near=, far=))
        K = GRAPH_STEPS
        tr.capture_step(poses[0:K], ffocal, fimg, near=bounds[:, :1], far=bounds[:, 1:], n_steps=K)
        tr.replay_step(poses[K:2 * K], ffocal, near=bounds[:, :1], far=bounds[:, 1:])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(nst // K):
            tr.replay_step(poses[(K * i) % len(poses):(K * i) % len(poses) + K], ffocal, near=bounds[:, :1],
                           far=bounds[:, 1:])
        torch.cuda.synchronize()
        dtg = (time.perf_counter() - t0) / (K * (nst // K))
        out["fern_64_128_train"][p].update(
            graph_rays_per_s=round(tr.R / dtg, 1), graph_ms_per_step=round(1e3 * dtg, 3),
            step_mfma_frac_graph=round(train_flops_per_ray(tr.Pc, tr.Pf) * tr.R / dtg / 1e12 / PEAK_TFLOPS[p], 4))
        del tr
    return out


def configs_at_n(pcfg, cfg, dev, poses, focal, image, world: int, steps: int = 10, warmup: int = 3):
    """At N > 1: BASELINE configs[3] (Fern 504x378, 64 + 128, 1024 rays per rank, per-image bounds) in fp32 and bf16,
    and configs[4] (Lego 800x800 bf16, 64 + 256) -- the same fused data-parallel step as the headline (weak scaling,
    two-bucket gradient all-reduce), each timed over `steps` steps between barrier + sync pairs, max over ranks, value
    = all ranks' rays / time. (At N = 1 the same workloads are in `extras`.)"""
    import copy as _copy

    def timed(tr, prec, pose_list, foc, img, **kw):
        for i in range(warmup):
            tr.step(pose_list[i % len(pose_list)][None], foc, img, **kw)
        parallel.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            tr.step(pose_list[(warmup + i) % len(pose_list)][None], foc, img, **kw)
        torch.cuda.synchronize()
        parallel.barrier()
        dt = parallel.max_over_ranks(time.perf_counter() - t0, device=dev)
        return {"rays_per_s": round(tr.R * world * steps / dt, 1), "ms_per_step": round(1e3 * dt / steps, 3),
                "step_mfma_frac": round(train_flops_per_ray(tr.Pc, tr.Pf) * tr.R * steps / dt / 1e12
                                        / PEAK_TFLOPS[prec], 4)}

    out = {}
    fcfg = Config.fromfile(str(yanerf_boot.PKG_DIR / "configs/nerf/fern.yml")).pipeline
    fcfg.renderer.n_pts_per_ray_fine_training = 128
    fcfg.renderer.n_pts_per_ray_fine_evaluation = 128
    fimg = torch.rand(1, 378, 504, 3, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    ffocal = torch.tensor([407.56], device=dev)
    bounds = torch.tensor([[1.3, 5.9]])
    out["fern_64_128_train"] = {"config": f"BASELINE configs[3] at {world} GPUs: Fern 504x378, 64 + 128, 1024 rays "
                                          "per rank, per-image bounds"}
    for p in ("fp32", "bf16"):
        tr = NeRFTrainer(fcfg, precision=p, device=dev)
        out["fern_64_128_train"][p] = timed(tr, p, poses, ffocal, fimg, near=bounds[:, :1], far=bounds[:, 1:])
        del tr
    c4 = _copy.deepcopy(pcfg)
    c4.renderer.n_pts_per_ray_fine_training = 256
    c4.renderer.n_pts_per_ray_fine_evaluation = 256
    out["lego256_bf16_train"] = {"config": f"BASELINE configs[4] at {world} GPUs: Lego 800x800 bf16, 64 + 256, 4096 "
                                           "rays per rank"}
    for p in ("bf16", "bf16s"):  # both bf16 storage modes (bf16s: bf16 throughout, the precision configs[4] names)
        tr = NeRFTrainer(c4, precision=p, device=dev, runner_cfg=cfg.runner, train_set_size=LEGO_TRAIN_IMAGES)
        r = timed(tr, p, poses, focal, image)
        if p == "bf16":
            out["lego256_bf16_train"].update(r)
        else:
            out["lego256_bf16_train"]["bf16s"] = r
        del tr
    return out


def psnr_leg(precision: str, steps: int, dev):
    """The `+ PSNR` half of the metric: the same fused training step (Lego config, 64 + 128, 4096 rays) trained on a
    procedural scene written in the nerf_synthetic format (tools/synthetic_scene.py: 40 train / 8 test views at
    100 x 100, read back through BlenderDataset into HBM), then scored as the reference's evaluation does (PSNR of the
    mean per-image MSE). No real dataset can be fetched here, so this is a synthetic-scene PSNR, not Lego's.

    Round 4: with the reference's initialisation (density-layer bias 0, nerf_mlp.py:69-71, whose own comment says
    "Sometimes this is not enough") this scene's training collapses to the transparent solution for seed 42 -- no
    density anywhere, each ray's colour painted on its background-opacity last sample (`rays_before_far_plane` 0,
    profiles/r4_density_collapse_probe.jsonl). The headline PSNR is therefore the run with the density-layer bias
    initialised to 1.0, which reconstructs the scene; the reference-init run and the bf16 run are reported beside it.
    Round 5: the reference itself, run in the build container on this scene at 50 x 50 (1,024 rays, 1,000 steps,
    profiles/r5_reference_collapse.jsonl), collapses from its own init (20.45 dB, 0 rays before the far plane) and
    reaches 33.95 dB from the bias-1.0 init; this build on the same runs: 20.48 / 33.90 dB (fp32), 33.81 dB (bf16)."""
    import tempfile
    sys.path.insert(0, str(ROOT / "tools"))
    from psnr_synthetic import run as psnr_run  # noqa: E402
    from synthetic_scene import write_scene  # noqa: E402
    with tempfile.TemporaryDirectory() as tmp:
        data = write_scene(Path(tmp) / "synthetic", 100, 40, 8, device=str(dev))
        r = psnr_run(data, precision, steps, dev, density_bias=1.0)
        r["reference_init_run"] = psnr_run(data, precision, steps, dev)
        if precision != "bf16":
            r["bf16_run"] = psnr_run(data, "bf16", steps, dev, density_bias=1.0)
    r["scene"] = "procedural blobs, 100x100, 40 train / 8 test views (synthetic, not Lego)"
    return r


def distributed_fields(dt_local: float, steps: int, exposed_ms, exchange: str, dev=None) -> dict:
    """What an N-rank line must show (SCALE runs): the process group's backend and size as the group itself reports
    them, every rank's own ms/step (min / max / all), and the exposed part of the gradient exchange per step (HIP
    events on the compute stream around the wait for the all-reduce; per rank, then max and mean over ranks).
    Reference: the DDP setup of scripts/run.py:162-166 and runners/utils.py:216-238."""
    import torch.distributed as dist
    ms = parallel.allgather_floats(1e3 * dt_local / steps, device=dev)
    ex = parallel.allgather_floats(float("nan") if exposed_ms is None else float(exposed_ms), device=dev)
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "grad_exchange": exchange,
            "ms_per_step_per_rank": [round(v, 4) for v in ms], "ms_per_step_min": round(min(ms), 4),
            "ms_per_step_max": round(max(ms), 4),
            "allreduce_exposed_ms_per_rank": [round(v, 4) for v in ex],
            "allreduce_exposed_ms_max": round(max(ex), 4), "allreduce_exposed_ms_mean": round(sum(ex) / len(ex), 4),
            "grad_bytes": 4 * 1_191_688}


def dist_selftest(steps: int) -> None:
    """`--dist-selftest`: the N-rank plumbing of this script without the GPU (CPU ranks over gloo under
    torch.distributed.run): the trainer's two-bucket exchange of the Lego-size flat gradient (1,191,688 fp32) timed
    for `steps` steps, then the same `distributed` fields the real run reports. Not a measurement of anything."""
    rank, world, _ = parallel.init_distributed(backend="gloo")
    n, n_coarse = 1_191_688, 595_844
    grad = torch.full((n,), float(rank + 1))
    parallel.barrier()
    t0 = time.perf_counter()
    ex = 0.0
    for _ in range(steps):
        h = parallel.allreduce_sum_async(grad[:n_coarse])
        h2 = parallel.allreduce_sum_async(grad[n_coarse:])
        t1 = time.perf_counter()
        parallel.finish_allreduce(h)
        parallel.finish_allreduce(h2)
        ex += time.perf_counter() - t1
        grad.div_(world)
    dt = time.perf_counter() - t0
    info = distributed_fields(dt, steps, 1e3 * ex / steps, "bucketed")
    expect = sum(range(1, world + 1)) / world  # the first step's mean; later steps average identical values
    info["selftest_grad_ok"] = bool(torch.allclose(grad, torch.full_like(grad, expect)))
    if rank == 0:
        print(json.dumps({"selftest": True, "n_gpus": world, "distributed": info}))
    parallel.barrier()
    torch.distributed.destroy_process_group()


DTYPES = {"fp32": "f32", "fp32x3": "f32 (3xbf16 split MFMA)",
          "bf16": "bf16 + fp8 (bf16 MFMA forward / dX; e4m3 saved activations and gradient rows; dW on the fp8 MFMA)",
          "bf16s": "bf16 (bf16 MFMA forward / dX / dW; bf16 saved activations and gradient rows)"}
LEGO_TRAIN_IMAGES = 100  # nerf_synthetic Lego's train split (the loader length scripts/run.py:243-271 converts with)
GRAPH_STEPS = 4  # training steps captured per HIP graph in the graph legs (NeRFTrainer.capture_step(n_steps=...))


def progress(msg: str) -> None:
    """A line on stderr per bench leg (rank 0): long runs keep writing, so a supervisor can tell them from a hang."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--precision", default=os.environ.get("YANERF_BENCH_PRECISION", "fp32"), choices=list(PEAK_TFLOPS))
    ap.add_argument("--rays", type=int, default=None, help="rays per rank per step (default: config, 4096)")
    ap.add_argument("--config", default=str(yanerf_boot.PKG_DIR / "configs/nerf/lego.yml"))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--secondary", default="fp32x3,bf16,bf16s",
                    help="comma list of other precisions to time on the same workload (reported under `secondary`)")
    ap.add_argument("--no-extras", action="store_true", help="skip the eval-render and drop-in-path timings")
    ap.add_argument("--psnr-steps", type=int, default=1000,
                    help="train this many steps on the procedural nerf_synthetic-format scene and report its test PSNR "
                         "(rank 0 at N=1; 0 = skip)")
    ap.add_argument("--dist-selftest", action="store_true",
                    help="CPU/gloo check of the N-rank plumbing and its JSON fields (no GPU work; not a benchmark)")
    args = ap.parse_args()
    env_world = parallel.env_rank_world()[1]
    if env_world != args.gpus:
        # never report an N-GPU run as some other world size
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks", file=sys.stderr)
        sys.exit(2)
    if args.dist_selftest:
        return dist_selftest(args.steps)
    backend = os.environ.get("YANERF_DIST_BACKEND") or "nccl"
    if env_world > 1 and backend == "nccl" and torch.cuda.device_count() < env_world:
        # RCCL needs one card per rank (a one-card rehearsal runs YANERF_DIST_BACKEND=gloo)
        print(f"bench.py: {env_world} RCCL ranks but {torch.cuda.device_count()} visible GPUs", file=sys.stderr)
        sys.exit(2)

    rank, world, local = parallel.init_distributed()
    local = parallel.device_index(local)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cfg = Config.fromfile(args.config)
    pcfg = cfg.pipeline
    H, W = int(pcfg.ray_sampler.image_height), int(pcfg.ray_sampler.image_width)
    focal_px = 0.5 * W / math.tan(0.5 * 0.6911112)  # nerf_synthetic camera_angle_x
    g = torch.Generator().manual_seed(42 + rank)  # seed + rank (run.py:70-73)
    image = torch.rand(1, H, W, 3, generator=g).to(dev)
    poses = torch.stack([torch.from_numpy(synthetic_pose(th, -30.0)) for th in np.linspace(-180, 180, 40,
                                                                                            endpoint=False)]).to(dev)
    focal = torch.tensor([focal_px], device=dev)

    def timed_window(tr, steps: int, first: int):
        parallel.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = None
        for i in range(steps):
            out = tr.step(poses[(first + i + rank) % len(poses)][None], focal, image)
        torch.cuda.synchronize()
        parallel.barrier()
        dt_local = time.perf_counter() - t0
        return out, dt_local, parallel.max_over_ranks(dt_local, device=dev)

    def run(precision: str, steps: int, warmup: int, probes: bool):
        # the reference runner's schedule (warm-up, exponential decay; init/min lr scaled by the world size), after
        # scripts/run.py's iteration -> epoch conversion over Lego's 100 training images at this world size
        tr = NeRFTrainer(pcfg, precision=precision, device=dev, runner_cfg=cfg.runner, n_rays=args.rays,
                         train_set_size=LEGO_TRAIN_IMAGES)
        for i in range(warmup):
            tr.step(poses[(i + rank) % len(poses)][None], focal, image)
        # the headline window: the production launch sequence, no probe events
        out, dt_local, dt = timed_window(tr, steps, warmup)
        mse_f = float(out["sq_fine"].mean().item() / 3.0)
        tr.dt_local = dt_local
        tr.dt_probed = None
        if probes:
            # a second window of as many steps with HIP events around the two forward launches (they have the GPU to
            # themselves) and, at N > 1, around the wait for the gradient exchange on the compute stream (its exposed
            # part); in the serial-backward modes at N = 1 the dX / dW / reduce launches too (the trainer then issues
            # the backward phase by phase). Its rate is reported beside the headline (`value_probed_window`)
            # (under the "early" schedule, bf16's default at every N, the coarse backward runs beside the fine forward:
            # that launch is then timed in the probe steps, alone on the GPU)
            shares = tr.overlap == "early"
            names = ["mlp_fwd_0"] + ([] if shares else ["mlp_fwd_1"]) + (["allreduce_exposed"] if tr.exchange else [])
            if tr.side is None and not tr.exchange:
                names += [f"mlp_{k}_{i}" for i in (1, 0) for k in ("dx", "dw", "reduce")]
            tr.enable_probes(names)
            _, tr.dt_local_probed, tr.dt_probed = timed_window(tr, steps, warmup + steps)
        return tr, dt, mse_f

    tr, dt, mse_f = run(args.precision, args.steps, args.warmup, probes=True)
    dist_info = distributed_fields(tr.dt_local, args.steps, tr.probe_ms().get("allreduce_exposed"), tr.grad_exchange,
                                   dev) if parallel.is_dist() else None
    dt_probed = tr.dt_probed
    R, Pc, Pf = tr.R, tr.Pc, tr.Pf
    rays_total = R * world * args.steps
    value = rays_total / dt
    ms_step = 1e3 * dt / args.steps
    probe = tr.probe_ms()
    flops_ray = train_flops_per_ray(Pc, Pf)
    # per-kernel rooflines of the fine pass (each kernel timed alone, after the timed region); `roofline` is the
    # dominant kernel by time, the others are listed beside it
    rk, dom, serial_ms = kernel_rooflines(tr, poses, focal, image, args.precision, live=probe)
    peak = PEAK_TFLOPS[args.precision]
    result = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "rays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": DTYPES[args.precision],
        "data": "synthetic (random 800x800 target per rank, 40 spherical poses; random-init Lego MLPs)",
        "config": {"workload": "lego_800x800_64c_128f_train_step", "rays_per_gpu": R, "pts_per_ray": Pc + Pf,
                   "global_batch_rays": R * world, "parallelism": f"dp{world}", "precision": args.precision},
        "roofline": rk[dom],
        "roofline_kernels": rk,
        "step_mfma_tflops": round(flops_ray * value / world / 1e12, 2),
        "step_mfma_frac": round(flops_ray * value / world / 1e12 / peak, 4),
        "value_probed_window": round(rays_total / dt_probed, 1),
        "timing": ("value: K unprobed steps (the production launch sequence); kernel_ms_in_timed_steps and the "
                   "rooflines' 'timed steps' figures: a second window of K steps with HIP-event probes, whose rate is "
                   "value_probed_window"),
        "kernel_ms_in_timed_steps": {k: round(v, 4) for k, v in probe.items() if k.startswith("mlp_")},
        "kernel_ms_serialised": serial_ms,
    }
    if dist_info is not None:
        result["distributed"] = dist_info
    del tr
    # the other precision modes on the same workload, reported beside the headline (never in `value`)
    notes = {"bf16": "throughput mode: bf16 weights/activations, fp32 accumulate, fp8 e4m3 storage of the saved "
                     "activations / gradient rows; gradients within the reference's own bf16-autocast error "
                     "(tests/test_gpu_fullsize.py)",
             "bf16s": "bf16 with bf16 storage throughout (the precision of the reference under torch.autocast bf16); "
                      "gradients within the reference's own bf16-autocast error (tests/test_gpu_fullsize.py)",
             "fp32x3": "fp32 operands as three bf16 planes, six bf16 MFMAs per product, fp32 saved "
                       "activations; passes the same strict parity gates as fp32 (tests/test_gpu_parity.py)",
             "fp32": "exact fp32 MFMA (v_mfma_f32_16x16x4_f32)"}
    sec = [p for p in args.secondary.split(",") if p and p not in ("none", args.precision)]
    if sec:
        result["secondary"] = {}
    progress("headline timed")
    for p2name in sec:
        tr2, dt2, _ = run(p2name, args.steps, args.warmup, probes=True)
        v2 = R * world * args.steps / dt2
        fwd2 = {k: round(v, 4) for k, v in tr2.probe_ms().items()}
        rk2, dom2, serial2 = kernel_rooflines(tr2, poses, focal, image, p2name, live=tr2.probe_ms())
        result["secondary"][p2name] = {
            "value": round(v2, 1), "unit": "rays/s",
            "value_probed_window": round(R * world * args.steps / tr2.dt_probed, 1),
            "ms_per_step": round(1e3 * dt2 / args.steps, 3),
            "dtype": DTYPES[p2name],
            "roofline": rk2[dom2],
            "roofline_kernels": rk2,
            "step_mfma_frac": round(flops_ray * v2 / world / 1e12 / PEAK_TFLOPS[p2name], 4),
            "kernel_ms_in_timed_steps": fwd2,
            "kernel_ms_serialised": serial2,
            "note": notes[p2name],
        }
        if p2name == "bf16":
            # the step priced against the MFMAs it issues: forward and dX on the bf16 MFMA, the dW (a third of the
            # step's FLOPs) at its instruction-matched peak (bf16_dw_instruction_peak)
            step_peak = 3.0 / (2.0 / PEAK_TFLOPS["bf16"] + 1.0 / bf16_dw_instruction_peak())
            result["secondary"][p2name].update({
                "step_peak_instruction_matched": round(step_peak, 1),
                "step_mfma_frac_instruction_matched": round(flops_ray * v2 / world / 1e12 / step_peak, 4)})
        del tr2
    if not args.no_extras and world == 1:
        # single-GPU characteristics (evaluation render, drop-in path, other configs, graph replay): at N > 1 every rank
        # would repeat them, and the graph capture is single-rank by design
        progress("extras")
        result["extras"] = extras(pcfg, cfg, dev, poses, focal, image, args.precision, tuple(sec))
    elif not args.no_extras:
        # BASELINE configs[3] / configs[4] on the same N ranks (the N-GPU half of those configs)
        result["configs_at_n"] = configs_at_n(pcfg, cfg, dev, poses, focal, image, world)
    if rank == 0 and world == 1 and args.psnr_steps > 0:
        progress("psnr")
        result["psnr"] = psnr_leg(args.precision, args.psnr_steps, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("cpu baseline")
        result["cpu_baseline"] = cpu_baseline(pcfg, Pc, Pf - Pc)
        result["vs_cpu_baseline"] = round(value / result["cpu_baseline"]["value"], 1)
        result["reference_cpu"] = REFERENCE_CPU
        result["vs_reference_cpu"] = round(value / REFERENCE_CPU["value"], 1)
    if rank == 0:
        print(json.dumps(result))
    parallel.barrier()
    if parallel.is_dist():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
