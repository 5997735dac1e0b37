"""Fused NeRF training step on the HIP path.

One step = the reference's train_one_epoch inner step (runners/apis.py:55-89) for one image per rank:
ray sampling (ray_sampler.py:149-246) -> coarse NeRFMLP -> EA composite -> sample_pdf refine -> fine NeRFMLP
-> composite -> objective = mse(fine) + mse(coarse) (nerf_pipeline.py:284-305) -> backward -> gradient
all-reduce over ranks (DDP semantics, run.py:162-166) -> Adam (run.py:158-160).

Every stage is a kernel of libyanerf_hip.so launched on the current stream with workspaces allocated once, so a
step issues a fixed launch sequence with no host synchronisation and no autograd graph. The models are ordinary
NeRFMLP modules whose parameters are views into one flat buffer (checkpoints keep the reference's state_dict).
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Dict, List, Optional, Sequence

import torch

from . import _C, ops, parallel
from .lr_schedule import lr_at, scaled_lrs, setup_iter_based_runner, train_loader_len  # noqa: F401
from .pipelines.models import MODELS

F32 = torch.float32


class _Pass:
    """Workspaces of one render pass (coarse or fine) for R rays x P samples."""

    def __init__(self, spec: ops.MlpSpec, R: int, P: int, dev):
        d = spec.desc()
        L = _C.lib()
        self.desc = d
        self.P = P
        N = R * P
        self.sigma = torch.empty(N, dtype=F32, device=dev)
        self.rgb = torch.empty(N, spec.color_dim, dtype=F32, device=dev)
        self.saved = torch.empty(L.yanerf_mlp_saved_bytes(ctypes.byref(d), spec.precision, N), dtype=torch.uint8,
                                 device=dev)
        self.feats = torch.empty(R, spec.color_dim, dtype=F32, device=dev)
        self.depth = torch.empty(R, dtype=F32, device=dev)
        self.alpha = torch.empty(R, dtype=F32, device=dev)
        self.w = torch.empty(R, P, dtype=F32, device=dev)
        self.sq = torch.empty(R, dtype=F32, device=dev)
        self.g_feats = torch.empty(R, spec.color_dim, dtype=F32, device=dev)
        self.g_sigma = torch.empty(R, P, dtype=F32, device=dev)
        self.g_rgb = torch.empty(R, P, spec.color_dim, dtype=F32, device=dev)
        self.ws_bytes = L.yanerf_mlp_bwd_workspace_bytes(ctypes.byref(d), spec.precision, N)


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class NeRFTrainer:
    def __init__(self, pipeline_cfg, *, precision: str = "fp32", device="cuda", lr: Optional[float] = None,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: Optional[float] = None, seed: int = 42,
                 n_rays: Optional[int] = None, overlap: Optional[bool] = None, runner_cfg=None,
                 train_set_size: Optional[int] = None, batch_size: int = 1, grad_exchange: Optional[str] = None):
        """pipeline_cfg: the `pipeline:` section of a reference config (lego.yml / fern.yml).
        runner_cfg: its `runner:` section. When given, every step uses the reference schedule
        (lr_schedule.lr_at: decay, then warm-up; init_lr / min_lr linearly scaled by the world size under
        torch.distributed, scripts/run.py:152-156) and its weight_decay; `lr` then must be None. Without it the
        learning rate is the constant `lr` (default 5e-4).
        train_set_size: the number of training images (Lego 100, Fern 17). Given with runner_cfg, the config is first
        converted as scripts/run.py:144 does (lr_schedule.setup_iter_based_runner over the rank's training loader of
        that many images at this world size and `batch_size`): num_iters and lr_decay_iters are rescaled, which at
        world > 1 changes the schedule. Without it the runner config is used as written (exact at world 1 when the
        train set divides num_iters).
        grad_exchange (world > 1 only): "bucketed" = one all-reduce per model, the coarse bucket started right after the
        coarse MLP backward and overlapped with the fine one; "single" = one all-reduce of the whole flat gradient
        after both backwards (the plain DDP-equivalent); "auto" (default) = bucketed for steps of at least
        BUCKETED_MIN_POINTS points (the Lego steps), single below (the 1,024-ray Fern step, where the second bucket's
        launches and stream hand-offs cost more than its overlap saves: measured over RCCL at world size 1, Fern bf16
        +6 % bucketed vs +2.5 % single against no process group, profiles/r6_exchange_world1.txt). Env
        YANERF_GRAD_EXCHANGE sets the default. Every choice gives the same sums.
        seed: the weights are initialised from `seed` on every rank (then broadcast from rank 0, as DDP does); the
        trainer's own Philox stream (pixel sampling, jitter, density noise, refinement) is keyed by seed + rank,
        as scripts/run.py:70-71 seeds each rank. torch's global generator is left untouched."""
        self.dev = torch.device(device)
        rs, rd, mc = pipeline_cfg["ray_sampler"], pipeline_cfg["renderer"], pipeline_cfg["model"]
        self._check_supported(pipeline_cfg)
        self.R = int(n_rays or rs["n_rays_per_image_sampled_from_mask"])
        self.Pc = int(rs["n_pts_per_ray_training"])
        self.Pn = int(rd["n_pts_per_ray_fine_training"])
        self.append = bool(rd.get("append_coarse_samples_to_fine", True))
        self.Pf = self.Pc + self.Pn if self.append else self.Pn
        self.near, self.far = float(rs["min_depth"]), float(rs["max_depth"])
        self.W, self.H = int(rs["image_width"]), int(rs["image_height"])
        self.stratified = bool(rs.get("stratified_point_sampling_training", True))
        self.random_refine = bool(rd.get("stratified_sampling_coarse_training", True))
        self.noise_std = float(rd.get("density_noise_std_train", 0.0))
        self.march = ops.RaymarchCfg(
            capping_function=rd.get("capping_function", "exponential"),
            weight_function=rd.get("weight_function", "product"),
            background_opacity=float(rd.get("background_opacity", 1e10)), blend_output=bool(rd.get("blend_output",
                                                                                                  False)),
            background_density_bias=float(rd.get("background_density_bias", 0.0)),
            hard_background=bool(rd.get("hard_background", False)),
            bg_color=tuple(float(x) for x in rd.get("bg_color", (0.0,))))
        mcfg = dict(mc)
        mcfg["precision"] = precision
        with torch.random.fork_rng(devices=[]):  # seeded init without resetting the caller's generator
            torch.manual_seed(seed)
            self.models = [MODELS.build(dict(mcfg)).to(self.dev) for _ in range(2)]  # coarse, fine
        self.specs = [m.spec() for m in self.models]
        self.params: List[List[torch.nn.Parameter]] = [m.hip_params() for m in self.models]
        self.flat = parallel.FlatParams(self.params[0] + self.params[1])
        self.n_coarse = sum(p.numel() for p in self.params[0])  # the coarse model's slice of the flat buffers
        parallel.broadcast_(self.flat.data)
        self.world, self.rank = parallel.world_rank()
        self.rng = ops.philox_stream(int(seed) + self.rank)
        self.exp_avg = torch.zeros_like(self.flat.data)
        self.exp_avg_sq = torch.zeros_like(self.flat.data)
        if runner_cfg is not None:
            if lr is not None:
                raise ValueError("NeRFTrainer: pass either runner_cfg (the reference schedule) or a constant lr")
            if list(runner_cfg.get("lr_param_groups", None) or []):
                raise NotImplementedError("NeRFTrainer: runner.lr_param_groups (runners/utils.py:148-184) is not "
                                          "supported by the fused step (one Adam group); use the registry pipeline")
            if train_set_size is not None:
                runner_cfg = setup_iter_based_runner(
                    runner_cfg, train_loader_len(int(train_set_size), self.world, batch_size), self.world, batch_size)
            # the optimizer's init_lr (param_group["init_lr"], runners/utils.py:148-151), world-scaled
            self.init_lr = scaled_lrs(runner_cfg, self.world)[0]
            wd = runner_cfg.get("weight_decay", 0.0) if weight_decay is None else weight_decay
        else:
            self.init_lr = 5e-4 if lr is None else float(lr)
            wd = 0.0 if weight_decay is None else weight_decay
        self.runner_cfg = runner_cfg
        self.lr, self.betas, self.eps, self.weight_decay = self.init_lr, betas, eps, float(wd)
        self.step_count = 0
        L = _C.lib()
        self.packed = [torch.empty(L.yanerf_mlp_packed_bytes(ctypes.byref(s.desc()), s.precision), dtype=torch.uint8,
                                   device=self.dev) for s in self.specs]
        R = self.R
        self.o = torch.empty(R, 3, dtype=F32, device=self.dev)
        self.d = torch.empty(R, 3, dtype=F32, device=self.dev)
        self.zc = torch.empty(R, self.Pc, dtype=F32, device=self.dev)
        self.zf = torch.empty(R, self.Pf, dtype=F32, device=self.dev)
        self.xys = torch.empty(R, 2, dtype=F32, device=self.dev)
        self.passes = [_Pass(self.specs[0], R, self.Pc, self.dev), _Pass(self.specs[1], R, self.Pf, self.dev)]
        # one backward workspace per pass: the coarse MLP backward runs on a side stream, overlapping the fine pass
        self.ws = [torch.empty(p.ws_bytes, dtype=torch.uint8, device=self.dev) for p in self.passes]
        # measured (tools/ab_overlap.py, step ms serial -> overlapped): bf16 3.741 -> 3.677 (round 2), fp32 30.82 ->
        # 30.48, fp32x3 20.17 -> 20.36 (its dW holds 144 KB of LDS per workgroup, so the two backwards only contend).
        # Default: on for bf16 only. In fp32 (the parity mode and the bench headline) every kernel of the step then
        # runs alone on the GPU, so the per-kernel timings in a rocprofv3 trace of the benched steps are the kernels'
        # own (the roofline kernel, the fine dW, is not stretched by the coarse backward beside it) at a 1 % cost.
        # overlap: False = serial, True / "both" = the whole coarse backward on the side stream beside the fine one,
        # "split" = the coarse input-side walk (dX) first on the main stream, then its weight gradients (dW, a
        # byte-bound kernel) on the side stream beside the fine dX (an MFMA-bound kernel)
        # Round 4, after the bf16 dW grid became one round of workgroups (tools/ab_overlap.py, bf16 step ms):
        # serial 3.590, both 3.648, split 3.613, early 3.548 -> bf16 defaults to "early" (the coarse backward beside
        # the refinement and the fine forward); fp32 serial 29.15 / early 29.15 / both 29.44 keeps serial.
        if overlap is None:
            overlap = "early" if precision in ("bf16", "bf16s") else False
        self.overlap = "both" if overlap is True else overlap
        self.side = torch.cuda.Stream(device=self.dev) if overlap else None
        # the gradient exchange runs whenever a process group is up (at world 1 too: bench.py's YANERF_PG_AT_WORLD1
        # rehearsal runs the N-rank schedule, collectives included, on one card)
        self.exchange = parallel.is_dist()
        self._h_early = None  # the coarse bucket's all-reduce, started on the side stream ("early")
        self.grad_exchange = grad_exchange or os.environ.get("YANERF_GRAD_EXCHANGE", "auto")
        if self.grad_exchange == "auto":
            self.grad_exchange = "bucketed" if self.R * (self.Pc + self.Pf) >= self.BUCKETED_MIN_POINTS else "single"
        if self.grad_exchange not in ("bucketed", "single"):
            raise ValueError(f"NeRFTrainer: grad_exchange {self.grad_exchange!r} (auto | bucketed | single)")
        self.grad_ptrs = [_C.ptr_array([p.grad.data_ptr() for p in ps]) for ps in self.params]
        self.param_ptrs = [_C.ptr_array([p.data_ptr() for p in ps]) for ps in self.params]
        # both models' packs in one launch (yanerf_mlp_pack_multi): the descriptors, the per-model parameter tables and
        # the packed buffers as the C arrays it takes
        self._pack_descs = (_C.MlpDesc * len(self.specs))(*[s.desc() for s in self.specs])
        self._pack_params = _C.ptr_array([ctypes.addressof(t) for t in self.param_ptrs])
        self._pack_dst = _C.ptr_array([t.data_ptr() for t in self.packed])
        self._pack_prec = {s.precision for s in self.specs}
        self.events: Optional[Dict[str, List]] = None  # optional per-phase timing probes
        self.kernel_probes = False  # serialise the backward kernels (per-kernel timing; see step())
        self.fused_composite = True  # yanerf_composite_train per pass (False: the three separate launches)
        # device-side step state, so one step is a fixed launch sequence with no per-step host scalars (hipGraph):
        # [0] the Philox offset base every random kernel adds to its (step-relative) offset, [1] the row of the Adam
        # table holding this step's (-lr / bias correction 1, sqrt(bias correction 2)); yanerf_step_advance moves
        # both at the end of each step. The host mirrors them (_dstate_host) and rewrites them only on a mismatch.
        self._dstate = torch.zeros(2, dtype=torch.int64, device=self.dev)
        self._dstate_host = None
        self._tab = torch.empty(self.TAB_STEPS, 2, dtype=F32, device=self.dev)
        self._tab_base, self._tab_key = 0, None
        self._pinned_keep: List[torch.Tensor] = []
        self.graph = None  # capture_step() / replay_step()
        self._render_graph = None  # render_graph(): (key, graph, static pose/focal, static outputs, buffers)
        self._capturing = False
        # evaluation (full-grid rendering) settings of the same configs (ray_sampler.py:54-56; renderer.py:29-52)
        self.Pc_eval = int(rs.get("n_pts_per_ray_evaluation", self.Pc))
        self.Pn_eval = int(rd.get("n_pts_per_ray_fine_evaluation", self.Pn))
        self.stratified_eval = bool(rs.get("stratified_point_sampling_evaluation", False))
        self.random_refine_eval = bool(rd.get("stratified_sampling_coarse_evaluation", False))
        self._eval_ws: Dict[int, Dict[str, torch.Tensor]] = {}

    TAB_STEPS = 1024  # Adam schedule rows uploaded at a time
    BUCKETED_MIN_POINTS = 1 << 19  # grad_exchange "auto": the two-bucket exchange from this many points per step

    def _pack(self, st):
        """Pack both models' current parameters into their kernel layouts: one launch when they share a precision."""
        L = _C.lib()
        if len(self._pack_prec) == 1:
            _C.check(L.yanerf_mlp_pack_multi(len(self.specs), self._pack_descs, self.specs[0].precision,
                                             self._pack_params, self._pack_dst, st), "yanerf_mlp_pack_multi")
            return
        for i, s in enumerate(self.specs):
            _C.check(L.yanerf_mlp_pack(ctypes.byref(s.desc()), s.precision, self.param_ptrs[i], _p(self.packed[i]),
                                       st), "yanerf_mlp_pack")

    # --------------------------------------------------------------------------------------- device step state
    def _lr_of_step(self, it: int) -> float:
        if self.runner_cfg is None:
            return self.lr
        return lr_at(self.runner_cfg, it, self.world, init_lr=self.init_lr)

    def _pinned(self, t: torch.Tensor) -> torch.Tensor:
        """A pinned copy of a small host tensor, kept alive until the next sync point (async H2D source)."""
        p = t.pin_memory() if torch.cuda.is_available() else t
        self._pinned_keep = self._pinned_keep[-7:] + [p]
        return p

    def _sync_step_state(self, span: int = 1) -> int:
        """Make the device step state describe the next step (Philox base = the host stream's offset, Adam table row =
        this step's), uploading the schedule table when the next `span` steps leave it or its inputs changed. Returns
        the host Philox offset at the start of the step. In steady state nothing is uploaded (no host sync)."""
        seed, off = self.rng.get_state()
        s = self.step_count
        key = (None if self.runner_cfg is not None else float(self.lr), float(self.init_lr), tuple(self.betas))
        if self._tab.shape[0] != self.TAB_STEPS:
            self._tab, self._tab_key = torch.empty(self.TAB_STEPS, 2, dtype=F32, device=self.dev), None
        if self._tab_key != key or not (self._tab_base <= s and s + span <= self._tab_base + self.TAB_STEPS):
            L = _C.lib()
            host = torch.empty(self.TAB_STEPS, 2, dtype=F32)
            base = host.data_ptr()
            for i in range(self.TAB_STEPS):
                # the reference schedules before the step (apis.py:66-68); Adam's step count is 1-based
                _C.check(L.yanerf_adam_scalars(float(self._lr_of_step(s + i)), float(self.betas[0]),
                                               float(self.betas[1]), s + i + 1,
                                               ctypes.cast(base + 8 * i, ctypes.POINTER(ctypes.c_float))),
                         "yanerf_adam_scalars")
            self._tab.copy_(self._pinned(host), non_blocking=True)
            self._tab_base, self._tab_key = s, key
            self._dstate_host = None
        want = (int(off), s - self._tab_base)
        if self._dstate_host != want:
            self._dstate.copy_(self._pinned(torch.tensor(want, dtype=torch.int64)), non_blocking=True)
            self._dstate_host = want
        return int(off)

    # --------------------------------------------------------------------------------------- timing probes
    def enable_probes(self, names: Sequence[str]):
        self.events = {n: [] for n in names}

    def _probe(self, name, fn, stream=None):
        if self.events is None or name not in self.events:
            return fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        r = fn()
        e.record(stream)
        self.events[name].append((s, e))
        return r

    def probe_ms(self) -> Dict[str, float]:
        out = {}
        for n, evs in (self.events or {}).items():
            if evs:
                out[n] = sum(s.elapsed_time(e) for s, e in evs) / len(evs)
        return out

    # --------------------------------------------------------------------------------------- one step
    @staticmethod
    def _check_supported(pipeline_cfg) -> None:
        """Refuse (instead of silently ignoring) the reference options the fused step does not implement; the
        registry NeRFPipeline runs them."""
        rs, rd = pipeline_cfg["ray_sampler"], pipeline_cfg["renderer"]
        lw = pipeline_cfg.get("loss_weights", None) or {}
        for k, v in dict(lw).items():
            if k not in ("loss_rgb_mse", "loss_prev_stage_rgb_mse") or float(v) != 1.0:
                raise NotImplementedError(f"NeRFTrainer: loss_weights {dict(lw)} (the fused step computes "
                                          f"loss_rgb_mse + loss_prev_stage_rgb_mse); use the registry NeRFPipeline")
        if float(rs.get("scene_extent", 0.0) or 0.0) > 0.0:
            raise NotImplementedError("NeRFTrainer: scene_extent > 0 (ray_sampler.py:100-110) is not supported")
        if str(rs.get("sampling_mode_training", "mask_sample")) != "mask_sample":
            raise NotImplementedError("NeRFTrainer: only MASK_SAMPLE training ray sampling is fused")
        if int(pipeline_cfg.get("num_passes", 2)) != 2:
            raise NotImplementedError("NeRFTrainer: the fused step renders exactly two passes (coarse, fine)")

    def _check_inputs(self, pose, focal, image) -> None:
        for name, t in (("pose", pose), ("focal", focal), ("image", image)):
            if not isinstance(t, torch.Tensor) or t.device != self.dev or t.dtype != F32:
                raise ValueError(f"NeRFTrainer.step: {name} must be a float32 tensor on {self.dev}")
        C = self.specs[0].color_dim
        if image.numel() != self.H * self.W * C or image.shape[-1] != C:
            raise ValueError(f"NeRFTrainer.step: image of shape {tuple(image.shape)}, expected [1, {self.H}, "
                             f"{self.W}, {C}] (the configured image size and color_dim)")
        if pose.numel() not in (12, 16) or focal.numel() != 1:
            raise ValueError(f"NeRFTrainer.step: one camera per step (pose {tuple(pose.shape)}, focal "
                             f"{tuple(focal.shape)})")

    def current_lr(self) -> float:
        """The learning rate of the next step: the reference schedule at passed_iter = steps taken so far, from the
        optimizer's init_lr (the config's, world-scaled, or the one a loaded checkpoint restored: the reference's
        schedulers read param_group["init_lr"], runners/utils.py:65-86)."""
        if self.runner_cfg is None:
            return self.lr
        return lr_at(self.runner_cfg, self.step_count, self.world, init_lr=self.init_lr)

    def step(self, pose: torch.Tensor, focal: torch.Tensor, image: torch.Tensor, near=None,
             far=None) -> Dict[str, torch.Tensor]:
        """One training step on one camera: pose [1,3,4] (or [1,4,4]), focal [1], image [1,H,W,C] float32, resident
        on the device. near/far override the configured depth range: floats, or LLFF's per-image bound tensors,
        which are averaged as _xy_to_ray_bundle does (ray_sampler.py:280-283).

        Randomness comes from the trainer's Philox stream, or, inside ops.injected_randomness(...), from the
        injected draws in the reference's order: pixel_ids [1,R] int64, jitter_u [1,R,Pc], noise (coarse [R,Pc],
        then fine [R,Pf]), pdf_u [R,Pn]. The reference's training step is replayed that way by the parity tests."""
        self._check_inputs(pose, focal, image)
        near, far, bounds = ops.depth_bounds(self.near if near is None else near, self.far if far is None else far,
                                             self.dev)
        L = _C.lib()
        st = ops._stream()
        if not self._capturing:
            self._sync_step_state()
        off0 = self.rng.get_state()[1]  # the device Philox base: kernels get offsets relative to it
        rbase = ctypes.c_void_p(self._dstate.data_ptr())
        R = self.R
        pose = pose.reshape(1, -1, 4)[:, :3, :4].contiguous()
        focal = focal.reshape(1).contiguous()
        image = image.reshape(1, self.H, self.W, -1).contiguous()
        C = image.shape[-1]
        inj_ids = ops.INJECT.take("pixel_ids")
        inj_jit = ops.INJECT.take("jitter_u") if self.stratified else None
        if inj_ids is not None:
            inj_ids = inj_ids.to(self.dev, torch.int64).reshape(1, R).contiguous()
        if inj_jit is not None:
            inj_jit = inj_jit.to(self.dev, F32).reshape(1, R, self.Pc).contiguous()
        # pack the current parameters into the kernel layout (both models, one launch; on the side stream beside the
        # ray generation it measured slower: profiles/r5_ab_pack_launches.txt)
        self._pack(st)
        # rays: uniform pixel sampling without replacement + stratified depths (Philox, or injected draws)
        seed, off = self.rng.next(R * self.Pc)
        jmode = 0 if not self.stratified else (1 if inj_jit is not None else 2)
        _C.check(L.yanerf_raygen(_p(pose), _p(focal), None, _p(inj_ids), 1, R, self.W, self.H, float(self.W),
                                 float(self.H), near, far, self.Pc, jmode, _p(inj_jit), seed, off - off0, _p(self.o),
                                 _p(self.d), _p(self.zc), _p(self.xys), None, _p(bounds), rbase, st), "yanerf_raygen")
        scale = 1.0 / (R * C)
        out = {}
        for k, (z, ps) in enumerate(((self.zc, self.passes[0]), (self.zf, self.passes[1]))):
            spec = self.specs[k]
            if k == 1:
                seed, off = self.rng.next(R * self.Pn)
                u = ops.INJECT.take("pdf_u") if self.random_refine else None
                zi = ops.INJECT.take("z_fine")
                if zi is not None:  # test mode: the reference's refined depths (ops.injected_randomness)
                    self.zf.copy_(zi.to(self.dev, F32).reshape(R, self.Pf))
                else:
                    if u is not None:
                        u = u.to(self.dev, F32).reshape(R, self.Pn).contiguous()
                    _C.check(L.yanerf_refine(_p(self.zc), _p(self.passes[0].w), R, self.Pc, self.Pn,
                                             0 if self.random_refine else 1, _p(u), seed, off - off0,
                                             int(self.append), _p(self.zf), rbase, st), "yanerf_refine")
            P = ps.P
            self._probe(f"mlp_fwd_{k}", lambda: _C.check(L.yanerf_mlp_forward(
                ctypes.byref(ps.desc), spec.precision, _p(self.packed[k]), _p(self.o), _p(self.d), _p(z), R, P,
                _p(ps.sigma), _p(ps.rgb), _p(ps.saved), st), "yanerf_mlp_forward"))
            noise = None
            if self.noise_std > 0:
                noise = ops.INJECT.take("noise")
                if noise is not None:
                    noise = noise.to(self.dev, F32).reshape(R, P).contiguous()
                    o = self.march.opts(1, self.noise_std)
                else:
                    seed, off = self.rng.next(R * P)
                    o = self.march.opts(2, self.noise_std, seed, off - off0, self._dstate.data_ptr())
            else:
                o = self.march.opts(0, 0.0)
            if self.fused_composite:
                # composite forward + photometric loss + composite backward in one launch (bit-identical to the three
                # calls below, tests/test_gpu_trainer.py)
                _C.check(L.yanerf_composite_train(ctypes.byref(o), _p(ps.sigma), _p(ps.rgb), _p(z), _p(self.d), None,
                                                  _p(noise), _p(image), _p(self.xys), 1, R, P, C, self.H, self.W,
                                                  scale, _p(ps.feats), _p(ps.depth), _p(ps.alpha), _p(ps.w),
                                                  _p(ps.sq), _p(ps.g_feats), _p(ps.g_sigma), _p(ps.g_rgb), st),
                         "yanerf_composite_train")
            else:
                _C.check(L.yanerf_composite_forward(ctypes.byref(o), _p(ps.sigma), _p(ps.rgb), _p(z), _p(self.d),
                                                    None, _p(noise), R, P, C, _p(ps.feats), _p(ps.depth),
                                                    _p(ps.alpha), _p(ps.w), st), "yanerf_composite_forward")
                _C.check(L.yanerf_rgb_loss(_p(ps.feats), _p(image), _p(self.xys), 1, R, self.H, self.W, C, scale,
                                           _p(ps.sq), _p(ps.g_feats), st), "yanerf_rgb_loss")
                _C.check(L.yanerf_composite_backward(ctypes.byref(o), _p(ps.sigma), _p(ps.rgb), _p(z), _p(self.d),
                                                     None, _p(noise), _p(ps.g_feats), None, None, R, P, C,
                                                     _p(ps.g_sigma), _p(ps.g_rgb), st), "yanerf_composite_backward")
            out["sq_coarse" if k == 0 else "sq_fine"] = ps.sq
            if k == 0 and self._early():
                # the coarse pass's loss and gradients are complete here and nothing of the fine pass depends on them:
                # its MLP backward (dX: MFMA-bound, dW: bandwidth-bound) runs on the side stream beside the refinement
                # and the fine forward (MFMA-bound) instead of after it. Under data parallelism (bucketed exchange) the
                # coarse bucket's all-reduce is started on the side stream right behind it, so it also runs beside the
                # fine pass; only the fine bucket's all-reduce is exposed.
                self.side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self.side):
                    self._mlp_backward(0, ctypes.c_void_p(self.side.cuda_stream), self.side)
                    if self.exchange and self.grad_exchange == "bucketed":
                        self._h_early = parallel.allreduce_sum_async(self.flat.grad[:self.n_coarse])
        early = self._early()
        avg_over = 1  # > 1: the flat gradient holds the sum over the ranks; Adam averages it in place (yanerf_adam_table)
        if self.exchange and not self.kernel_probes and self.grad_exchange == "bucketed":
            # Under data parallelism the gradient exchange is split in two buckets, one per model, overlapped with
            # the backward: the coarse MLP's backward runs first (or, "early", beside the fine forward on
            # the side stream), its 2.4 MB all-reduce starts on the collective stream right behind it and runs while
            # the fine MLP's backward (the longer one) occupies the GPU; only the fine bucket's all-reduce is exposed
            # before Adam. Per element the result is the same sum over ranks.
            # Probe "allreduce_exposed": HIP events on the compute stream around the wait, i.e. the time the step
            # stalls on the exchange after its last backward kernel.
            if early:
                self._mlp_backward(1, st)
                h2 = parallel.allreduce_sum_async(self.flat.grad[self.n_coarse:])
                torch.cuda.current_stream().wait_stream(self.side)
                h, self._h_early = self._h_early, None
            else:
                self._mlp_backward(0, st)
                h = parallel.allreduce_sum_async(self.flat.grad[:self.n_coarse])
                self._mlp_backward(1, st)
                h2 = parallel.allreduce_sum_async(self.flat.grad[self.n_coarse:])
            self._probe("allreduce_exposed", lambda: (parallel.finish_allreduce(h), parallel.finish_allreduce(h2)))
            avg_over = self.world  # DDP's divide by the world size, inside the Adam launch (no launch of its own)
        elif self.exchange and not self.kernel_probes:
            # "single": both backwards, then one all-reduce of the whole flat gradient (all of it exposed)
            self._mlp_backward(1, st)
            if early:
                torch.cuda.current_stream().wait_stream(self.side)
            else:
                self._mlp_backward(0, st)
            self._probe("allreduce_exposed", lambda: parallel.allreduce_sum_(self.flat.grad))
            avg_over = self.world
        elif self.kernel_probes:
            # timing probe mode (bench.py's per-kernel roofline): every MLP backward kernel alone on the stream, in the
            # order dX, dW, slab reduce; the result is identical to the other schedules
            for k in (1, 0):
                for ph in (1, 4, 8):
                    self._mlp_backward(k, st, phase=ph)
        elif self.side is None:
            if self.events is not None and any(n.startswith(("mlp_dx_", "mlp_dw_")) for n in self.events):
                # serial backward with timing probes (bench.py's live per-kernel roofline): the same kernels in the
                # same order as one phase-3 call, issued phase by phase so each gets its own event pair
                for k in (1, 0):
                    for ph in (1, 4, 8):
                        self._mlp_backward(k, st, phase=ph)
            else:
                self._mlp_backward(1, st)
                self._mlp_backward(0, st)
        elif early:
            self._mlp_backward(1, st)
            torch.cuda.current_stream().wait_stream(self.side)
        elif self.overlap == "split":
            self._mlp_backward(0, st, phase=1)
            self.side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.side):
                self._mlp_backward(0, ctypes.c_void_p(self.side.cuda_stream), self.side, phase=2)
            self._mlp_backward(1, st)
            torch.cuda.current_stream().wait_stream(self.side)
        else:
            # the two MLP backwards are independent: the coarse one runs on the side stream beside the fine one (the
            # overlap fills each kernel's tail wave and the gaps between the dX / dW / reduce launches); the forward
            # kernels keep the GPU to themselves, so their timing (the bench's roofline) is unaffected
            self.side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.side):
                self._mlp_backward(0, ctypes.c_void_p(self.side.cuda_stream), self.side)
            self._mlp_backward(1, st)
            torch.cuda.current_stream().wait_stream(self.side)
        if self.kernel_probes:
            parallel.allreduce_mean_(self.flat.grad)
        self.lr = self.current_lr()  # the reference schedules before the step (apis.py:66-68)
        self.step_count += 1
        # Adam with this step's scalars from the device table (the values yanerf_adam computes for this lr and step)
        _C.check(L.yanerf_adam_table(_p(self.flat.data), _p(self.flat.grad), _p(self.exp_avg), _p(self.exp_avg_sq),
                                     self.flat.numel, _p(self._tab), ctypes.c_void_p(self._dstate.data_ptr() + 8),
                                     float(self.betas[0]), float(self.betas[1]), float(self.eps),
                                     float(self.weight_decay), avg_over, st), "yanerf_adam_table")
        delta = self.rng.get_state()[1] - off0
        _C.check(L.yanerf_step_advance(rbase, delta, st), "yanerf_step_advance")
        if self._dstate_host is not None:
            self._dstate_host = (self._dstate_host[0] + delta, self._dstate_host[1] + 1)
        return out

    # --------------------------------------------------------------------------------------- hipGraph
    def capture_step(self, pose: torch.Tensor, focal: torch.Tensor, image: torch.Tensor, near=None, far=None,
                     n_steps: int = 1):
        """Capture `n_steps` consecutive training steps as ONE HIP graph (torch.cuda.CUDAGraph over the launch sequence
        of step(), n_steps times). Every per-step scalar lives on the device (Philox base, Adam table row;
        _sync_step_state), so replay_step() runs the captured steps with each step's own draws, learning rate and bias
        corrections, bit for bit the steps step() would run. Step k of a replay reads pose / focal / depth range from
        row k of static buffers: pose [n_steps, 3|4, 4] and focal [n_steps] (or one row, used for every step) are
        copied into them at each replay; the image buffer is captured by reference (replay_step(image=...) copies a
        different one into it). near / far: floats, or LLFF's per-image bound tensors (averaged as step() does; one
        value for all steps, or n_steps rows); without them the range of the previous replay stays. Several steps per
        graph amortise the graph launch and the input copies over the steps (a 1,024-ray step is ~1 ms). Run at least
        one eager step first (the library's kernels load on first launch). Single rank only (a gloo exchange cannot be
        captured)."""
        if self.exchange:
            raise NotImplementedError("NeRFTrainer.capture_step: single rank only (no process group)")
        if self.events is not None or self.kernel_probes:
            raise ValueError("NeRFTrainer.capture_step: disable timing probes first")
        K = int(n_steps)
        if not 1 <= K <= self.TAB_STEPS:
            raise ValueError(f"NeRFTrainer.capture_step: n_steps {n_steps} out of [1, {self.TAB_STEPS}]")
        poses = self._step_rows(pose.reshape(-1, pose.shape[-2], 4)[:, :3, :4], K, "pose")
        self._check_inputs(poses[0:1], focal.reshape(-1)[0:1], image)
        self._g_K = K
        self._g_pose = poses.contiguous().clone()
        self._g_focal = self._step_rows(focal.reshape(-1), K, "focal").contiguous().clone()
        self._g_image = image.reshape(1, self.H, self.W, -1).contiguous()
        self._g_bounds = torch.empty(K, 2, dtype=F32, device=self.dev)
        self._set_graph_bounds(near, far)
        self._g_bounds_key = self._host_bounds_key(near, far)
        self._sync_step_state(span=K)
        rng0, step0, lr0, dstate0 = self.rng.get_state(), self.step_count, self.lr, self._dstate_host
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        self._capturing = True
        try:
            with torch.cuda.graph(g):
                for k in range(K):
                    out = self.step(self._g_pose[k:k + 1], self._g_focal[k:k + 1], self._g_image,
                                    self._g_bounds[k, 0:1], self._g_bounds[k, 1:2])
        finally:
            self._capturing = False
        # the capture ran nothing: undo the captured steps' host bookkeeping; each replay re-applies it
        self._g_rng_delta = self.rng.get_state()[1] - rng0[1]
        self.rng.set_state(rng0)
        self.step_count, self.lr, self._dstate_host = step0, lr0, dstate0
        self.graph, self._g_out = g, out
        return out

    def _step_rows(self, x: torch.Tensor, K: int, name: str) -> torch.Tensor:
        """x with K rows along dim 0 (one row is repeated for every captured step)."""
        if x.shape[0] == K:
            return x
        if x.shape[0] == 1:
            return x.expand(K, *x.shape[1:])
        raise ValueError(f"NeRFTrainer: {name} has {x.shape[0]} rows for {K} captured steps")

    def _host_bounds_key(self, near, far):
        """The (near, far) rows of host-side bounds (floats or CPU tensors: LLFF's per-image bounds come from the
        loader on the host), so a replay with the same values skips rewriting the graph's static bounds buffer (its
        fill launches cost ~10 us each on a ~1 ms step); None when either is a device tensor or missing. The rows are
        read as _set_graph_bounds reads them."""
        K = self._g_K
        out = []
        for v in (near, far):
            if v is None or (isinstance(v, torch.Tensor) and v.device.type != "cpu"):
                return None
            if isinstance(v, torch.Tensor):
                per_step = v.dim() > 1 or (K > 1 and v.dim() == 1 and v.numel() == K)
                out.append(tuple(v.float().reshape(v.shape[0] if per_step else 1, -1).mean(-1).tolist()))
            else:
                out.append(float(v))
        return tuple(out)

    def _set_graph_bounds(self, near, far):
        """Write the depth range of the captured steps into the static [K, 2] buffer: None = the config's value;
        floats; tensors averaged per step (ray_sampler.py:280-283) -- [K, ...] rows (one per captured step), a 1-D
        tensor of K values when K > 1 (one per step), or any other shape = one image's bounds, averaged into one value
        for every step -- host tensors on the host, device tensors on the device (no host sync)."""
        K = self._g_bounds.shape[0]
        for i, (v, dflt) in enumerate(((near, self.near), (far, self.far))):
            v = dflt if v is None else v
            if isinstance(v, torch.Tensor):
                per_step = v.dim() > 1 or (K > 1 and v.dim() == 1 and v.numel() == K)
                v = v.float().reshape(v.shape[0] if per_step else 1, -1).mean(-1)
                if v.numel() not in (1, K):
                    raise ValueError(f"NeRFTrainer: {v.numel()} depth bounds for {K} captured steps")
                if v.device.type == "cpu":
                    v = v.tolist()
            if isinstance(v, torch.Tensor):
                self._g_bounds[:, i].copy_(v.expand(K))
            elif isinstance(v, list) and len(v) == K and K > 1:
                self._g_bounds[:, i].copy_(torch.tensor(v, dtype=F32), non_blocking=False)
            else:
                self._g_bounds[:, i].fill_(float(v[0] if isinstance(v, list) else v))

    def replay_step(self, pose: Optional[torch.Tensor] = None, focal: Optional[torch.Tensor] = None,
                    image: Optional[torch.Tensor] = None, near=None, far=None) -> Dict[str, torch.Tensor]:
        """The captured step(s) by replaying the graph (capture_step): n_steps training steps on `pose` / `focal`
        (n_steps rows or one; copied into the static buffers; default: the previous ones), the captured image buffer
        and the depth range near / far (default: the previous replay's). Returns the last step's outputs."""
        if self.graph is None:
            raise RuntimeError("NeRFTrainer.replay_step: call capture_step first")
        K = self._g_K
        if near is not None or far is not None:
            key = self._host_bounds_key(near, far)
            if key is None or key != self._g_bounds_key:  # host bounds equal to the previous replay's: nothing to write
                # the side not given keeps its per-step rows ([K, 1]: one row per captured step, not one image's bounds)
                cur = (self._g_bounds[:, 0:1].clone(), self._g_bounds[:, 1:2].clone())
                self._set_graph_bounds(cur[0] if near is None else near, cur[1] if far is None else far)
                self._g_bounds_key = key
        if pose is not None:
            self._g_pose.copy_(self._step_rows(pose.reshape(-1, pose.shape[-2], 4)[:, :3, :4], K, "pose"))
        if focal is not None:
            self._g_focal.copy_(self._step_rows(focal.reshape(-1), K, "focal"))
        if image is not None and image.data_ptr() != self._g_image.data_ptr():
            self._g_image.copy_(image.reshape(self._g_image.shape))
        self._sync_step_state(span=K)  # no-op in steady state; uploads the next schedule rows every TAB_STEPS steps
        self.graph.replay()
        seed, off = self.rng.get_state()
        self.rng.set_state((seed, off + self._g_rng_delta))
        self.step_count += K
        self.lr = self._lr_of_step(self.step_count - 1)
        self._dstate_host = (self._dstate_host[0] + self._g_rng_delta, self._dstate_host[1] + K)
        return self._g_out

    def _early(self) -> bool:
        """The "early" schedule: the coarse MLP backward on the side stream right after the coarse composite, beside
        the refinement and the fine forward (kernel-probe steps serialise every backward kernel instead)."""
        return self.overlap == "early" and not self.kernel_probes

    def _mlp_backward(self, k: int, st, stream=None, phase: int = 3):
        L = _C.lib()
        ps, spec = self.passes[k], self.specs[k]
        name = {3: "mlp_bwd", 1: "mlp_dx", 2: "mlp_dwr", 4: "mlp_dw", 8: "mlp_reduce"}[phase] + f"_{k}"
        self._probe(name, lambda: _C.check(L.yanerf_mlp_backward_phase(
            ctypes.byref(ps.desc), spec.precision, _p(self.packed[k]), _p(ps.saved), _p(ps.rgb), _p(ps.g_sigma),
            _p(ps.g_rgb), self.R, ps.P, self.grad_ptrs[k], _p(self.ws[k]), phase, st), "yanerf_mlp_backward"), stream)

    # --------------------------------------------------------------------------------------- evaluation
    def _eval_buffers(self, R: int) -> Dict[str, torch.Tensor]:
        if R not in self._eval_ws:
            Pf = self.Pc_eval + self.Pn_eval if self.append else self.Pn_eval
            dev, C = self.dev, self.specs[0].color_dim
            b = dict(o=torch.empty(R, 3, device=dev), d=torch.empty(R, 3, device=dev),
                     zc=torch.empty(R, self.Pc_eval, device=dev), zf=torch.empty(R, Pf, device=dev),
                     xys=torch.empty(R, 2, device=dev), sigma=torch.empty(R * Pf, device=dev),
                     rgb=torch.empty(R * Pf, C, device=dev), feats=torch.empty(2, R, C, device=dev),
                     depth=torch.empty(2, R, device=dev), alpha=torch.empty(R, device=dev),
                     w=torch.empty(R, Pf, device=dev))
            self._eval_ws = {R: b}  # keep one size
        return self._eval_ws[R]

    @torch.no_grad()
    def render(self, pose: torch.Tensor, focal: torch.Tensor, H: Optional[int] = None, W: Optional[int] = None,
               near: Optional[float] = None, far: Optional[float] = None, chunk: int = 65536,
               shard: bool = False):
        """Full-grid evaluation render of one camera with the current weights, on the fused inference kernels:
        the reference's EVALUATION pass (nerf_pipeline.py:217-236: FULL_GRID rays, deterministic depths and
        refinement, no density noise), in chunks of `chunk` rays (it chunks by 131072 points in Python; the result
        does not depend on the chunking). Returns (rgb [H,W,C] fine, rgb [H,W,C] coarse, depth [H,W] fine).

        shard=True (under torch.distributed): every rank renders its contiguous block of image rows
        (parallel.shard_range) and one all_gather per output assembles the image on every rank. Rays are
        independent, so the result equals the single-GPU render; there is no other exchange."""
        L = _C.lib()
        st = ops._stream()
        H = int(H or self.H)
        W = int(W or self.W)
        near = self.near if near is None else float(near)
        far = self.far if far is None else float(far)
        pose = pose.reshape(1, -1, 4)[:, :3, :4].contiguous()
        focal = focal.reshape(1).contiguous()
        self._pack(st)
        world, rank = parallel.world_rank() if shard else (1, 0)
        rows = parallel.shard_range(H, rank, world)
        p0, n = rows.start * W, len(rows) * W
        R = max(1, min(chunk, n))
        b = self._eval_buffers(R)
        C = self.specs[0].color_dim
        out_f = torch.empty(n, C, device=self.dev)
        out_c = torch.empty(n, C, device=self.dev)
        out_d = torch.empty(n, device=self.dev)
        opts = self.march.opts(0, 0.0)
        for r0 in range(0, n, R):
            r = min(R, n - r0)
            ids = torch.arange(p0 + r0, p0 + r0 + r, device=self.dev, dtype=torch.int64)
            seed, off = self.rng.next(r * self.Pc_eval)
            _C.check(L.yanerf_raygen(_p(pose), _p(focal), None, _p(ids), 1, r, W, H, float(self.W), float(self.H),
                                     near, far, self.Pc_eval, 2 if self.stratified_eval else 0, None, seed, off,
                                     _p(b["o"]), _p(b["d"]), _p(b["zc"]), _p(b["xys"]), None, None, None, st),
                     "yanerf_raygen")
            zs = (b["zc"], b["zf"])
            for k in range(2):
                spec = self.specs[k]
                P = self.Pc_eval if k == 0 else zs[1].shape[1]
                if k == 1:
                    seed, off = self.rng.next(r * self.Pn_eval)
                    _C.check(L.yanerf_refine(_p(b["zc"]), _p(b["w"]), r, self.Pc_eval, self.Pn_eval,
                                             0 if self.random_refine_eval else 1, None, seed, off, int(self.append),
                                             _p(b["zf"]), None, st), "yanerf_refine")
                desc = spec.desc()
                _C.check(L.yanerf_mlp_forward(ctypes.byref(desc), spec.precision, _p(self.packed[k]), _p(b["o"]),
                                              _p(b["d"]), _p(zs[k]), r, P, _p(b["sigma"]), _p(b["rgb"]), None, st),
                         "yanerf_mlp_forward")
                _C.check(L.yanerf_composite_forward(ctypes.byref(opts), _p(b["sigma"]), _p(b["rgb"]), _p(zs[k]),
                                                    _p(b["d"]), None, None, r, P, C, _p(b["feats"][k]),
                                                    _p(b["depth"][k]), _p(b["alpha"]), _p(b["w"]), st),
                         "yanerf_composite_forward")
            out_c[r0:r0 + r] = b["feats"][0, :r]
            out_f[r0:r0 + r] = b["feats"][1, :r]
            out_d[r0:r0 + r] = b["depth"][1, :r]
        out_f, out_c, out_d = out_f.view(-1, W, C), out_c.view(-1, W, C), out_d.view(-1, W)
        if world > 1:
            out_f, out_c, out_d = (parallel.gather_rows(t, H) for t in (out_f, out_c, out_d))
        return out_f, out_c, out_d

    @torch.no_grad()
    def render_graph(self, pose: torch.Tensor, focal: torch.Tensor, H: Optional[int] = None, W: Optional[int] = None,
                     near: Optional[float] = None, far: Optional[float] = None, chunk: int = 65536):
        """render() as ONE graph launch per image: the first call for an (H, W, near, far, chunk) captures the whole
        chunk loop (weight pack, per chunk raygen -> coarse MLP -> composite -> refine -> fine MLP -> composite, and
        the output copies; nerf_pipeline.py:217-236, 327-377) into a HIP graph, later calls copy pose / focal into its
        static inputs and replay it. Bit for bit render() (tests/test_gpu_trainer.py). The reference's evaluation
        sampling is deterministic (no stratified depths, deterministic refinement); a config with random evaluation
        draws would freeze them in the graph, so it is refused. Single rank; the returned tensors are the graph's
        static outputs, overwritten by the next replay."""
        if self.stratified_eval or self.random_refine_eval:
            raise NotImplementedError("NeRFTrainer.render_graph: random evaluation sampling cannot be replayed")
        key = (int(H or self.H), int(W or self.W), None if near is None else float(near),
               None if far is None else float(far), int(chunk))
        if self._render_graph is None or self._render_graph[0] != key:
            sp = pose.reshape(1, -1, 4)[:, :3, :4].contiguous().clone()
            sf = focal.reshape(1).contiguous().clone()
            rng_pre = self.rng.get_state()
            self.render(sp, sf, *key[:4], chunk=chunk)  # eager first: the evaluation buffers exist before the capture
            torch.cuda.synchronize(self.dev)
            # the capture draws from the offsets an eager render() at this point would (the warm-up's draws are undone)
            self.rng.set_state(rng_pre)
            rng0 = self.rng.get_state()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                outs = self.render(sp, sf, *key[:4], chunk=chunk)
            # the capture ran nothing: rewind the counter; every replay advances it by what an eager render() draws,
            # so training steps after an evaluation draw the same pixels / jitter / noise whichever render path ran
            delta = self.rng.get_state()[1] - rng0[1]
            self.rng.set_state(rng_pre)  # (the eager warm-up's draws are not counted either)
            # the graph writes into these evaluation buffers: keep them alive even if a later eager render() of
            # another size replaces the trainer's buffer cache
            keep = dict(self._eval_ws)
            self._render_graph = (key, g, sp, sf, outs, keep, delta)
        _, g, sp, sf, outs, _, delta = self._render_graph
        sp.copy_(pose.reshape(1, -1, 4)[:, :3, :4])
        sf.copy_(focal.reshape(1))
        g.replay()
        seed, off = self.rng.get_state()
        self.rng.set_state((seed, off + delta))
        return outs

    def evaluate(self, images, shard: bool = True) -> Dict[str, float]:
        """Render every camera of a DeviceImageSet and score it as the reference's eval_one_epoch + create_stats do:
        per-image MSE of each stage (pipelines/utils.py:137-158), PSNR of the MEAN MSE (runners/utils.py:270-283).
        Under torch.distributed (shard=True) the images are split as the reference's evaluation DistributedSampler
        splits them (parallel.eval_order) and the per-image MSEs are all-gathered per iteration (apis.py:173-177,
        201), so every rank returns the same numbers as a single-GPU evaluation."""
        world, rank = parallel.world_rank() if shard else (1, 0)
        n = len(images)
        mse = []
        for i in parallel.eval_order(n, rank, world):
            pose, focal, img, nr, fr = images.item(i)
            near = None if nr is None else float(nr.mean())  # per-image bounds -> scalar (ray_sampler.py:280-283)
            far = None if fr is None else float(fr.mean())
            f, c, _ = self.render(pose, focal, images.H, images.W, near, far)
            m = torch.stack([torch.mean((f - img[0]) ** 2), torch.mean((c - img[0]) ** 2)]).view(1, 2)
            mse.append(parallel.allgather_cat(m) if world > 1 else m)
        allm = torch.cat(mse, dim=0)[:n]  # dataset order; DistributedSampler padding dropped
        mf, mc = (float(x) for x in allm.mean(dim=0).tolist())
        return {"loss_rgb_mse": mf, "loss_prev_stage_rgb_mse": mc, "loss_rgb_psnr": -10.0 * math.log10(max(mf, 1e-12)),
                "loss_prev_stage_rgb_psnr": -10.0 * math.log10(max(mc, 1e-12))}

    # --------------------------------------------------------------------------------------- checkpoints
    def pipeline_state_dict(self) -> Dict[str, torch.Tensor]:
        """The two models' parameters under the reference NeRFPipeline's keys (checkpoint.py)."""
        sd = {}
        for i, m in enumerate(self.models):
            for k, v in m.state_dict().items():
                sd[f"implicit_functions.{i}._fn.{k}"] = v.detach().cpu().clone()
        return sd

    def load_pipeline_state_dict(self, sd: Dict[str, torch.Tensor]):
        from . import checkpoint
        for m, msd in zip(self.models, checkpoint.split_pipeline_state(sd, len(self.models))):
            m.load_state_dict(msd)  # copies into the flat-buffer views (parameters are not re-allocated)

    def optimizer_state_dict(self) -> Dict:
        from . import checkpoint
        return checkpoint.adam_state_from_flat(self.params[0] + self.params[1], self.exp_avg, self.exp_avg_sq,
                                               self.step_count, self.lr, self.betas, self.eps, self.weight_decay,
                                               init_lr=self.init_lr)

    def load_optimizer_state_dict(self, osd: Dict):
        from . import checkpoint
        step = checkpoint.adam_state_to_flat(osd, self.params[0] + self.params[1], self.exp_avg, self.exp_avg_sq)
        self.step_count = step or 0
        g = osd.get("param_groups", [{}])[0]
        self.lr = float(g.get("lr", self.lr))
        self.init_lr = float(g.get("init_lr", self.init_lr))
        self.betas = tuple(g.get("betas", self.betas))
        self.eps = float(g.get("eps", self.eps))
        self.weight_decay = float(g.get("weight_decay", self.weight_decay))

    @staticmethod
    def objective(out: Dict[str, torch.Tensor]) -> torch.Tensor:
        """mse(fine) + mse(coarse) from the per-ray squared errors (device tensor; no host sync)."""
        n = out["sq_fine"].numel() * 3
        return (out["sq_fine"].sum() + out["sq_coarse"].sum()) / n
