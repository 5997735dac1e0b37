#!/usr/bin/env python
"""Per-kernel timing of the MLP kernels at the Lego fine-pass size (4096 rays x 192 points), interleaved A/B in
one process (HIP events on the launch stream). Variants: forward with / without the saved-activation stream,
backward (dX + dW + reduce) and its three kernels alone. Development tool; prints one JSON line."""
import ctypes
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import yanerf_boot  # noqa: E402,F401
from yanerf_amd import _C, ops  # noqa: E402
from yanerf_amd.pipelines.models import MODELS  # noqa: E402


def main(R=4096, P=192, reps=10):
    dev = torch.device("cuda:0")
    L = _C.lib()
    res = {}
    for prec in (sys.argv[1].split(",") if len(sys.argv) > 1 else ("fp32", "bf16", "fp32x3")):
        torch.manual_seed(0)
        m = MODELS.build(dict(type="NeRFMLP", precision=prec)).to(dev)
        spec = m.spec()
        d = spec.desc()
        packed = m.packed_weights(spec)
        o = torch.randn(R, 3, device=dev) * 0.2 + torch.tensor([0.0, 0.0, 4.0], device=dev)
        dv = torch.randn(R, 3, device=dev)
        z = torch.sort(torch.rand(R, P, device=dev) * 4 + 2, -1)[0]
        N = R * P
        sigma = torch.empty(N, device=dev)
        rgb = torch.empty(N, 3, device=dev)
        saved = torch.empty(L.yanerf_mlp_saved_bytes(ctypes.byref(d), spec.precision, N), dtype=torch.uint8,
                            device=dev)
        ws = torch.empty(L.yanerf_mlp_bwd_workspace_bytes(ctypes.byref(d), spec.precision, N), dtype=torch.uint8,
                         device=dev)
        gs = torch.randn(N, device=dev)
        gr = torch.randn(N, 3, device=dev)
        grads = [torch.empty_like(p) for p in m.hip_params()]
        gp = _C.ptr_array([g.data_ptr() for g in grads])
        P_ = ops._p
        st = ops._stream()

        def fwd(with_saved):
            _C.check(L.yanerf_mlp_forward(ctypes.byref(d), spec.precision, P_(packed), P_(o), P_(dv), P_(z), R, P,
                                          P_(sigma), P_(rgb), P_(saved) if with_saved else None, st), "fwd")

        def bwd():
            _C.check(L.yanerf_mlp_backward(ctypes.byref(d), spec.precision, P_(packed), P_(saved), P_(rgb), P_(gs),
                                           P_(gr), R, P, gp, P_(ws), st), "bwd")

        def bwd_phase(ph):
            _C.check(L.yanerf_mlp_backward_phase(ctypes.byref(d), spec.precision, P_(packed), P_(saved), P_(rgb),
                                                 P_(gs), P_(gr), R, P, gp, P_(ws), ph, st), "bwd_phase")

        variants = {"fwd_train": lambda: fwd(True), "fwd_infer": lambda: fwd(False), "bwd": bwd,
                    "bwd_dx": lambda: bwd_phase(1), "bwd_dw": lambda: bwd_phase(4), "bwd_reduce": lambda: bwd_phase(8)}
        times = {k: [] for k in variants}
        for k in variants:  # warm
            variants[k]()
        torch.cuda.synchronize()
        for _ in range(reps):
            for k, f in variants.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                f()
                e.record()
                times[k].append((s, e))
        torch.cuda.synchronize()
        # digest of the weight gradients of one more backward: A/B variants that must be bitwise equal compare it
        bwd()
        torch.cuda.synchronize()
        import hashlib
        res[f"{prec}_grad_digest"] = hashlib.sha1(b"".join(g.cpu().numpy().tobytes() for g in grads)).hexdigest()[:16]
        for with_saved in (False, True):  # forward outputs of both instantiations
            sigma.zero_(), rgb.zero_()
            fwd(with_saved)
            torch.cuda.synchronize()
            res[f"{prec}_out_digest_{'train' if with_saved else 'infer'}"] = hashlib.sha1(
                sigma.cpu().numpy().tobytes() + rgb.cpu().numpy().tobytes()).hexdigest()[:16]
        flop = 2.0 * 589_952 * N
        for k, evs in times.items():
            ms = sorted(a.elapsed_time(b) for a, b in evs)
            med = ms[len(ms) // 2]
            fl = flop * (2.0 if k == "bwd" else 1.0 if k.startswith("fwd") or k in ("bwd_dx", "bwd_dw") else 0.0)
            res[f"{prec}_{k}"] = {"ms": round(med, 4), "tflops": round(fl / med / 1e9, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    import os
    main(R=int(os.environ.get("YANERF_MB_R", 4096)), P=int(os.environ.get("YANERF_MB_P", 192)))
