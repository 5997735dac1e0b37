#!/usr/bin/env python
"""Does the bf16 weight-gradient kernel read its fp8 gradient rows (dZ, written by the dX kernel just before) from the
MI355X's 256 MB Infinity Cache when they fit in it? The premise of a backward that interleaves dX and dW per point chunk
so dZ skips the HBM round trip. For several point counts: dW timed right after dX, and dW
timed after a 1 GiB write has swept the caches; per-point ns of each. Development tool (GPU); one JSON line.

    python tools/mall_probe.py [bf16]
"""
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


def main(reps=7):
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    dev = torch.device("cuda:0")
    L = _C.lib()
    torch.manual_seed(0)
    m = MODELS.build(dict(type="NeRFMLP", precision=prec)).to(dev)
    spec = m.spec()
    d = spec.desc()
    packed = m.packed_weights(spec)
    grads = [torch.empty_like(p) for p in m.hip_params()]
    gp = _C.ptr_array([g.data_ptr() for g in grads])
    sweep = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    P_ = ops._p
    st = ops._stream()
    out = {"precision": prec}
    for R in (256, 512, 1024, 2048, 4096):
        P = 192
        N = R * P
        o = torch.randn(R, 3, device=dev) * 0.2 + torch.tensor([0.0, 0.0, 4.0], device=dev)
        dv = torch.randn(R, 3, device=dev)
        z = torch.sort(torch.rand(R, P, device=dev) * 4 + 2, -1)[0]
        sigma, rgb = torch.empty(N, device=dev), torch.empty(N, 3, device=dev)
        saved = torch.empty(L.yanerf_mlp_saved_bytes(ctypes.byref(d), spec.precision, N), dtype=torch.uint8, device=dev)
        ws = torch.empty(L.yanerf_mlp_bwd_workspace_bytes(ctypes.byref(d), spec.precision, N), dtype=torch.uint8,
                         device=dev)
        gs, gr = torch.randn(N, device=dev), torch.randn(N, 3, device=dev)
        _C.check(L.yanerf_mlp_forward(ctypes.byref(d), spec.precision, P_(packed), P_(o), P_(dv), P_(z), R, P, P_(sigma),
                                      P_(rgb), P_(saved), st), "fwd")

        def phase(ph):
            _C.check(L.yanerf_mlp_backward_phase(ctypes.byref(d), spec.precision, P_(packed), P_(saved), P_(rgb), P_(gs),
                                                 P_(gr), R, P, gp, P_(ws), ph, st), "bwd")

        hot, cold = [], []
        for _ in range(reps):
            for lst, sw in ((hot, False), (cold, True)):
                phase(1)  # dX: writes dZ
                if sw:
                    sweep.fill_(1)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                phase(4)  # dW alone
                e.record()
                lst.append((s, e))
        torch.cuda.synchronize()
        med = lambda evs: sorted(a.elapsed_time(b) for a, b in evs)[len(evs) // 2]  # noqa: E731
        h, c = med(hot), med(cold)
        gb = ws.numel() / 1e9
        out[f"R{R}"] = {"points": N, "dW_after_dX_ms": round(h, 4), "dW_after_sweep_ms": round(c, 4),
                        "ns_per_point_hot": round(1e6 * h / N, 3), "ns_per_point_cold": round(1e6 * c / N, 3),
                        "bwd_workspace_gb": round(gb, 3)}
        del saved, ws
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
