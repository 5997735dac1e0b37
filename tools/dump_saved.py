#!/usr/bin/env python
"""Dump the fp32 forward's saved-activation buffer for a small fixed batch (A/B of store-path variants: the bytes
must be identical). Development tool: python tools/dump_saved.py OUT.npy [prec]"""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import yanerf_boot  # noqa: E402,F401
from yanerf_amd import _C, ops  # noqa: E402
from yanerf_amd.pipelines.models import MODELS  # noqa: E402


def main():
    out, prec = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "fp32")
    dev = torch.device("cuda:0")
    L = _C.lib()
    torch.manual_seed(0)
    m = MODELS.build(dict(type="NeRFMLP", precision=prec)).to(dev)
    spec = m.spec()
    d = spec.desc()
    packed = m.packed_weights(spec)
    R, P = 64, 64
    o = torch.randn(R, 3, device=dev) * 0.2 + torch.tensor([0.0, 0.0, 4.0], device=dev)
    dv = torch.randn(R, 3, device=dev)
    z = torch.sort(torch.rand(R, P, device=dev) * 4 + 2, -1)[0]
    N = R * P
    sigma = torch.empty(N, device=dev)
    rgb = torch.empty(N, 3, device=dev)
    saved = torch.zeros(L.yanerf_mlp_saved_bytes(ctypes.byref(d), spec.precision, N), dtype=torch.uint8, device=dev)
    P_ = ops._p
    _C.check(L.yanerf_mlp_forward(ctypes.byref(d), spec.precision, P_(packed), P_(o), P_(dv), P_(z), R, P, P_(sigma),
                                  P_(rgb), P_(saved), ops._stream()), "fwd")
    torch.cuda.synchronize()
    np.save(out, saved.cpu().numpy())


if __name__ == "__main__":
    main()
