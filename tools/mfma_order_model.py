"""Which summation order and rounding do gfx950's f32 and bf16 MFMAs use? (tools/probes/probe_mfma_order.hip)

    python tools/mfma_order_model.py gen  f32|bf16 N in.bin       # operands (seeded, wide exponent range)
    python tools/mfma_order_model.py check f32|bf16 in.bin out.bin # match rate of each candidate model

Candidate models for D[i][j] = C[i][j] + sum_k A[i][k] B[k][j] (k over the instruction's K, in lane-group order):
  chain_fma      acc = fma(a_k, b_k, acc) for k = 0, 1, ... from C
  chain_fma_rev  the same from the last k down
  exact_round    C + every product summed exactly, one round-to-nearest-even to fp32
  exact_prod_then_c  the products summed exactly and rounded, then + C rounded
  chain_mul_add  acc = round(acc + round(a_k b_k))
The result picks the summation order trial (e) of make_golden.gen_sensitivity emulates (oracle side: tests/golden/
mfma_order.c)."""
from __future__ import annotations

import math
import struct
import sys

import numpy as np


def _operands(kind, n, rng):
    K = 4 if kind == "f32" else 32
    def vals(shape):
        m = rng.uniform(1.0, 2.0, size=shape) * rng.choice([-1.0, 1.0], size=shape)
        e = rng.integers(-6, 7, size=shape)
        v = (m * np.exp2(e)).astype(np.float32)
        if kind == "bf16":  # representable in bf16 (truncate the low 16 bits)
            v = (v.view(np.uint32) & np.uint32(0xFFFF0000)).view(np.float32)
        return v
    A = vals((n, 16, K))
    B = vals((n, K, 16))
    C = vals((n, 16, 16)).astype(np.float32)
    # a quarter of the trials: C nearly cancels the dot product (exposes intermediate roundings)
    q = n // 4
    dot = np.einsum("tik,tkj->tij", A[:q].astype(np.float64), B[:q].astype(np.float64))
    C[:q] = (-dot * (1.0 + rng.uniform(-1e-3, 1e-3, size=dot.shape))).astype(np.float32)
    return A, B, C


def _lanes(kind, A, B, C):
    """per-lane operand arrays in the probe's input order"""
    n = A.shape[0]
    l = np.arange(64)
    g, li = l // 16, l % 16
    if kind == "f32":
        a = A[:, li, g]  # [n, 64]
        b = B[:, g, li]
    else:
        j = np.arange(8)
        a = A[:, li[:, None], 8 * g[:, None] + j[None, :]]  # [n, 64, 8]
        b = B[:, 8 * g[:, None] + j[None, :], li[:, None]]
        a = (a.view(np.uint32) >> 16).astype(np.uint16)
        b = (b.view(np.uint32) >> 16).astype(np.uint16)
    r = np.arange(4)
    c = C[:, 4 * g[:, None] + r[None, :], li[:, None]]  # [n, 64, 4]
    return a, b, c


def gen(kind, n, path, seed=5):
    rng = np.random.default_rng(seed)
    A, B, C = _operands(kind, n, rng)
    a, b, c = _lanes(kind, A, B, C)
    with open(path, "wb") as f:
        f.write(struct.pack("ii", 0 if kind == "f32" else 1, n))
        f.write(np.ascontiguousarray(a).tobytes())
        f.write(np.ascontiguousarray(b).tobytes())
        f.write(np.ascontiguousarray(c, dtype=np.float32).tobytes())
    np.savez(path + ".npz", A=A, B=B, C=C)


def _f32(x):
    return float(np.float32(x))


def _fma32(a, b, c):
    # correctly rounded fp32 fma: the exact a*b + c (fsum of exact double terms) rounded once to fp32 (a double-rounding
    # tie has probability ~2^-29 per operation)
    return _f32(math.fsum((float(a) * float(b), float(c))))


def models(kind, A, B, C, i, j, t):
    K = A.shape[2]
    a = [float(A[t, i, k]) for k in range(K)]
    b = [float(B[t, k, j]) for k in range(K)]
    c = float(C[t, i, j])
    out = {}
    acc = c
    for k in range(K):
        acc = _fma32(a[k], b[k], acc)
    out["chain_fma"] = acc
    acc = c
    for k in reversed(range(K)):
        acc = _fma32(a[k], b[k], acc)
    out["chain_fma_rev"] = acc
    prods = [a[k] * b[k] for k in range(K)]
    out["exact_round"] = _f32(math.fsum(prods + [c]))
    out["exact_prod_then_c"] = _f32(_f32(math.fsum(prods)) + c)
    acc = c
    for k in range(K):
        acc = _f32(acc + _f32(a[k] * b[k]))
    out["chain_mul_add"] = acc
    if kind == "bf16":
        # groups of 4 / 8 / 16 products exact, rounded, chained onto the accumulator in k order
        for G in (2, 4, 8, 16):
            acc = c
            for k0 in range(0, K, G):
                acc = _f32(math.fsum(prods[k0:k0 + G] + [acc]))
            out[f"exact_groups{G}_onto_acc"] = acc
    return out


def check(kind, inp, outp, limit=400):
    d = np.load(inp + ".npz")
    A, B, C = d["A"], d["B"], d["C"]
    n = A.shape[0]
    D = np.fromfile(outp, dtype=np.float32).reshape(n, 64, 4)
    l = np.arange(64)
    g, li = l // 16, l % 16
    Dm = np.zeros((n, 16, 16), np.float32)
    for r in range(4):
        Dm[:, 4 * g + r, li] = D[:, :, r]
    hits, tot = {}, 0
    for t in range(min(n, limit)):
        for i in range(16):
            for j in range(16):
                m = models(kind, A, B, C, i, j, t)
                tot += 1
                for k, v in m.items():
                    hits[k] = hits.get(k, 0) + (np.float32(v) == Dm[t, i, j])
    for k, v in sorted(hits.items(), key=lambda kv: -kv[1]):
        print(f"{kind} {k:24s} {v}/{tot} = {v / tot:.6f}")


if __name__ == "__main__":
    if sys.argv[1] == "gen":
        gen(sys.argv[2], int(sys.argv[3]), sys.argv[4])
    else:
        check(sys.argv[2], sys.argv[3], sys.argv[4])
