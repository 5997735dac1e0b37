#!/usr/bin/env python
"""Which float arithmetic does torch.optim.Adam (foreach, on the GPU; and the CPU single-tensor path) use per
element? Emulates one Adam step in numpy with/without fused multiply-adds at each of the three contractible sites
(lerp, addcmul, addcdiv) and reports which emulation matches torch bit for bit. Used to pin yanerf_adam's
arithmetic (render.hip adam_kernel) to torch's."""
import itertools
import json
import sys

import numpy as np
import torch


def fma32(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


FLAGS = ("lerp_fma", "addcmul_fma", "wd_fma", "div_by_reciprocal", "addcdiv_fma", "addcdiv_scale_first",
         "addcmul_gg_first")


def emulate(p, g, m, v, step, lr, b1, b2, eps, wd, f_lerp, f_cmul, f_wd, f_recip, f_cdiv, f_sf, f_gg):
    f32 = np.float32
    if wd != 0:
        g = fma32(np.full_like(p, f32(wd)), p, g) if f_wd else (g + (f32(wd) * p).astype(np.float32)).astype(f32)
    w1 = f32(1 - b1)
    d = (g - m).astype(np.float32)
    m2 = fma32(np.full_like(d, w1), d, m) if f_lerp else (m + (w1 * d).astype(np.float32)).astype(np.float32)
    v1 = (v * f32(b2)).astype(np.float32)
    if f_gg:  # foreach addcmul: self + value * (t1 * t2)
        gg = (g * g).astype(np.float32)
        v2 = fma32(np.full_like(gg, f32(1 - b2)), gg, v1) if f_cmul else \
            (v1 + (f32(1 - b2) * gg).astype(np.float32)).astype(np.float32)
    else:
        a2 = (f32(1 - b2) * g).astype(np.float32)
        v2 = fma32(a2, g, v1) if f_cmul else (v1 + (a2 * g).astype(np.float32)).astype(np.float32)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    ss = f32(-(lr / bc1))
    sq = np.sqrt(v2).astype(np.float32)
    if f_recip:
        den = (sq * (f32(1.0) / f32(bc2 ** 0.5))).astype(np.float32)
    else:
        den = (sq / f32(bc2 ** 0.5)).astype(np.float32)
    den = (den + f32(eps)).astype(np.float32)
    if f_sf:  # CPU addcdiv: self + value * t1 / t2 = self + ((value * t1) / t2)
        if f_cdiv:
            return None, m2, v2
        p2 = (p + ((ss * m2).astype(np.float32) / den).astype(np.float32)).astype(np.float32)
        return p2, m2, v2
    q = (m2 / den).astype(np.float32)
    p2 = fma32(np.full_like(q, ss), q, p) if f_cdiv else (p + (ss * q).astype(np.float32)).astype(np.float32)
    return p2, m2, v2


def main():
    dev = sys.argv[1] if len(sys.argv) > 1 else "cuda"
    rng = np.random.default_rng(0)
    n = 1 << 16
    res = {}
    for wd in (0.0, 0.01):
        p0 = rng.standard_normal(n).astype(np.float32)
        out = {}
        for foreach in ((True, False) if dev != "cpu" else (False,)):
            p = torch.nn.Parameter(torch.from_numpy(p0.copy()).to(dev))
            opt = torch.optim.Adam([p], lr=5e-4, weight_decay=wd, foreach=foreach)
            pn, mn, vn = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
            matches = {}
            for step in range(1, 4):
                g = (rng.standard_normal(n) * 1e-3).astype(np.float32)
                p.grad = torch.from_numpy(g).to(dev)
                opt.step()
                tp = p.detach().cpu().numpy().copy()
                st = opt.state[p]
                tm, tv = st["exp_avg"].cpu().numpy().copy(), st["exp_avg_sq"].cpu().numpy().copy()
                for flags in itertools.product((0, 1), repeat=len(FLAGS)):
                    e = emulate(pn, g, mn, vn, step, 5e-4, 0.9, 0.999, 1e-8, wd, *flags)
                    ok = [int((a.view(np.int32) == b.view(np.int32)).sum()) if a is not None else -1
                          for a, b in zip(e, (tp, tm, tv))]
                    matches.setdefault(str(flags), []).append(ok)
                pn, mn, vn = tp, tm, tv  # continue from torch's state
            out[f"foreach={foreach}"] = matches
        res[f"wd={wd}"] = out
    full, best = {}, {}
    for wd, o in res.items():
        for k, m in o.items():
            full[f"{wd} {k}"] = [dict(zip(FLAGS, eval(fl))) for fl, v in m.items()
                                 if all(x == n for step in v for x in step)]
            ranked = sorted(m.items(), key=lambda kv: -sum(x for step in kv[1] for x in step))[:4]
            best[f"{wd} {k}"] = [(dict(zip(FLAGS, eval(fl))), v) for fl, v in ranked]
    print(json.dumps({"device": dev, "n": n, "bit_exact_emulations": full, "best": best}))


if __name__ == "__main__":
    main()
