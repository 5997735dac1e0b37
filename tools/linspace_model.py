"""torch.linspace (CPU, float32) is the scalar formula with fused multiply-adds: start + step * i on the first half,
end - step * (n - 1 - i) on the second (aten linspace_kernel, contracted by the compiler), bit for bit -- the model
csrc/common.hpp torch_linspace_at and oracle.torch_linspace implement. Checks it against torch on random
(start, end, n).    python tools/linspace_model.py [cases]"""
import sys

import numpy as np
import torch


def model(a, b, n):
    a, b = np.float32(a), np.float32(b)
    if n == 1:
        return np.array([a], np.float32)
    s = np.float32((b - a) / np.float32(n - 1))
    i = np.arange(n, dtype=np.float64)
    return np.where(np.arange(n) < n // 2, np.float64(s) * i + np.float64(a),
                    -np.float64(s) * (n - 1 - i) + np.float64(b)).astype(np.float32)


if __name__ == "__main__":
    rng = np.random.default_rng(0)
    bad = tot = 0
    for k in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3000):
        a = float(rng.uniform(-10, 10))
        b = a + float(rng.uniform(0.01, 20))
        n = int(rng.integers(1, 300))
        t = torch.linspace(a, b, n).numpy()
        bad += int((t != model(a, b, n)).sum())
        tot += n
    print(f"linspace model: {bad} mismatches of {tot} values")
