"""CPU pins of the numerical models the round-5 parity work rests on (no GPU):

* the MI355X's v_mfma_f32_16x16x4_f32 is a fused multiply-add chain over its four lane groups -- checked against 300
  hardware-measured tiles (tests/golden/mfma_f32_probe.npz, tools/probes/probe_mfma_order.hip);
* tests/golden/mfma_order.c (the reference trial in the HIP kernels' order, make_golden.hip_order_model) implements
  that chain for a whole Linear layer;
* torch.linspace (CPU, float32) is the fused-multiply-add scalar formula that oracle.torch_linspace and the ray
  generation kernel implement;
* parity_gates.split_gate's set-membership assertion."""
import ctypes
import subprocess
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O
from parity_gates import split_gate

GOLDEN = Path(__file__).resolve().parent / "golden"


def _fma32(a, b, c):
    # a * b is exact in float64 for float32 operands; the add rounds in double, then to float32 (a double-rounding
    # tie never occurred on these data)
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def test_f32_mfma_is_an_fma_chain_over_lane_groups(golden):
    g = golden("mfma_f32_probe")
    A, B, C, D = g["A"], g["B"], g["C"], g["D"]  # [t,16,4], [t,4,16], [t,16,16], [t,16,16]
    acc = C.copy()
    for k in range(4):  # lane group g = k
        acc = _fma32(A[:, :, k][:, :, None], B[:, k, :][:, None, :], acc)
    assert np.array_equal(acc, D)
    # the exactly rounded dot product is NOT what the hardware computes (so the order matters)
    exact = (np.einsum("tik,tkj->tij", A.astype(np.float64), B.astype(np.float64)) + C).astype(np.float32)
    assert (exact != D).any()


@pytest.fixture(scope="module")
def hip_order_lib(tmp_path_factory):
    so = tmp_path_factory.mktemp("mo") / "mfma_order.so"
    subprocess.run(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", "-o", str(so), str(GOLDEN / "mfma_order.c"), "-lm"],
                   check=True)
    lib = ctypes.CDLL(str(so))
    lib.hip_order_linear.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return lib


@pytest.mark.parametrize("K,bias_first", [(63, 1), (256, 1), (319, 1), (283, 1), (256, 0), (128, 0)])
def test_mfma_order_c_is_the_kernel_chain(hip_order_lib, K, bias_first):
    """hip_order_linear = bias (or 0, bias added after) then, per 16-wide K-block kb, k-steps s = 0..3, lane groups
    g = 0..3: acc = fma(W[n][16kb + 4g + s], x[m][16kb + 4g + s], acc) -- the fp32 GEMM of csrc/mlp.hip."""
    rng = np.random.default_rng(K + bias_first)
    M, N = 37, 20
    x = rng.standard_normal((M, K)).astype(np.float32)
    w = (rng.standard_normal((N, K)) * 0.1).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    y = np.empty((M, N), np.float32)
    hip_order_lib.hip_order_linear(x.ctypes.data, M, K, w.ctypes.data, N, b.ctypes.data, bias_first, 0, y.ctypes.data)
    acc = np.broadcast_to(b if bias_first else np.zeros(N, np.float32), (M, N)).astype(np.float32)
    for kb in range((K + 15) // 16):
        for s in range(4):
            for gg in range(4):
                k = 16 * kb + 4 * gg + s
                if k < K:
                    acc = _fma32(x[:, k][:, None], w[:, k][None, :], acc)
    if not bias_first:
        acc = (acc + b).astype(np.float32)
    assert np.array_equal(y, acc)


def test_oracle_linspace_is_torch_linspace():
    rng = np.random.default_rng(3)
    for _ in range(300):
        a = float(rng.uniform(-10, 10))
        b = a + float(rng.uniform(0.01, 20))
        n = int(rng.integers(1, 300))
        assert np.array_equal(O.torch_linspace(a, b, n), torch.linspace(a, b, n).numpy()), (a, b, n)
    for a, b, n in ((2.0, 6.0, 64), (1.3125, 7.25, 64), (0.0, 1.0, 128), (0.0, 799.0, 800)):
        assert np.array_equal(O.torch_linspace(a, b, n), torch.linspace(a, b, n).numpy())


def test_split_gate_asserts_set_membership(tmp_path, monkeypatch):
    """A ray with other refined depths outside every trial set of the reference's sensitivity golden fails the gate;
    inside one, it passes (and in hip_exact mode it must be inside the hip-arithmetic trial's set)."""
    import parity_gates
    monkeypatch.setattr(parity_gates, "REPORTS", tmp_path / "reports.jsonl")
    R, P = 4, 3
    z_ref = np.tile(np.linspace(2, 6, P, dtype=np.float32), (R, 1))
    z = z_ref.copy()
    z[1] += 1e-3  # ray 1 moved
    rgb = np.zeros((R, 3), np.float32)

    def fine_at(rows, zz):
        return np.zeros((len(rows), 3)), np.zeros(len(rows))

    class _O:  # the refinement of "our" weights reproduces z exactly
        @staticmethod
        def refine(zc, w, n, random_sampling=False):
            return z

    sens = dict(z_fine=z_ref, z_fine_f64=z_ref.astype(np.float64), max_z_move=np.zeros(R, np.float32),
                max_z_move_hip_order=np.zeros(R, np.float32), max_z_move_weights=np.zeros(R, np.float32))
    kw = dict(fine_at=fine_at, coarse=(_O, z_ref, np.zeros((R, P)), P))
    with pytest.raises(AssertionError):
        split_gate(rgb, rgb, z, z_ref, sensitivity=sens, tag="cpu-outside", **kw)
    sens["max_z_move_weights"] = np.array([0, 1, 0, 0], np.float32)
    # inside the weight-perturbation trial alone: a diagnostic, not a bound -- allowed only when budgeted
    with pytest.raises(AssertionError):
        split_gate(rgb, rgb, z, z_ref, sensitivity=sens, tag="cpu-weights-only", **kw)
    split_gate(rgb, rgb, z, z_ref, sensitivity=sens, tag="cpu-weights-only", max_outside_without_weights=1, **kw)
    sens["max_z_move"] = np.array([0, 1, 0, 0], np.float32)
    split_gate(rgb, rgb, z, z_ref, sensitivity=sens, tag="cpu-inside", **kw)
    with pytest.raises(AssertionError):
        split_gate(rgb, rgb, z, z_ref, sensitivity=sens, tag="cpu-hip-exact", hip_exact=True, **kw)
    sens["max_z_move_hip_order"] = np.array([0, 1, 0, 0], np.float32)
    split_gate(rgb, rgb, z, z_ref, sensitivity=sens, tag="cpu-hip-exact", hip_exact=True, **kw)
