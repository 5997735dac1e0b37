"""Deterministic NeRFMLP parameter sets for golden vectors and parity tests.

Test infrastructure only. The golden generator (make_golden.py, run in the
survey container against /root/reference) and the parity tests (run anywhere)
both call `make_nerf_mlp_params`, so multi-MB Lego weight tensors never need to
be committed: only the seed and a checksum travel in the fixture.

Parameter names and shapes follow the reference state_dict layout of
`NeRFMLP` (reference yanerf/pipelines/models/nerf_mlp.py:50-83, 244-261):
  xyz_encoder.mlp.{i}.0.weight / .bias, intermediate_linear.*, density_layer.*,
  color_layer.0.* (LinearWithRepeat), color_layer.2.*
The generator uses numpy's PCG64 stream, which is stable across platforms.
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import numpy as np

LEGO_ARCH = dict(
    n_layers=8, input_skips=[5], n_harmonic_functions_xyz=10, n_hidden_neurons_xyz=256,
    n_harmonic_functions_dir=4, n_hidden_neurons_dir=128, color_dim=3,
)
SMALL_ARCH = dict(  # reference tests/configs/pipelines/models/nerf_mlp.yml
    n_layers=5, input_skips=[2], n_harmonic_functions_xyz=8, n_hidden_neurons_xyz=64,
    n_harmonic_functions_dir=4, n_hidden_neurons_dir=32, color_dim=3,
)


def param_shapes(arch: dict) -> List[Tuple[str, Tuple[int, ...]]]:
    # NOTE reference quirk: NeRFMLP._construct_xyz_encoder (nerf_mlp.py:88-95) does not pass
    # `hidden_dim`, so MLPWithInputSkips keeps its default trunk width 256 (nerf_mlp.py:225) and only the
    # LAST layer outputs n_hidden_neurons_xyz (nerf_mlp.py:246).
    nl = arch["n_layers"]
    trunk = 256
    hid = arch["n_hidden_neurons_xyz"]
    # embeds = [PE(x), global code] (nerf_mlp.py:299-335): latent_dim extra input columns for layer 0 and skips
    xyz_dim = 3 * (2 * arch["n_harmonic_functions_xyz"] + 1) + arch.get("latent_dim", 0)
    dir_dim = 3 * (2 * arch["n_harmonic_functions_dir"] + 1)
    hdir = arch["n_hidden_neurons_dir"]
    out = []
    for i in range(nl):
        din = trunk if i > 0 else xyz_dim
        if i > 0 and i in arch["input_skips"]:
            din = trunk + xyz_dim
        dout = trunk if i + 1 < nl else hid
        out.append((f"xyz_encoder.mlp.{i}.0.weight", (dout, din)))
        out.append((f"xyz_encoder.mlp.{i}.0.bias", (dout,)))
    out += [
        ("intermediate_linear.weight", (hid, hid)),
        ("intermediate_linear.bias", (hid,)),
        ("density_layer.weight", (1, hid)),
        ("density_layer.bias", (1,)),
        ("color_layer.0.weight", (hdir, hid + dir_dim)),
        ("color_layer.0.bias", (hdir,)),
        ("color_layer.2.weight", (arch["color_dim"], hdir)),
        ("color_layer.2.bias", (arch["color_dim"],)),
    ]
    return out


def make_nerf_mlp_params(arch: dict, seed: int, density_bias: float = 0.1) -> Dict[str, np.ndarray]:
    rng = np.random.Generator(np.random.PCG64(seed))
    params: Dict[str, np.ndarray] = {}
    for name, shape in param_shapes(arch):
        if name.endswith("weight"):
            fan_out, fan_in = shape
            a = math.sqrt(6.0 / (fan_in + fan_out))
            params[name] = rng.uniform(-a, a, size=shape).astype(np.float32)
        else:
            fan_in = None
            wname = name[: -len("bias")] + "weight"
            fan_in = dict(param_shapes(arch))[wname][1]
            b = 1.0 / math.sqrt(fan_in)
            params[name] = rng.uniform(-b, b, size=shape).astype(np.float32)
    params["density_layer.bias"][:] = density_bias
    return params


def checksum(params: Dict[str, np.ndarray]) -> np.ndarray:
    return np.array([float(np.sum(params[k].astype(np.float64))) for k in sorted(params)], dtype=np.float64)


def load_trained_params(path=None) -> List[Dict[str, np.ndarray]]:
    """The two trained Lego-architecture MLPs (coarse, fine) of trained_weights.npz, reference state_dict names
    (keys `implicit_functions.{i}._fn.<name>` in the file; see make_golden.py TRAINED_*)."""
    from pathlib import Path
    path = Path(path) if path else Path(__file__).resolve().parent / "trained_weights.npz"
    out: List[Dict[str, np.ndarray]] = [{}, {}]
    with np.load(path, allow_pickle=False) as z:
        for k in z.files:
            i, name = int(k.split(".")[1]), k.split("._fn.", 1)[1]
            out[i][name] = z[k].astype(np.float32)
    return out
