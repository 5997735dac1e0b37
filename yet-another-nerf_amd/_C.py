"""ctypes binding of libyanerf_hip.so (C ABI declared in include/yanerf_hip.h).

The HIP library is the ONLY compute path of this package: if it is missing or fails to load, importing
the ops raises immediately (there is no CPU or torch fallback).
"""
from __future__ import annotations

import ctypes
import hashlib
import os
from ctypes import POINTER, Structure, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_uint32, c_uint64, c_void_p
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("YANERF_HIP_LIB", PKG / "libyanerf_hip.so"))
# the files the library's build id hashes, in the Makefile's order (csrc/Makefile: SRC_SHA)
SOURCES = [PKG / "csrc" / f for f in ("render.hip", "mlp.hip", "common.hpp")] + [
    PKG.parent / "include" / "yanerf_hip.h", PKG / "csrc" / "Makefile"]


def source_id() -> str:
    """SHA-256 prefix of the HIP sources in this tree (what a library built from them reports as its build id)."""
    h = hashlib.sha256()
    for f in SOURCES:
        h.update(f.read_bytes())
    return h.hexdigest()[:16]

PREC_F32 = 0
PREC_BF16 = 1
PREC_F32X3 = 2  # fp32 as three bf16 terms, six bf16 MFMAs per product (include/yanerf_hip.h)
PREC_BF16S = 3  # bf16 with bf16 storage throughout (no fp8 sections; include/yanerf_hip.h)

# every symbol include/yanerf_hip.h declares (checked by tests/test_capi.py)
EXPORTS = (
    "yanerf_last_error", "yanerf_version", "yanerf_build_id", "yanerf_raygen", "yanerf_mlp_num_params",
    "yanerf_mlp_packed_bytes",
    "yanerf_mlp_pack", "yanerf_mlp_pack_multi", "yanerf_mlp_saved_bytes", "yanerf_mlp_bwd_workspace_bytes",
    "yanerf_mlp_dw_plan", "yanerf_mlp_forward",
    "yanerf_mlp_backward", "yanerf_mlp_backward_phase", "yanerf_composite_forward", "yanerf_composite_backward",
    "yanerf_composite_train", "yanerf_sample_pdf",
    "yanerf_refine", "yanerf_rgb_loss", "yanerf_adam", "yanerf_adam_scalars", "yanerf_adam_table", "yanerf_step_advance",
    "yanerf_scatter_rays",
)


class MlpDesc(Structure):
    _fields_ = [
        ("n_layers", c_int32), ("skip_mask", c_uint32), ("n_freq_xyz", c_int32), ("n_freq_dir", c_int32),
        ("append_xyz", c_int32), ("append_dir", c_int32), ("hidden_xyz", c_int32), ("hidden_dir", c_int32),
        ("color_dim", c_int32),
    ]


class RaymarchOpts(Structure):
    _fields_ = [
        ("capping", c_int32), ("weight_fn", c_int32), ("blend_output", c_int32), ("hard_background", c_int32),
        ("density_relu", c_int32), ("background_opacity", c_float), ("background_density_bias", c_float),
        ("bg_default", c_float * 4), ("bg_default_n", c_int32), ("noise_mode", c_int32), ("noise_std", c_float),
        ("seed", c_uint64), ("offset", c_uint64), ("rng_base", c_void_p),
    ]


class HipError(RuntimeError):
    pass


_lib = None


def lib():
    """Load (once) and return the HIP library; raise HipError if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise HipError(
            f"libyanerf_hip.so not found at {LIB_PATH}; build it with `python -c \"import __graft_entry__ as g; "
            f"g.build()\"` or `make -C yet-another-nerf_amd/csrc`. There is no CPU fallback."
        )
    L = ctypes.CDLL(str(LIB_PATH))
    P = c_void_p
    i64 = c_int64
    sig = {
        "yanerf_last_error": (c_char_p, []),
        "yanerf_version": (c_int, []),
        "yanerf_build_id": (c_char_p, []),
        "yanerf_raygen": (c_int, [P, P, P, P, i64, i64, i64, i64, c_float, c_float, c_float, c_float, i64, c_int, P,
                                  c_uint64, c_uint64, P, P, P, P, P, P, P, P]),
        "yanerf_mlp_num_params": (c_int, [POINTER(MlpDesc)]),
        "yanerf_mlp_packed_bytes": (i64, [POINTER(MlpDesc), c_int]),
        "yanerf_mlp_pack": (c_int, [POINTER(MlpDesc), c_int, P, P, P]),
        "yanerf_mlp_pack_multi": (c_int, [c_int, POINTER(MlpDesc), c_int, P, P, P]),
        "yanerf_mlp_saved_bytes": (i64, [POINTER(MlpDesc), c_int, i64]),
        "yanerf_mlp_bwd_workspace_bytes": (i64, [POINTER(MlpDesc), c_int, i64]),
        "yanerf_mlp_dw_plan": (c_int, [POINTER(MlpDesc), c_int, i64, POINTER(c_int), POINTER(c_int), POINTER(i64),
                                       POINTER(i64), POINTER(i64)]),
        "yanerf_mlp_forward": (c_int, [POINTER(MlpDesc), c_int, P, P, P, P, i64, i64, P, P, P, P]),
        "yanerf_mlp_backward": (c_int, [POINTER(MlpDesc), c_int, P, P, P, P, P, i64, i64, P, P, P]),
        "yanerf_mlp_backward_phase": (c_int, [POINTER(MlpDesc), c_int, P, P, P, P, P, i64, i64, P, P, c_int, P]),
        "yanerf_composite_forward": (c_int, [POINTER(RaymarchOpts), P, P, P, P, P, P, i64, i64, i64, P, P, P, P, P]),
        "yanerf_composite_backward": (c_int, [POINTER(RaymarchOpts), P, P, P, P, P, P, P, P, P, i64, i64, i64, P, P,
                                              P]),
        "yanerf_composite_train": (c_int, [POINTER(RaymarchOpts), P, P, P, P, P, P, P, P, i64, i64, i64, i64, i64,
                                           i64, c_float, P, P, P, P, P, P, P, P, P]),
        "yanerf_sample_pdf": (c_int, [P, P, i64, i64, i64, c_int, P, c_uint64, c_uint64, P, P]),
        "yanerf_refine": (c_int, [P, P, i64, i64, i64, c_int, P, c_uint64, c_uint64, c_int, P, P, P]),
        "yanerf_rgb_loss": (c_int, [P, P, P, i64, i64, i64, i64, i64, c_float, P, P, P]),
        "yanerf_scatter_rays": (c_int, [P, P, i64, i64, i64, i64, i64, P, P, P, P]),
        "yanerf_adam": (c_int, [P, P, P, P, i64, c_double, c_double, c_double, c_double, c_double, i64, P]),
        "yanerf_adam_scalars": (c_int, [c_double, c_double, c_double, i64, POINTER(c_float)]),
        "yanerf_adam_table": (c_int, [P, P, P, P, i64, P, P, c_double, c_double, c_double, c_double, i64, P]),
        "yanerf_step_advance": (c_int, [P, c_uint64, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if "YANERF_HIP_LIB" not in os.environ:  # an explicitly chosen library (A/B builds) is taken as given
        built, src = L.yanerf_build_id().decode(), source_id()
        if built != src:
            raise HipError(f"{LIB_PATH} was built from other sources (build id {built}, sources {src}): rebuild it with "
                           f"`python -c \"import __graft_entry__ as g; g.build()\"`")
    _lib = L
    return L


def check(status: int, what: str) -> None:
    if status != 0:
        msg = lib().yanerf_last_error().decode(errors="replace")
        raise HipError(f"{what} failed: {msg}")


def dw_plan(desc: MlpDesc, precision: int, n_points: int) -> dict:
    """The split-K weight-gradient plan for n_points (yanerf_mlp_dw_plan): tiles, splits, points per stage and the
    stages per split."""
    t, s = c_int(), c_int()
    sp, lo, hi = c_int64(), c_int64(), c_int64()
    check(lib().yanerf_mlp_dw_plan(ctypes.byref(desc), precision, int(n_points), ctypes.byref(t), ctypes.byref(s),
                                   ctypes.byref(sp), ctypes.byref(lo), ctypes.byref(hi)), "yanerf_mlp_dw_plan")
    return dict(tiles=t.value, splits=s.value, stage_points=sp.value, stages_per_split=[lo.value, hi.value],
                points_per_split=[lo.value * sp.value, hi.value * sp.value])


def ptr_array(ptrs):
    """Host array of device pointers (for the params/grads tables)."""
    arr = (c_void_p * len(ptrs))(*ptrs)
    return arr
