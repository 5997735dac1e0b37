"""The C-ABI library builds, loads without a GPU and exports every entry point include/yanerf_hip.h declares;
host-side argument validation and size queries behave (no kernel launches here)."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

import yanerf_boot  # noqa: F401
from yanerf_amd import _C

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "yanerf_hip.h"


def header_functions():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int64_t|int)\s+(yanerf_\w+)\s*\(", text, re.M)))


def test_header_and_binding_agree():
    assert set(header_functions()) == set(_C.EXPORTS)


def test_library_exports_every_symbol():
    lib = _C.lib()
    for name in header_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(_C.LIB_PATH)], capture_output=True, text=True, check=True)
    exported = {line.split()[-1] for line in out.stdout.splitlines() if " T " in line}
    missing = set(header_functions()) - exported
    assert not missing, missing


def test_struct_layout_matches_c(tmp_path):
    """ctypes structs == the C header's layout (compiled with gcc against include/yanerf_hip.h)."""
    src = tmp_path / "layout.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "yanerf_hip.h"\n'
        "int main(){printf(\"%zu %zu %zu %zu %zu\\n\", sizeof(yanerf_mlp_desc), sizeof(yanerf_raymarch_opts),"
        " offsetof(yanerf_raymarch_opts, bg_default), offsetof(yanerf_raymarch_opts, seed),"
        " offsetof(yanerf_raymarch_opts, noise_std));return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals == [ctypes.sizeof(_C.MlpDesc), ctypes.sizeof(_C.RaymarchOpts), _C.RaymarchOpts.bg_default.offset,
                    _C.RaymarchOpts.seed.offset, _C.RaymarchOpts.noise_std.offset]


def lego_desc(**kw):
    d = dict(n_layers=8, skip_mask=1 << 5, n_freq_xyz=10, n_freq_dir=4, append_xyz=1, append_dir=1, hidden_xyz=256,
             hidden_dir=128, color_dim=3)
    d.update(kw)
    return _C.MlpDesc(*d.values())


def test_mlp_size_queries():
    L = _C.lib()
    d = lego_desc()
    assert L.yanerf_mlp_num_params(ctypes.byref(d)) == 24
    f32 = L.yanerf_mlp_packed_bytes(ctypes.byref(d), _C.PREC_F32)
    bf = L.yanerf_mlp_packed_bytes(ctypes.byref(d), _C.PREC_BF16)
    assert f32 > bf > 0
    # saved activations grow with the point count, rounded up to the kernel's point tile; rows are padded to an
    # odd multiple of 256 B (HBM channel spread), so the size is ~linear, never below the unpadded bytes
    s1 = L.yanerf_mlp_saved_bytes(ctypes.byref(d), _C.PREC_F32, 64)
    s2 = L.yanerf_mlp_saved_bytes(ctypes.byref(d), _C.PREC_F32, 128)
    assert s1 < s2 and L.yanerf_mlp_saved_bytes(ctypes.byref(d), _C.PREC_F32, 65) == s2
    rows = 64 + 256 * 8 + 256 + 32 + 128  # PE | 8 trunk layers | Y | dir PE | colour hidden
    assert s2 >= rows * 128 * 4 + 9 * 128 * 32
    assert L.yanerf_mlp_bwd_workspace_bytes(ctypes.byref(d), _C.PREC_BF16, 1 << 20) > 0


def test_dw_plan_query():
    """yanerf_mlp_dw_plan (host only): the split-K plan the backward launches with. At the headline fine pass (4096 rays
    x 192 points) every split reduces hundreds of stages; every point is in exactly one split."""
    d = lego_desc()
    n = 4096 * 192
    for prec in (_C.PREC_F32, _C.PREC_F32X3, _C.PREC_BF16):
        p = _C.dw_plan(d, prec, n)
        lo, hi = p["stages_per_split"]
        assert p["tiles"] > 0 and 1 <= p["splits"] and lo <= hi <= lo + 1 and lo >= 100, (prec, p)
        nst = -(-n // p["stage_points"])
        assert lo * p["splits"] <= nst <= hi * p["splits"], (prec, p)
    # bf16: whole rounds of one workgroup per CU, as many rounds as the fp8 scale slots need (configs[4]'s 320-point
    # fine pass needs two)
    b1, b2 = _C.dw_plan(d, _C.PREC_BF16, n), _C.dw_plan(d, _C.PREC_BF16, 4096 * 320)
    assert b1["tiles"] * b1["splits"] <= 256 < b1["tiles"] * b2["splits"] <= 512, (b1, b2)
    assert _C.dw_plan(d, _C.PREC_BF16, 48 * 192)["stages_per_split"][1] < 16  # the 48-ray golden: a few stages
    assert L_error_on_bad_plan()


def L_error_on_bad_plan() -> bool:
    L = _C.lib()
    i, s = ctypes.c_int(), ctypes.c_int()
    a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    rc = L.yanerf_mlp_dw_plan(ctypes.byref(lego_desc()), 1, -5, ctypes.byref(i), ctypes.byref(s), ctypes.byref(a),
                              ctypes.byref(b), ctypes.byref(c))
    return rc == 1 and "n_points" in L.yanerf_last_error().decode()


@pytest.mark.parametrize("bad,msg", [
    (dict(n_freq_xyz=11), "xyz embedding"), (dict(n_freq_dir=5), "dir embedding"), (dict(hidden_xyz=300), "xyz"),
    (dict(hidden_dir=256), "dir"), (dict(n_layers=0), "n_layers"), (dict(color_dim=5), "color_dim"),
    (dict(skip_mask=1), "skip")])
def test_mlp_desc_validation(bad, msg):
    L = _C.lib()
    d = lego_desc(**bad)
    assert L.yanerf_mlp_num_params(ctypes.byref(d)) == -1
    assert msg in L.yanerf_last_error().decode()


def test_argument_validation_returns_error_without_launch():
    L = _C.lib()
    o = _C.RaymarchOpts()
    o.bg_default_n = 1
    assert L.yanerf_composite_forward(ctypes.byref(o), None, None, None, None, None, None, 4, 1000, 3, None, None,
                                      None, None, None) == 1
    assert "P=1000" in L.yanerf_last_error().decode()
    assert L.yanerf_refine(None, None, 4, 2, 8, 1, None, 0, 0, 1, None, None, None) == 1
    assert L.yanerf_raygen(None, None, None, None, 1, 1, 1, 1, 1.0, 1.0, 0.0, 1.0, 4, 0, None, 0, 0, None, None, None,
                           None, None, None, None, None) == 1


def test_mlp_backward_phase_validation():
    """yanerf_mlp_backward_phase rejects a phase outside 1..3 and null buffers before any launch."""
    L = _C.lib()
    d = lego_desc()
    dummy = ctypes.c_void_p(16)
    grads = (ctypes.c_void_p * 32)(*([16] * 32))
    args = [ctypes.byref(d), 0, dummy, dummy, dummy, dummy, dummy, 4, 64, grads, dummy]
    assert L.yanerf_mlp_backward_phase(*args, 0, None) == 1
    assert "phase 0" in L.yanerf_last_error().decode()
    assert L.yanerf_mlp_backward_phase(*args, 4, None) == 1
    args[2] = None
    assert L.yanerf_mlp_backward_phase(*args, 1, None) == 1
    assert "null" in L.yanerf_last_error().decode()


def test_composite_noise_mode_needs_noise():
    """noise_mode 1 (injected density noise) with a null noise pointer is an argument error in every composite entry
    point (no launch, so no device null dereference)."""
    L = _C.lib()
    o = _C.RaymarchOpts()
    o.bg_default_n = 1
    o.noise_mode = 1
    d = ctypes.c_void_p(16)
    assert L.yanerf_composite_forward(ctypes.byref(o), d, d, d, d, None, None, 4, 8, 3, d, d, d, d, None) == 1
    assert "needs noise" in L.yanerf_last_error().decode()
    assert L.yanerf_composite_backward(ctypes.byref(o), d, d, d, d, None, None, d, None, None, 4, 8, 3, d, d,
                                       None) == 1
    assert "needs noise" in L.yanerf_last_error().decode()
    assert L.yanerf_composite_train(ctypes.byref(o), d, d, d, d, None, None, d, d, 1, 4, 8, 3, 8, 8, 1.0, d, d, d, d,
                                    d, d, d, d, None) == 1
    assert "needs noise" in L.yanerf_last_error().decode()


def test_mlp_pack_multi_validation():
    """yanerf_mlp_pack_multi rejects an empty model list, a bad descriptor, a bad precision and null parameter /
    buffer pointers before any launch (CPU: nothing reaches the device)."""
    L = _C.lib()
    d = (_C.MlpDesc * 2)(lego_desc(), lego_desc())
    prm = (ctypes.c_void_p * 24)(*([16] * 24))
    tables = _C.ptr_array([ctypes.addressof(prm), ctypes.addressof(prm)])
    dst = _C.ptr_array([16, 16])
    assert L.yanerf_mlp_pack_multi(0, d, _C.PREC_BF16, tables, dst, None) == 1
    assert "bad arguments" in L.yanerf_last_error().decode()
    assert L.yanerf_mlp_pack_multi(2, d, 7, tables, dst, None) == 1
    assert "precision" in L.yanerf_last_error().decode()
    bad = (_C.MlpDesc * 2)(lego_desc(), lego_desc(n_layers=0))
    assert L.yanerf_mlp_pack_multi(2, bad, _C.PREC_BF16, tables, dst, None) == 1
    assert "n_layers" in L.yanerf_last_error().decode()
    assert L.yanerf_mlp_pack_multi(2, d, _C.PREC_BF16, tables, _C.ptr_array([16, 0]), None) == 1
    assert "model 1" in L.yanerf_last_error().decode()
    prm0 = (ctypes.c_void_p * 24)(*([16] * 23 + [0]))
    assert L.yanerf_mlp_pack_multi(2, d, _C.PREC_BF16, _C.ptr_array([ctypes.addressof(prm), ctypes.addressof(prm0)]),
                                   dst, None) == 1
    assert "parameter 23 is null" in L.yanerf_last_error().decode()


def test_integration_stub_struct_matches_the_c_layout():
    """The ctypes stub INTEGRATION.md shows a maintainer (its RaymarchOpts mirror) has the field names, offsets and size
    of the binding the package uses, whose layout test_struct_layout_matches_c pins to the C header."""
    import re
    from pathlib import Path
    text = (Path(__file__).resolve().parents[1] / "INTEGRATION.md").read_text()
    block = re.search(r"```python\n(.*?)```", text[text.index("### ctypes stub"):], re.S).group(1)
    src = block[block.index("class RaymarchOpts"):block.index("def composite_forward")]
    ns = {"ctypes": ctypes}
    exec(src, ns)
    doc, ours = ns["RaymarchOpts"], _C.RaymarchOpts
    assert ctypes.sizeof(doc) == ctypes.sizeof(ours)
    assert [f[0] for f in doc._fields_] == [f[0] for f in ours._fields_]
    for (name, _), (_, _) in zip(doc._fields_, ours._fields_):
        assert getattr(doc, name).offset == getattr(ours, name).offset, name
