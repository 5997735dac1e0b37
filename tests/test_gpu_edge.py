"""Edge cases of the HIP path against the reference's torch semantics (needs an MI355X: marked `gpu`).

The reference is plain torch, so an empty ray bundle flows through it as empty tensors: nn.Linear on zero rows gives
zero-row outputs and all-zero parameter gradients, the raymarcher's reductions give empty features / depths, and
scatter_rays_to_image (pipelines/utils.py:299-323) returns the background image. Every entry point of the C ABI
here returns before touching its (possibly NULL) point buffers when the bundle is empty, and the MLP backward writes
zero gradients, checked with guard zones around every gradient buffer.
"""
import ctypes

import numpy as np
import pytest
import torch

from weights import LEGO_ARCH, SMALL_ARCH, make_nerf_mlp_params

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def ops():
    import yanerf_amd.ops as ops_
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return ops_


def build(arch, precision, seed=3):
    from yanerf_amd.pipelines.models import MODELS
    m = MODELS.build(dict(type="NeRFMLP", **arch, precision=precision)).to(DEV)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in make_nerf_mlp_params(arch, seed).items()})
    return m


@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp32x3", "bf16s"])
def test_empty_bundle_through_the_mlp(ops, precision):
    """NeRFMLP.forward on a [1, 0, P] bundle: [1, 0, P, 1] densities and [1, 0, P, 3] colours, and a backward through
    them gives every parameter an all-zero gradient, as nn.Linear does on an empty batch."""
    m = build(LEGO_ARCH, precision)
    o = torch.zeros(1, 0, 3, device=DEV)
    d = torch.zeros(1, 0, 3, device=DEV)
    z = torch.zeros(1, 0, 64, device=DEV)
    out = m(o, d, z)
    assert out["rays_densities"].shape == (1, 0, 64, 1) and out["rays_features"].shape == (1, 0, 64, 3)
    (out["rays_densities"].sum() + out["rays_features"].sum()).backward()
    torch.cuda.synchronize()
    for name, p in m.named_parameters():
        assert p.grad is not None and bool((p.grad == 0).all()), name


def test_empty_backward_zeroes_exactly_the_gradients(ops):
    """yanerf_mlp_backward with R = 0 and NULL point buffers: each gradient buffer (a slice of one NaN-filled block with
    a 64-float guard after it) is zeroed over exactly its parameter's size, the guards stay NaN, for the Lego and the
    small reference architecture."""
    from yanerf_amd import _C
    L = _C.lib()
    for arch in (LEGO_ARCH, SMALL_ARCH):
        m = build(arch, "fp32")
        spec = m.spec()
        desc = spec.desc()
        shapes = [p.shape for p in m.hip_params()]
        sizes = [int(np.prod(s)) for s in shapes]
        G = 64
        block = torch.full((sum(sizes) + G * len(sizes),), float("nan"), device=DEV)
        offs = np.cumsum([0] + [s + G for s in sizes])[:-1]
        ptrs = _C.ptr_array([block[int(o):].data_ptr() for o in offs])
        for phase in (1, 4, 3):
            block.fill_(float("nan"))
            rc = L.yanerf_mlp_backward_phase(ctypes.byref(desc), spec.precision, None, None, None, None, None, 0, 64,
                                             ptrs, None, phase, ops._stream())
            assert rc == 0, L.yanerf_last_error().decode()
            torch.cuda.synchronize()
            b = block.cpu().numpy()
            for o, s in zip(offs, sizes):
                seg, guard = b[o:o + s], b[o + s:o + s + G]
                if phase == 3:  # the phases that write gradients (2, 3, 8) zero them
                    assert (seg == 0).all()
                else:  # dX / dW-only phases write none
                    assert np.isnan(seg).all()
                assert np.isnan(guard).all()


def test_empty_bundle_render_ops(ops):
    """raygen, composite (forward + backward), sample_pdf, refine and rgb_loss on zero rays: empty outputs of the
    reference's shapes, no error, nothing launched."""
    pose = torch.eye(4, device=DEV)[:3][None]
    focal = torch.tensor([100.0], device=DEV)
    o, d, z, xys, ids = ops.raygen(pose, focal, n_pts=64, near=2.0, far=6.0, cfg_w=32, cfg_h=32,
                                   pixel_ids=torch.zeros(1, 0, dtype=torch.int64, device=DEV), grid_hw=(32, 32),
                                   jitter="philox")
    assert o.shape == (1, 0, 3) and d.shape == (1, 0, 3) and z.shape == (1, 0, 64) and xys.shape == (1, 0, 2)
    sigma = torch.zeros(1, 0, 64, 1, device=DEV, requires_grad=True)
    rgb = torch.zeros(1, 0, 64, 3, device=DEV, requires_grad=True)
    f, dep, a, w = ops.composite(ops.RaymarchCfg(), sigma, rgb, z, d, noise_std=0.2)
    assert f.shape == (1, 0, 3) and dep.shape == (1, 0, 1) and a.shape == (1, 0, 1) and w.shape == (1, 0, 64)
    f.sum().backward()
    assert sigma.grad.shape == sigma.shape and rgb.grad.shape == rgb.shape
    bins = torch.zeros(0, 63, device=DEV)
    assert ops.sample_pdf(bins, torch.zeros(0, 62, device=DEV), 128).shape == (0, 128)
    assert ops.refine(z, w, 128, det=False).shape == (1, 0, 192)
    sq, g = ops.rgb_loss(torch.zeros(1, 0, 3, device=DEV), torch.rand(1, 8, 8, 3, device=DEV),
                         torch.zeros(1, 0, 2, device=DEV), 1.0)
    assert sq.shape == (1, 0) and g.shape == (1, 0, 3)
    torch.cuda.synchronize()


def test_empty_scatter_is_the_background(ops):
    """scatter_rays_to_image with no rays: the [B, H, W, C] background (zeros without a bg colour), as the reference's
    scatter onto a fresh image."""
    from yanerf_amd.pipelines.utils import scatter_rays_to_image
    v = torch.zeros(2, 0, 3, device=DEV)
    xy = torch.zeros(2, 0, 2, device=DEV)
    img = scatter_rays_to_image(v, xy, 5, 7)
    assert img.shape == (2, 5, 7, 3) and bool((img == 0).all())
    bg = torch.tensor([0.25, 0.5, 1.0], device=DEV)
    img = ops.scatter_rays(v, xy, 5, 7, bg_color=bg)
    assert bool((img == bg).all())
