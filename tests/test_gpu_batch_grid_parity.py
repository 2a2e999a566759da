"""The default batch-grid blend against the CPU oracle.

On grids whose backward has more than 8192 pixel blocks (every cfg 3 / cfg 4 step) the
backward runs interleaved pixel blocks (pr_blend.hip block_pixel) with the fused scalar
reduction; the forward keeps consecutive blocks.  Here a 5 x 256^2 batch (K = 8, Sr = Sa = 4:
20480 / 10240 forward / backward blocks, so the backward is interleaved) with the reference's
injected draws, packed fragments with the rasterizer's valid-prefix counts attached, is
compared with oracle/blend_oracle.py (reference smoothrast.py:39-59, smoothagg.py:44-73,
random_rasterizer.py:34-56):

* image, d dists, d zbuf, d colours (texel variant) / d bary (vertex-colour variant) at
  conftest.assert_close (1e-5 elementwise relative), the smoothing scalars at 2e-5;
* the per-slot gradients of the default layout bitwise equal to the consecutive layout's
  (PR_BLEND_INTERLEAVE=0): B6's lane split depends on the launch, not on the block's entries;
* the fused scalar reduction bitwise equal to the finalize kernel (PR_BLEND_SYNC=0 semantics via
  the module switch) and to its acq_rel-ordered form (PR_BLEND_SYNC_ORDER=release), on this grid.
"""
import os

import numpy as np
import pytest
import torch

from conftest import assert_close
from oracle import blend_oracle as bo
from pertrenderer_amd import Noise, perturbed_blend
from pertrenderer_amd.blend import perturbed_blend_vertex
from pertrenderer_amd.renderer.rasterizer import attach_valid_counts

pytestmark = pytest.mark.gpu
N, H, W, K, S = 5, 256, 256, 8, 4
SCALAR_RTOL = 2e-5


def _frags(seed, with_vertex):
    g = torch.Generator().manual_seed(seed)
    cnt = torch.randint(0, K + 1, (N, H, W), generator=g)
    cnt[:, : H // 4] = 0  # an empty band: empty blocks in the consecutive layout
    valid = torch.arange(K) < cnt[..., None]
    F_, V = 3000, 1600
    p2f = torch.where(valid, torch.randint(0, F_, (N, H, W, K), generator=g), torch.full((N, H, W, K), -1))
    dists = torch.where(valid, (torch.rand((N, H, W, K), generator=g) - 0.5) * 6e-3, torch.full((N, H, W, K), -1.0))
    zbuf = torch.where(valid, (5.0 + 2.0 * torch.rand((N, H, W, K), generator=g)).sort(-1).values,
                       torch.full((N, H, W, K), -1.0))
    f = dict(p2f=p2f, dists=dists, zbuf=zbuf, cnt=cnt.to(torch.int32))
    if with_vertex:
        b = torch.rand((N, H, W, K, 3), generator=g) + 0.05
        f["bary"] = torch.where(valid[..., None], b / b.sum(-1, keepdim=True), torch.full_like(b, -1.0))
        f["faces"] = torch.randint(0, V, (F_, 3), generator=g)
        f["vc"] = torch.rand((V, 3), generator=g)
    else:
        f["colors"] = torch.rand((N, H, W, K, 3), generator=g)
    f["nr"] = torch.randn((S, N, H, W, K), generator=g)
    f["na"] = torch.randn((S, N, H, W, K + 1), generator=g)
    f["gimg"] = torch.randn((N, H, W, 4), generator=g)
    f["zn"] = torch.tensor([1.0, 0.5, 1.0, 2.0, 1.0]).reshape(N, 1, 1, 1)
    f["zf"] = torch.tensor([100.0, 20.0, 50.0, 100.0, 80.0]).reshape(N, 1, 1, 1)
    return f


def _texels(f):
    """TexturesVertex sampling (interpolate_face_attributes) on the CPU, differentiable in bary and
    the vertex colours; padded slots give 0 colours."""
    p2f = f["p2f"]
    fc = f["vc"][f["faces"]]  # (F,3,3)
    pc = fc[p2f.clamp(min=0)]  # (N,H,W,K,3 corners,3)
    t = (f["bary"][..., None] * pc).sum(-2)
    return torch.where((p2f >= 0)[..., None], t, torch.zeros_like(t))


def _oracle(f, vertex):
    sig, gam, alp = (torch.tensor(v) for v in (1e-3, 1e-2, 1.0))
    if vertex:
        bary = f["bary"].clone().requires_grad_(True)
        vc = f["vc"].clone().requires_grad_(True)
        colors = _texels(dict(f, bary=bary, vc=vc))
    else:
        colors = f["colors"]
    img, saved = bo.blend_forward(f["p2f"], f["dists"], f["zbuf"], colors.detach(), f["nr"], f["na"], sig, gam, alp,
                                  1e-10, torch.tensor([0.1, 0.2, 0.3]), f["zn"], f["zf"])
    g = bo.blend_backward(f["gimg"], saved)
    if vertex:
        colors.backward(g["colors"])
        g["bary"] = torch.where((f["p2f"] >= 0)[..., None], bary.grad, torch.zeros_like(bary.grad))
        g["vc"] = vc.grad
    return img, g


def _gpu(f, vertex, dev):
    p2f = f["p2f"].to(dev)
    attach_valid_counts(p2f, f["cnt"].to(dev))
    d = f["dists"].to(dev).requires_grad_(True)
    z = f["zbuf"].to(dev).requires_grad_(True)
    s, gm, a = (torch.tensor(v, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
    noise = Noise.injected(f["nr"].to(dev), f["na"].to(dev))
    kw = dict(background=(0.1, 0.2, 0.3), znear=f["zn"].to(dev), zfar=f["zf"].to(dev), noise=noise)
    if vertex:
        b = f["bary"].to(dev).requires_grad_(True)
        vc = f["vc"].to(dev).requires_grad_(True)
        img = perturbed_blend_vertex(vc, f["faces"].to(dev), p2f, b, d, z, s, gm, a, S, S, **kw)
    else:
        c = f["colors"].to(dev).requires_grad_(True)
        img = perturbed_blend(c, p2f, d, z, s, gm, a, S, S, **kw)
    img.backward(f["gimg"].to(dev))
    torch.cuda.synchronize()
    out = dict(image=img.detach(), dists=d.grad, zbuf=z.grad, sigma=s.grad, gamma=gm.grad, alpha=a.grad)
    if vertex:
        out.update(bary=b.grad, vc=vc.grad)
    else:
        out.update(colors=c.grad)
    return out


def _env(updates, fn):
    old = {k: os.environ.get(k) for k in updates}
    try:
        for k, v in updates.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module", params=[False, True], ids=["texels", "vertex"])
def case(request):
    vertex = request.param
    f = _frags(seed=31 + vertex, with_vertex=vertex)
    img, g = _oracle(f, vertex)
    return vertex, f, img, g


def test_batch_grid_default_layout_matches_oracle(case, device):
    vertex, f, oimg, og = case
    # the backward grid exceeds 8192 blocks: the default interleaves it (make_geo)
    assert N * H * W // 32 > 8192
    out = _env({"PR_BLEND_INTERLEAVE": None}, lambda: _gpu(f, vertex, device))
    assert int((out["dists"] != 0).sum()) > 100000  # real coverage
    assert_close(out["image"], oimg, name="image")
    assert_close(out["dists"], og["dists"], name="d dists")
    assert_close(out["zbuf"], og["zbuf"], name="d zbuf")
    if vertex:
        assert_close(out["bary"], og["bary"], name="d bary")
        assert_close(out["vc"], og["vc"], name="d vertex colours")
    else:
        assert_close(out["colors"], og["colors"], name="d colours")
    for k in ("sigma", "gamma", "alpha"):
        assert out[k].device.type == "cpu" and out[k].dim() == 0
        assert_close(out[k], og[k], rtol=SCALAR_RTOL, name=k)


def test_batch_grid_layouts_bitwise(case, device):
    """Per-slot gradients do not depend on the pixel-block layout (B6's split is per launch)."""
    vertex, f, _, _ = case
    a = _env({"PR_BLEND_INTERLEAVE": None}, lambda: _gpu(f, vertex, device))
    b = _env({"PR_BLEND_INTERLEAVE": "0"}, lambda: _gpu(f, vertex, device))
    c = _env({"PR_BLEND_INTERLEAVE": "1"}, lambda: _gpu(f, vertex, device))
    for k in ("image", "dists", "zbuf") + (("bary",) if vertex else ("colors",)):
        assert torch.equal(a[k], b[k]), k
        assert torch.equal(a[k], c[k]), k
    for k in ("sigma", "gamma", "alpha"):  # per-block partials regroup with the blocks
        assert_close(a[k], b[k], rtol=SCALAR_RTOL, name=k)
    if vertex:  # float-atomic scatter
        assert_close(a["vc"], b["vc"], name="d vertex colours")


def test_batch_grid_fused_finalize_orders_bitwise(case, device):
    """The fused scalar reduction (default, relaxed arrivals), its acq_rel-ordered form and the
    separate finalize kernel give the same bits on an interleaved many-generation grid."""
    import pertrenderer_amd.blend as pb
    vertex, f, _, _ = case
    if vertex:
        pytest.skip("the texel case covers the reduction (same kernel tail)")
    a = _env({"PR_BLEND_SYNC_ORDER": None}, lambda: _gpu(f, vertex, device))
    b = _env({"PR_BLEND_SYNC_ORDER": "release"}, lambda: _gpu(f, vertex, device))
    old = pb._FUSED_FINALIZE
    try:
        pb._FUSED_FINALIZE = False
        c = _gpu(f, vertex, device)
    finally:
        pb._FUSED_FINALIZE = old
    for k in ("sigma", "gamma", "alpha", "dists", "zbuf", "colors", "image"):
        assert torch.equal(a[k], b[k]), k
        assert torch.equal(a[k], c[k]), k
