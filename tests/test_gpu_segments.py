"""The blend kernels' entry-balanced segment plan (pr_blend.hip: blend_plan_count_kernel +
blend_plan_list_kernel cut every pixel block into parts of about the same number of entries, one
workgroup per part) against the static grid.  The plan is opt-in (PR_BLEND_SEG=1): measured slower at cfg 2.

The per-pixel arithmetic of the forward is unchanged, so the image and the winners are bitwise
equal, and so are d bary / d texels (win counts times the image gradient).  d dists and d zbuf go
through the score-function sums d z, which the backward splits over more lanes in a part of few
entries (B6's nch), so they agree to fp32 summation order (1e-5; bitwise at the default segment
size on the bench frame); the smoothing scalars' per-workgroup partials are summed per segment
instead of per block (1e-4: with Cauchy noise these sums cancel heavily) and d vertex colours keep
their float-atomic summation order (1e-5).  Checked for several segment sizes (down to the
smallest, 2 (K+1) entries: most blocks then split into many parts), with Philox and injected
noise, Gaussian and Cauchy aggregation (the backward's compact and full entry layouts), texel and
vertex colours, a frame whose pixel count is not a multiple of the block size, a batch, a second
backward of the same forward (the queues reset) and wider lanes per pixel (PR_BLEND_SEG_LPP:
reductions in another order, 1e-5).
"""
import contextlib
import os

import pytest
import torch

import pertrenderer_amd as pa
from conftest import assert_close

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def env(**kw):
    old = {k: os.environ.get(k) for k in kw}
    try:
        for k, v in kw.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = str(v)
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _frame(device, size=256, K=50, batch=1):
    import bench
    wl = bench.Workload(device, image_size=size, K=K, samples=8, batch=batch)
    from pertrenderer_amd.renderer import Rotate, so3_exponential_map
    R = so3_exponential_map(wl.log_rot)
    mesh = wl.base.update_padded(Rotate(R).transform_points(wl.base.verts_padded()))
    frag = wl.renderer.rasterizer(mesh, cameras=wl.cameras)
    return mesh, frag


def _run(device, mesh, frag, vertex=True, agg_kind="gaussian", noise="philox", twice=False, seed=5):
    dists = frag.dists.detach().requires_grad_(True)
    zbuf = frag.zbuf.detach().requires_grad_(True)
    bary = frag.bary_coords.detach().requires_grad_(True)
    vc = mesh.textures.verts_features_packed().detach().requires_grad_(True)
    sig, gam, alp = (torch.tensor(v, device=device, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
    N, H, W, K = frag.pix_to_face.shape
    if noise == "philox":
        nz = pa.blend.Noise.philox(seed_r=11 + seed, seed_a=23 + seed)
    else:
        g = torch.Generator().manual_seed(seed)
        nz = pa.blend.Noise.injected(torch.randn((8, N, H, W, K), generator=g).to(device),
                                     torch.randn((8, N, H, W, K + 1), generator=g).to(device))
    if vertex:
        img = pa.blend.perturbed_blend_vertex(vc, mesh.faces_packed(), frag.pix_to_face, bary, dists, zbuf, sig,
                                              gam, alp, 8, 8, background=(0.2, 0.4, 0.6), noise=nz,
                                              agg_kind=agg_kind)
        leaves = [dists, zbuf, bary, vc, sig, gam, alp]
    else:
        from pertrenderer_amd.renderer.interp import interpolate_vertex_attributes
        tex = interpolate_vertex_attributes(frag.pix_to_face, frag.bary_coords, vc.detach(),
                                            mesh.faces_packed()).detach().requires_grad_(True)
        img = pa.blend.perturbed_blend(tex, frag.pix_to_face, dists, zbuf, sig, gam, alp, 8, 8,
                                       background=(0.2, 0.4, 0.6), noise=nz, agg_kind=agg_kind)
        leaves = [dists, zbuf, tex, sig, gam, alp]
    g = torch.randn(img.shape, device=device, generator=torch.Generator(device).manual_seed(3))
    grads = torch.autograd.grad(img, leaves, g, retain_graph=twice)
    if twice:
        again = torch.autograd.grad(img, leaves, g)
        for a, b in zip(grads[:-3], again[:-3]):
            if a is not None:
                assert_close(b, a, name="second backward")
        for a, b in zip(grads[-3:], again[-3:]):
            assert torch.equal(a, b)  # the same segments, partials summed in the same order
    torch.cuda.synchronize()
    return [img.detach()] + list(grads)


def _compare(a, b, vertex=True, exact=True):
    names = (["image", "d dists", "d zbuf", "d bary", "d vertex colours"] if vertex else
             ["image", "d dists", "d zbuf", "d texels"]) + ["d sigma", "d gamma", "d alpha"]
    for x, y, n in zip(a, b, names):
        if n in ("d sigma", "d gamma", "d alpha"):
            # sums of ~1e5 per-slot terms of both signs (Cauchy noise: heavy cancellation) in another
            # order: fp32 summation error, 1e-4 as the reference-golden scalar bars on large cases
            assert_close(x, y, rtol=1e-4, name=n)
        elif n in ("d dists", "d zbuf", "d vertex colours") or not exact:
            assert_close(x, y, rtol=1e-5, name=n)
        else:
            assert torch.equal(x, y), n


@pytest.mark.parametrize("seg", [None, 256, 102])
def test_segments_match_static_grid(device, seg):
    mesh, frag = _frame(device)
    with env(PR_BLEND_SEG=1, PR_BLEND_SEG_FWD=seg, PR_BLEND_SEG_BWD=seg):
        a = _run(device, mesh, frag)
    with env(PR_BLEND_SEG=0):
        b = _run(device, mesh, frag)
    _compare(a, b)


@pytest.mark.parametrize("agg_kind,noise,vertex", [("gaussian", "torch", False), ("cauchy", "philox", True),
                                                   ("cauchy", "torch", False)])
def test_segments_variants(device, agg_kind, noise, vertex):
    mesh, frag = _frame(device, size=96, K=30)
    with env(PR_BLEND_SEG=1, PR_BLEND_SEG_FWD=62, PR_BLEND_SEG_BWD=62):
        a = _run(device, mesh, frag, vertex=vertex, agg_kind=agg_kind, noise=noise)
    with env(PR_BLEND_SEG=0):
        b = _run(device, mesh, frag, vertex=vertex, agg_kind=agg_kind, noise=noise)
    _compare(a, b, vertex=vertex)


@pytest.mark.parametrize("size,batch", [(75, 1), (64, 3)])
def test_segments_ragged_and_batched(device, size, batch):
    mesh, frag = _frame(device, size=size, K=20, batch=batch)
    with env(PR_BLEND_SEG=1, PR_BLEND_SEG_FWD=42, PR_BLEND_SEG_BWD=42):
        a = _run(device, mesh, frag)
    with env(PR_BLEND_SEG=0):
        b = _run(device, mesh, frag)
    _compare(a, b)


def test_segments_second_backward(device):
    mesh, frag = _frame(device, size=128)
    with env(PR_BLEND_SEG=1):
        _run(device, mesh, frag, twice=True)


def test_segments_wider_lanes(device):
    mesh, frag = _frame(device, size=128)
    with env(PR_BLEND_SEG=1, PR_BLEND_SEG_FWD=102, PR_BLEND_SEG_BWD=102, PR_BLEND_SEG_LPP=32, PR_BLEND_SEG_LPP_BWD=16):
        a = _run(device, mesh, frag)
    with env(PR_BLEND_SEG=0):
        b = _run(device, mesh, frag)
    _compare(a, b, exact=False)


def test_plan_is_used(device):
    """With PR_BLEND_SEG=1 the fused blend of natively rasterized fragments plans its segments (so
    the tests above compare the two paths) -- a frame above the plan's size limit does not, and
    nothing is planned by default."""
    from pertrenderer_amd import _native as nat
    from pertrenderer_amd.blend import _counts_for
    mesh, frag = _frame(device, size=64)
    assert _counts_for(frag.pix_to_face) is not None
    p = nat.PRBlendParams()
    p.N, p.H, p.W, p.K, p.Sr, p.Sa = 1, 256, 256, 50, 8, 8
    assert nat.load().pr_blend_plan_size(nat.C.byref(p)) == 0
    with env(PR_BLEND_SEG=1):
        assert nat.load().pr_blend_plan_size(nat.C.byref(p)) > 0
        p.N, p.H, p.W = 16, 512, 512
        assert nat.load().pr_blend_plan_size(nat.C.byref(p)) == 0
