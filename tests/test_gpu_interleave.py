"""Interleaved blend pixel blocks (pr_blend.hip block_pixel, default on; PR_BLEND_INTERLEAVE=0 gives
the consecutive blocks) against the consecutive layout.

Every pixel is computed from its own fragments with Philox counters keyed by its physical index,
so the forward image must be bitwise equal in both layouts, and so must the backward's per-slot
gradients: B6's lane split per entry depends on the launch only (the agg sample count), never
on the pass's entry count, so a pixel's d z is summed in the same order whatever block holds it
(rounds 1-4 split light passes' sample groups over more lanes, so the two layouts summed some
pixels differently).  The smoothing scalars' gradients are per-block partial
sums reduced in another grouping, and the vertex-colour gradient is a float-atomic scatter: those
two compare at conftest.assert_close (1e-5 elementwise relative).  Cases: the bench frame
at 128^2 (vertex colours, Gaussian pair with and without variance reduction), a batch of two
frames whose blocks must keep to their own image (texel colours, scattered valid prefixes,
per-image planes), a shape whose pixel count is no multiple of the block (layout off: identical),
and the standalone aggregate (weights out).
"""
import os

import pytest
import torch

import pertrenderer_amd as pa
from conftest import assert_close
from pertrenderer_amd.blend import Noise, perturbed_aggregate

pytestmark = pytest.mark.gpu


def _with(value, fn):
    old = os.environ.get("PR_BLEND_INTERLEAVE")
    try:
        os.environ["PR_BLEND_INTERLEAVE"] = value
        return fn()
    finally:
        if old is None:
            os.environ.pop("PR_BLEND_INTERLEAVE", None)
        else:
            os.environ["PR_BLEND_INTERLEAVE"] = old


def _compare(a, b, names, loose):
    for x, y, n in zip(a, b, names):
        if n in loose:
            assert_close(x, y, rtol=2e-5 if x.dim() == 0 else 1e-5, name=n)
        else:
            assert torch.equal(x, y), n


def _bench_frame(device, agg_vr):
    import bench
    wl = bench.Workload(device, image_size=128, K=50, samples=8)
    from pertrenderer_amd.renderer import Rotate, so3_exponential_map
    R = so3_exponential_map(wl.log_rot)
    mesh = wl.base.update_padded(Rotate(R).transform_points(wl.base.verts_padded()))
    frag = wl.renderer.rasterizer(mesh, cameras=wl.cameras)

    def run():
        dists = frag.dists.detach().requires_grad_(True)
        zbuf = frag.zbuf.detach().requires_grad_(True)
        bary = frag.bary_coords.detach().requires_grad_(True)
        vc = mesh.textures.verts_features_packed().detach().requires_grad_(True)
        sig, gam, alp = (torch.tensor(v, device=device, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
        img = pa.blend.perturbed_blend_vertex(vc, mesh.faces_packed(), frag.pix_to_face, bary, dists, zbuf, sig,
                                              gam, alp, 8, 8, background=(0.2, 0.4, 0.6),
                                              noise=Noise.philox(seed_r=17, seed_a=29), agg_vr=agg_vr)
        g = torch.randn(img.shape, device=device, generator=torch.Generator(device).manual_seed(3))
        img.backward(g)
        torch.cuda.synchronize()
        return [img.detach(), dists.grad, zbuf.grad, bary.grad, vc.grad, sig.grad, gam.grad, alp.grad]
    return run


@pytest.mark.parametrize("agg_vr", [True, False])
def test_interleaved_blocks_bench_frame(device, agg_vr):
    run = _bench_frame(device, agg_vr)
    a = _with("1", run)
    b = _with("0", run)
    assert int((a[1] != 0).sum()) > 1000  # the frame has real coverage
    _compare(a, b, ("image", "d dists", "d zbuf", "d bary", "d vertex colours", "d sigma", "d gamma", "d alpha"),
             loose=("d vertex colours", "d sigma", "d gamma", "d alpha"))


def _frags(device, N, H, W, K, seed):
    g = torch.Generator(device).manual_seed(seed)
    cnt = torch.randint(0, K + 1, (N, H, W), generator=g, device=device)
    cnt[:, : H // 3] = 0  # an empty band: empty and mixed blocks in the consecutive layout
    k = torch.arange(K, device=device)
    valid = k < cnt[..., None]
    p2f = torch.where(valid, torch.randint(0, 900, (N, H, W, K), generator=g, device=device), -1)
    dists = ((torch.rand((N, H, W, K), generator=g, device=device) - 0.5) * 6e-3)
    zbuf = torch.where(valid, (5.0 + 2.0 * torch.rand((N, H, W, K), generator=g, device=device)).sort(-1).values, -1.)
    colors = torch.rand((N, H, W, K, 3), generator=g, device=device)
    return p2f, dists, zbuf, colors


@pytest.mark.parametrize("N,H,W,K", [(2, 64, 48, 20), (1, 30, 31, 12)])
def test_interleaved_blocks_texel_batch(device, N, H, W, K):
    p2f, d0, z0, c0 = _frags(device, N, H, W, K, seed=N + H)
    zn = torch.tensor([1.0, 0.5][:N], device=device)
    zf = torch.tensor([100.0, 20.0][:N], device=device)

    def run():
        dists, zbuf, colors = (t.clone().requires_grad_(True) for t in (d0, z0, c0))
        sig, gam, alp = (torch.tensor(v, device=device, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
        img = pa.perturbed_blend(colors, p2f, dists, zbuf, sig, gam, alp, 8, 16, background=(0.1, 0.2, 0.3),
                                 znear=zn, zfar=zf, noise=Noise.philox(seed_r=5, seed_a=7))
        g = torch.randn(img.shape, device=device, generator=torch.Generator(device).manual_seed(1))
        img.backward(g)
        torch.cuda.synchronize()
        return [img.detach(), dists.grad, zbuf.grad, colors.grad, sig.grad, gam.grad, alp.grad]
    a = _with("1", run)
    b = _with("0", run)
    _compare(a, b, ("image", "d dists", "d zbuf", "d colours", "d sigma", "d gamma", "d alpha"),
             loose=("d sigma", "d gamma", "d alpha"))


def test_interleaved_blocks_aggregate(device):
    N, H, W, K = 1, 32, 64, 16
    p2f, _, zbuf, _ = _frags(device, N, H, W, K, seed=11)
    mask = p2f >= 0
    prob0 = torch.rand((N, H, W, K), device=device, generator=torch.Generator(device).manual_seed(2))

    def run():
        prob = prob0.clone().requires_grad_(True)
        z = zbuf.clone().requires_grad_(True)
        gam, alp = (torch.tensor(v, device=device, requires_grad=True) for v in (1e-2, 1.0))
        Wt = perturbed_aggregate(z, 100.0, 1.0, prob, mask, gam, alp, 16, noise=Noise.philox(seed_a=9))
        g = torch.randn(Wt.shape, device=device, generator=torch.Generator(device).manual_seed(4))
        Wt.backward(g)
        torch.cuda.synchronize()
        return [Wt.detach(), prob.grad, z.grad, gam.grad, alp.grad]
    a = _with("1", run)
    b = _with("0", run)
    _compare(a, b, ("weights", "d prob", "d zbuf", "d gamma", "d alpha"), loose=("d gamma", "d alpha"))


@pytest.mark.parametrize("Sa", [8, 64])
def test_default_layout_on_a_batch_grid(device, Sa):
    """The default on a batch grid (5 x 256^2, backward grid > 8192 blocks; Sa = 64: B6 splits each
    entry's 16 sample groups over 4 lanes in both layouts): consecutive forward,
    interleaved backward -- the forward's winners and rast cache are read by physical pixel / slot,
    so the mixed pair equals the consecutive one (image and per-slot gradients bitwise, the
    smoothing scalars to the per-block partials' grouping)."""
    p2f, d0, z0, c0 = _frags(device, 5, 256, 256, 8, seed=21)

    def run():
        dists, zbuf, colors = (t.clone().requires_grad_(True) for t in (d0, z0, c0))
        sig, gam, alp = (torch.tensor(v, device=device, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
        img = pa.perturbed_blend(colors, p2f, dists, zbuf, sig, gam, alp, 8, Sa, background=(0.1, 0.2, 0.3),
                                 noise=Noise.philox(seed_r=3, seed_a=4))
        g = torch.randn(img.shape, device=device, generator=torch.Generator(device).manual_seed(5))
        img.backward(g)
        torch.cuda.synchronize()
        return [img.detach(), dists.grad, zbuf.grad, colors.grad, sig.grad, gam.grad, alp.grad]
    old = os.environ.pop("PR_BLEND_INTERLEAVE", None)
    try:
        a = run()
    finally:
        if old is not None:
            os.environ["PR_BLEND_INTERLEAVE"] = old
    b = _with("0", run)
    _compare(a, b, ("image", "d dists", "d zbuf", "d colours", "d sigma", "d gamma", "d alpha"),
             loose=("d sigma", "d gamma", "d alpha"))
