"""In-process multi-device sample sharding (pertrenderer_amd.multidevice, set_sample_devices):
the samples of one smooth_rgb_blend split over 2 and 4 logical shards (all on cuda:0 here; the
collectives are the same code path, copies instead of RCCL) reproduce the one-device full-S
result -- image bitwise (P and W are exact counts: power-of-two shards), gradients up to the
summation order of the shards' partials -- and the one-shard composition equals the fused
kernel pair with the same Philox keys.  Through the public surface: smooth_rgb_blend and
RandomSimpleShader with GaussianRast / GaussianAgg and ArctanRast / CauchyAgg."""
import os

import pytest
import torch
from conftest import ROOT

import pertrenderer_amd as pa
from pertrenderer_amd.random_rasterizer import smooth_rgb_blend
from pertrenderer_amd.renderer.rasterizer import Fragments
from pertrenderer_amd.renderer.renderer import BlendParams

pytestmark = pytest.mark.gpu


def _inputs(dev):
    g = torch.Generator().manual_seed(11)
    N, H, W, K = 1, 24, 20, 12
    cnt = torch.randint(0, K + 1, (N, H, W, 1), generator=g)
    valid = torch.arange(K).expand(N, H, W, K) < cnt
    p2f = torch.where(valid, torch.randint(0, 500, (N, H, W, K), generator=g), torch.full((N, H, W, K), -1))
    dists = torch.where(valid, (torch.rand((N, H, W, K), generator=g) - 0.5) * 6e-3, torch.full((N, H, W, K), -1.0))
    zbuf = torch.where(valid, (5.0 + torch.rand((N, H, W, K), generator=g)).sort(-1).values,
                       torch.full((N, H, W, K), -1.0))
    colors = torch.rand((N, H, W, K, 3), generator=g)
    gimg = torch.randn((N, H, W, 4), generator=g)
    return [t.to(dev) for t in (p2f, dists, zbuf, colors, gimg)]


def _run(dev, devices, pair, S=16, seed=7, fused=False):
    p2f, d0, z0, c0, gimg = _inputs(dev)
    d, z, c = (t.clone().requires_grad_(True) for t in (d0, z0, c0))
    rast, agg = pair(S)
    frag = Fragments(pix_to_face=p2f, zbuf=z, bary_coords=None, dists=d)
    pa.set_sample_devices(None if fused else devices)
    try:
        torch.manual_seed(seed)
        img = smooth_rgb_blend(c, frag, rast, agg, BlendParams(1e-3, 1e-2, (0.1, 0.2, 0.3)))
    finally:
        pa.set_sample_devices(None)
    (img * gimg).sum().backward()
    return dict(image=img.detach(), dists=d.grad, zbuf=z.grad, colors=c.grad, sigma=rast.sigma.grad,
                gamma=agg.gamma.grad, alpha=agg.alpha.grad)


PAIRS = {
    "gaussian": lambda S: (pa.GaussianRast(nb_samples=S, sigma=1e-3), pa.GaussianAgg(nb_samples=S, gamma=1e-2)),
    "cauchy": lambda S: (pa.ArctanRast(nb_samples=S, sigma=1e-3), pa.CauchyAgg(nb_samples=S, gamma=1e-2)),
}


def _close(a, b, rtol=1e-5):
    tol = rtol * float(b.abs().max()) + 1e-7
    assert float((a - b).abs().max()) <= tol, (float((a - b).abs().max()), tol)


@pytest.mark.parametrize("pair", sorted(PAIRS))
@pytest.mark.parametrize("shards", [2, 4])
def test_sharded_blend_matches_one_device(pair, shards, device):
    ref = _run(device, [device], PAIRS[pair], fused=True)  # the fused kernel pair, one device
    from pertrenderer_amd.multidevice import sharded_blend  # the one-shard composition
    p2f, d0, z0, c0, gimg = _inputs(device)
    d, z, c = (t.clone().requires_grad_(True) for t in (d0, z0, c0))
    rast, agg = PAIRS[pair](16)
    torch.manual_seed(7)
    kw = dict(rast_kind=rast.noise_kind, rast_vr=rast.variance_reduction, agg_kind=agg.noise_kind,
              agg_vr=agg.variance_reduction)
    img1 = sharded_blend(c, p2f, d, z, rast.sigma, agg.gamma, agg.alpha, 16, 16, devices=[device],
                         background=(0.1, 0.2, 0.3), **kw)
    (img1 * gimg).sum().backward()
    _close(img1.detach(), ref["image"])  # torch colour mix vs the kernel's: fp order only
    _close(d.grad, ref["dists"])
    _close(z.grad, ref["zbuf"])
    # the sharded run against the one-shard composition
    got = _run(device, [device] * shards, PAIRS[pair])
    assert torch.equal(got["image"], img1.detach())
    _close(got["dists"], d.grad)
    _close(got["zbuf"], z.grad)
    _close(got["colors"], c.grad)
    for k, ref_leaf in (("sigma", rast.sigma), ("gamma", agg.gamma), ("alpha", agg.alpha)):
        assert got[k].device.type == "cpu" and got[k].dim() == 0  # the reference's CPU 0-d leaves
        torch.testing.assert_close(got[k], ref_leaf.grad, rtol=2e-5, atol=1e-9)


def test_shader_uses_sharded_blend(device):
    """RandomSimpleShader with TexturesVertex: with sample devices set, the texel path through
    smooth_rgb_blend shards the samples; its image equals the fused one-device shader's."""
    from pertrenderer_amd.renderer import (FoVPerspectiveCameras, MeshRasterizer, MeshRenderer, Meshes,
                                           RasterizationSettings, TexturesVertex, look_at_view_transform)
    from pertrenderer_amd.renderer import load_obj
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    v, f = verts.to(device), faces.verts_idx.to(device)
    g = torch.Generator().manual_seed(3)
    mesh = Meshes([v], [f], TexturesVertex([torch.rand((v.shape[0], 3), generator=g).to(device)]))
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=device)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    rs = RasterizationSettings(image_size=48, blur_radius=9.2e-3, faces_per_pixel=16)
    out = []
    for devs in (None, [device, device]):
        rast, agg = pa.GaussianRast(nb_samples=8, sigma=1e-3), pa.GaussianAgg(nb_samples=8, gamma=1e-2)
        shader = pa.RandomSimpleShader(device=device, cameras=cams, smoothrast=rast, smoothagg=agg)
        r = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs), shader)
        pa.set_sample_devices(devs)
        try:
            torch.manual_seed(5)
            out.append(r(mesh).detach())
        finally:
            pa.set_sample_devices(None)
    torch.testing.assert_close(out[1], out[0], rtol=1e-5, atol=1e-6)
    assert float(out[0][..., 3].max()) > 0.5


def test_too_few_samples_per_device_raises(device):
    p2f, d, z, c, _ = _inputs(device)
    from pertrenderer_amd.multidevice import sharded_blend
    with pytest.raises(ValueError):
        sharded_blend(c, p2f, d, z, torch.tensor(1e-3), torch.tensor(1e-2), torch.tensor(1.0), 2, 2,
                      devices=[device] * 4)
