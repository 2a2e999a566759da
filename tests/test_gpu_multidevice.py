"""In-process multi-device sample sharding (pertrenderer_amd.multidevice, set_sample_devices):
the samples of one smooth_rgb_blend split over 1, 2, 3 and 4 logical shards (all on cuda:0 here;
the collectives are the same code path, copies instead of RCCL) reproduce the one-device fused
kernel pair with the same Philox keys -- image bitwise (P from exact integer counts, the image
from every sample's gathered winner by the fused kernel's own colour mix), gradients to 1e-5 of
their scale (the summation order of the shards' partials).  Texel colours through
smooth_rgb_blend, and the fused TexturesVertex blend through sharded_blend(vert_colors=...) and
RandomSimpleShader; GaussianRast / GaussianAgg and ArctanRast / CauchyAgg; and the sharded vertex
blend captured into a HIP graph with a DeviceSeed (fresh noise per replay, the eager values)."""
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
@pytest.mark.parametrize("shards", [1, 2, 3, 4])
def test_sharded_blend_matches_one_device(pair, shards, device):
    """3 shards split 16 samples 6 / 5 / 5: P still bitwise (integer counts, not weighted floats)."""
    ref = _run(device, [device], PAIRS[pair], fused=True)  # the fused kernel pair, one device
    got = _run(device, [device] * shards, PAIRS[pair])
    assert torch.equal(got["image"], ref["image"])
    _close(got["dists"], ref["dists"])
    _close(got["zbuf"], ref["zbuf"])
    _close(got["colors"], ref["colors"])
    for k in ("sigma", "gamma", "alpha"):
        assert got[k].device.type == "cpu" and got[k].dim() == 0  # the reference's CPU 0-d leaves
        torch.testing.assert_close(got[k], ref[k], rtol=2e-5, atol=1e-9)


def _vertex_inputs(dev):
    g = torch.Generator().manual_seed(13)
    N, H, W, K, F_, V = 1, 24, 20, 12, 300, 200
    cnt = torch.randint(0, K + 1, (N, H, W, 1), generator=g)
    valid = torch.arange(K).expand(N, H, W, K) < cnt
    p2f = torch.where(valid, torch.randint(0, F_, (N, H, W, K), generator=g), torch.full((N, H, W, K), -1))
    dists = torch.where(valid, (torch.rand((N, H, W, K), generator=g) - 0.5) * 6e-3, torch.full((N, H, W, K), -1.0))
    zbuf = torch.where(valid, (5.0 + torch.rand((N, H, W, K), generator=g)).sort(-1).values,
                       torch.full((N, H, W, K), -1.0))
    b = torch.rand((N, H, W, K, 3), generator=g) + 0.05
    bary = torch.where(valid[..., None], b / b.sum(-1, keepdim=True), torch.full_like(b, -1.0))
    faces = torch.randint(0, V, (F_, 3), generator=g)
    vc = torch.rand((V, 3), generator=g)
    gimg = torch.randn((N, H, W, 4), generator=g)
    out = [t.to(dev) for t in (p2f, dists, zbuf, bary, faces, vc, gimg)]
    from pertrenderer_amd.renderer.rasterizer import attach_valid_counts
    attach_valid_counts(out[0], cnt[..., 0].to(torch.int32).to(dev))
    return out


def _run_vertex(dev, devices, S=16, seed=9, scalars_on=None, noise=None):
    from pertrenderer_amd.blend import perturbed_blend_vertex
    from pertrenderer_amd.multidevice import sharded_blend
    p2f, d0, z0, b0, faces, v0, gimg = _vertex_inputs(dev)
    d, z, b, v = (t.clone().requires_grad_(True) for t in (d0, z0, b0, v0))
    where = scalars_on or "cpu"
    s, g, a = (torch.tensor(x, device=where, requires_grad=True) for x in (1e-3, 1e-2, 1.0))
    torch.manual_seed(seed)
    if devices is None:
        img = perturbed_blend_vertex(v, faces, p2f, b, d, z, s, g, a, S, S, background=(0.1, 0.2, 0.3), noise=noise)
    else:
        img = sharded_blend(b, p2f, d, z, s, g, a, S, S, devices=devices, background=(0.1, 0.2, 0.3),
                            vert_colors=v, faces=faces)
    (img * gimg).sum().backward()
    return dict(image=img.detach(), dists=d.grad, zbuf=z.grad, bary=b.grad, vc=v.grad, sigma=s.grad, gamma=g.grad,
                alpha=a.grad)


@pytest.mark.parametrize("shards", [1, 2, 4])
def test_sharded_vertex_blend_matches_fused(shards, device):
    """The fused TexturesVertex blend sharded: image bitwise, every gradient at 1e-5 of its scale."""
    ref = _run_vertex(device, None)
    got = _run_vertex(device, [device] * shards)
    assert torch.equal(got["image"], ref["image"])
    assert float(ref["image"][..., 3].max()) > 0.5
    for k in ("dists", "zbuf", "bary", "vc"):
        _close(got[k], ref[k])
    for k in ("sigma", "gamma", "alpha"):
        torch.testing.assert_close(got[k], ref[k], rtol=2e-5, atol=1e-9)


def test_shader_uses_sharded_blend(device):
    """RandomSimpleShader with TexturesVertex: with sample devices set, its fused vertex blend shards
    the samples; the image equals the fused one-device shader's bit for bit."""
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
    assert torch.equal(out[1], out[0])  # the fused TexturesVertex blend, sharded: bitwise
    assert float(out[0][..., 3].max()) > 0.5


def test_too_few_samples_per_device_raises(device):
    p2f, d, z, c, _ = _inputs(device)
    from pertrenderer_amd.multidevice import sharded_blend
    with pytest.raises(ValueError):
        sharded_blend(c, p2f, d, z, torch.tensor(1e-3), torch.tensor(1e-2), torch.tensor(1.0), 2, 2,
                      devices=[device] * 4)


def test_sharded_vertex_blend_captures_into_a_graph(device):
    """The sharded fused vertex blend over 2 logical shards with a graph-mode DeviceSeed and device
    smoothing scalars, captured into one HIP graph: every replay draws fresh noise and equals the
    eager call with the same key base (one-device fused kernels, same base and stream ids)."""
    from pertrenderer_amd.multidevice import sharded_blend
    from pertrenderer_amd.noise import DeviceSeed, Noise, use_device_seed
    p2f, d0, z0, b0, faces, v0, gimg = _vertex_inputs(device)
    d, z, b = (t.clone().requires_grad_(True) for t in (d0, z0, b0))
    s, g, a = (torch.tensor(x, device=device, requires_grad=True) for x in (1e-3, 1e-2, 1.0))
    ds = DeviceSeed(device, seed=777)
    use_device_seed(ds)

    def step():
        ds.advance()
        img = sharded_blend(b, p2f, d, z, s, g, a, 8, 8, devices=[device, device], background=(0.1, 0.2, 0.3),
                            vert_colors=v0, faces=faces)
        (img * gimg).sum().backward()
        return img
    try:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        for t in (d, z, b):
            t.grad = None
        with torch.cuda.graph(graph):
            img = step()
        outs, grads, bases = [], [], []
        for _ in range(3):
            graph.replay()
            torch.cuda.synchronize()
            outs.append(img.detach().clone())
            grads.append(d.grad.clone())
            bases.append(int(ds.tensor.item()))
    finally:
        use_device_seed(None)
    assert len(set(bases)) == 3 and not torch.equal(outs[0], outs[1])
    # the last replay against the one-device fused blend with that base: rast id 1, agg id 2
    from pertrenderer_amd.blend import perturbed_blend_vertex
    base = torch.tensor([bases[-1]], dtype=torch.int64, device=device)
    d2 = d0.clone().requires_grad_(True)
    ref = perturbed_blend_vertex(v0, faces, p2f, b0, d2, z0, s.detach(), g.detach(), a.detach(), 8, 8,
                                 background=(0.1, 0.2, 0.3), noise=Noise.philox(seed_r=1, seed_a=2, seeds=base))
    (ref * gimg).sum().backward()
    assert torch.equal(ref.detach(), outs[-1])
    _close(grads[-1], d2.grad)
