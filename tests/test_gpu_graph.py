"""Graph-capture support: device-resident smoothing scalars and device Philox seeds give
the same results as the host-side paths, and a captured render step replays with
fresh noise every time (no host work inside the graph)."""
import numpy as np
import pytest
import torch

import pertrenderer_amd as pa
from pertrenderer_amd import Noise, perturbed_blend
from pertrenderer_amd.noise import DeviceSeed, use_device_seed

pytestmark = pytest.mark.gpu


def _frags(device, N=1, H=24, W=20, K=30, seed=0):
    g = torch.Generator().manual_seed(seed)
    valid = torch.rand((N, H, W, K), generator=g) < 0.7
    p2f = torch.where(valid, torch.randint(0, 100, (N, H, W, K), generator=g), torch.full((N, H, W, K), -1))
    dists = torch.where(valid, (torch.rand((N, H, W, K), generator=g) - 0.5) * 6e-3, torch.full((N, H, W, K), -1.0))
    zbuf = torch.where(valid, 5 + torch.rand((N, H, W, K), generator=g), torch.full((N, H, W, K), -1.0))
    cols = torch.rand((N, H, W, K, 3), generator=g)
    return [t.to(device) for t in (p2f, dists, zbuf, cols)]


def _render(device, p2f, dists, zbuf, cols, scal_dev, noise):
    d = dists.clone().requires_grad_(True)
    z = zbuf.clone().requires_grad_(True)
    c = cols.clone().requires_grad_(True)
    dev = device if scal_dev else "cpu"
    s, g, a = (torch.tensor(v, device=dev, requires_grad=True) for v in (1e-3, 1e-2, 1.3))
    img = perturbed_blend(c, p2f, d, z, s, g, a, 8, 8, background=(0.1, 0.2, 0.3), noise=noise)
    (img ** 2).sum().backward()
    return img.detach(), [d.grad, z.grad, c.grad, s.grad, g.grad, a.grad]


def test_device_scalars_match_host_scalars(device):
    fr = _frags(device)
    n = Noise.philox(seed_r=5, seed_a=6)
    i1, g1 = _render(device, *fr, False, n)
    i2, g2 = _render(device, *fr, True, n)
    assert torch.equal(i1, i2)
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a.cpu(), b.cpu(), rtol=0, atol=0)
    assert g2[3].is_cuda and g1[3].device.type == "cpu"


def test_device_seed_keys_and_graph_replay(device):
    fr = _frags(device, seed=1)
    ds = DeviceSeed(device, seed=1234)
    use_device_seed(ds)
    try:
        d = fr[1].clone().requires_grad_(True)
        s, g, a = (torch.tensor(v, device=device, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            ds.advance()
            perturbed_blend(fr[3], fr[0], d, fr[2], s, g, a, 8, 8).sum().backward()
        torch.cuda.current_stream().wait_stream(side)
        d.grad = None
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            ds.advance()
            img = perturbed_blend(fr[3], fr[0], d, fr[2], s, g, a, 8, 8)
            img.sum().backward()
        outs, grads, bases = [], [], []
        for _ in range(3):
            graph.replay()
            torch.cuda.synchronize()
            outs.append(img.clone())
            grads.append(d.grad.clone())
            bases.append(int(ds.tensor.item()))
        assert len(set(bases)) == 3
        assert not torch.equal(outs[0], outs[1]) and not torch.equal(outs[1], outs[2])
    finally:
        use_device_seed(None)
    # the last replay equals an eager call with the same base and stream ids (1: rast, 2: agg)
    base = torch.tensor([bases[-1]], dtype=torch.int64, device=device)
    d2 = fr[1].clone().requires_grad_(True)
    ref = perturbed_blend(fr[3], fr[0], d2, fr[2], s, g, a, 8, 8,
                          noise=Noise.philox(seed_r=1, seed_a=2, seeds=base))
    ref.sum().backward()
    assert torch.equal(ref.detach(), outs[-1])
    assert torch.equal(d2.grad, grads[-1])


def test_fixed_noise_ignores_device_seed(device):
    """GaussianAgg(fixed_noise=True) reseeds the global generator with 1 before its draw
    (smoothagg.py:18-19), so its noise is the same on every call even while a DeviceSeed base
    advances; without fixed_noise the same calls draw fresh noise."""
    from pertrenderer_amd.random_rasterizer import smooth_rgb_blend
    from pertrenderer_amd.renderer import BlendParams, Fragments
    p2f, dists, zbuf, cols = _frags(device, seed=2)
    mask = p2f >= 0
    prob = torch.rand(p2f.shape, generator=torch.Generator().manual_seed(3)).to(device) * mask
    frag = Fragments(p2f, zbuf, None, dists)
    ds = DeviceSeed(device, seed=99)
    use_device_seed(ds)
    try:
        for fixed in (True, False):
            agg = pa.GaussianAgg(nb_samples=8, gamma=2e-2, fixed_noise=fixed)
            # sigma so small that the Heaviside never flips: the image depends on the agg noise only
            rast = pa.GaussianRast(nb_samples=8, sigma=1e-12)
            ws, imgs = [], []
            for _ in range(3):
                ds.advance()
                ws.append(agg.aggregate(zbuf, 100.0, 1.0, prob, mask).detach())
                imgs.append(smooth_rgb_blend(cols, frag, rast, agg, BlendParams(1e-3, 2e-2, (0, 0, 0))).detach())
            if fixed:
                assert all(torch.equal(ws[0], w) for w in ws[1:])
                assert all(torch.equal(imgs[0], i) for i in imgs[1:])
            else:
                assert not torch.equal(ws[0], ws[1]) and not torch.equal(ws[1], ws[2])
                assert not torch.equal(imgs[0], imgs[1])
    finally:
        use_device_seed(None)


def _seed_next(s):
    """pr_seed_advance's update (pr_common.h seed_next) on the host."""
    m = (1 << 64) - 1
    z = (s + 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & m
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & m
    return z ^ (z >> 31)


def test_deferred_seed_advance_rides_on_the_face_pass(device):
    """DeviceSeed.advance() is applied by the next native face pass (MeshRasterizer ->
    pr_project_rast_fwd, PRProjectArgs.seed_advance), or flushed by a draw before one: either way
    the keys are those of the eager update, advanced once per call, in graph replays too."""
    import bench
    wl = bench.Workload(device, image_size=32, K=8, samples=4)
    ds = DeviceSeed(device, seed=4321)
    use_device_seed(ds)
    try:
        u = lambda t: int(t.item()) & ((1 << 64) - 1)
        b0 = u(ds.tensor)
        ds.advance()
        ds.advance()  # two pending advances, one face pass
        assert u(ds.tensor) == b0  # deferred
        wl.forward()
        torch.cuda.synchronize()
        assert ds._pending == 0 and u(ds.tensor) == _seed_next(_seed_next(b0))
        # a draw with no face pass before it flushes
        b1 = u(ds.tensor)
        ds.advance()
        fr = _frags(device, seed=4)
        perturbed_blend(fr[3], fr[0], fr[1], fr[2], torch.tensor(1e-3), torch.tensor(1e-2), torch.tensor(1.0), 4, 4)
        torch.cuda.synchronize()
        assert ds._pending == 0 and u(ds.tensor) == _seed_next(b1)
        # captured: every replay advances once, through the face pass
        wl.device_scalars()
        graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            ds.advance()
            wl.forward().backward()
        torch.cuda.current_stream().wait_stream(side)
        with torch.cuda.graph(graph):
            ds.advance()
            wl.forward().backward()
        assert ds._pending == 0
        b2 = u(ds.tensor)
        graph.replay()
        graph.replay()
        torch.cuda.synchronize()
        assert u(ds.tensor) == _seed_next(_seed_next(b2))
    finally:
        use_device_seed(None)
