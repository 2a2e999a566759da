"""Gradients w.r.t. the camera planes znear / zfar, and the background colour, when they are
tensors that require grad.

The reference computes z_inv = (zfar - zbuf) / (zfar - znear) * mask in torch (smoothagg.py:198,
planes from the cameras: random_rasterizer.py:172-173), so such planes get gradients there.  The
native kernels take the planes as constants; blend.plane_link attaches d znear / d zfar from the
kernels' d zbuf.  Checked against the oracle, which differentiates the reference's z_inv
expression by torch autograd (oracle/blend_oracle.py plane_grads), with injected reference draws."""
import numpy as np
import pytest
import torch

from conftest import assert_close
from oracle import blend_oracle as bo
from pertrenderer_amd import Noise, perturbed_aggregate, perturbed_blend, soft_blend
from pertrenderer_amd.renderer.rasterizer import attach_valid_counts
from test_gpu_blend import _synthetic

pytestmark = pytest.mark.gpu


def _planes(N, scalar, device, zn=1.5, zf=40.0):
    if scalar:  # one 0-d plane shared by the batch
        return (torch.tensor(zn, device=device, requires_grad=True), torch.tensor(zf, device=device, requires_grad=True))
    return (torch.linspace(zn, zn + 0.5, N, device=device).reshape(N, 1, 1, 1).requires_grad_(True),
            torch.linspace(zf, zf + 10.0, N, device=device).reshape(N, 1, 1, 1).requires_grad_(True))


@pytest.mark.parametrize("counts", [False, True])
@pytest.mark.parametrize("scalar", [False, True])
def test_blend_plane_gradients_match_oracle(counts, scalar, device):
    N, H, W, K, Sr, Sa = 2, 12, 10, 20, 8, 8
    f = _synthetic(N, H, W, K, Sr, Sa, seed=41)
    zn, zf = _planes(N, scalar, device)
    p2f = torch.tensor(f["pix_to_face"], device=device)
    if counts:
        attach_valid_counts(p2f, (p2f >= 0).sum(-1).to(torch.int32))
    d = torch.tensor(f["dists"], device=device, requires_grad=True)
    z = torch.tensor(f["zbuf"], device=device, requires_grad=True)
    c = torch.tensor(f["colors"], device=device, requires_grad=True)
    s, g, a = (torch.tensor(float(f[k]), requires_grad=True) for k in ("sigma", "gamma", "alpha"))
    noise = Noise.injected(torch.tensor(f["noise_r"], device=device), torch.tensor(f["noise_a"], device=device))
    img = perturbed_blend(c, p2f, d, z, s, g, a, Sr, Sa, eps=float(f["eps"]), background=tuple(f["background"]),
                          znear=zn, zfar=zf, noise=noise, live_only=True)  # the link turns live-only off
    (img * torch.tensor(f["grad_image"], device=device)).sum().backward()
    T = lambda x: torch.from_numpy(np.asarray(x))
    ozn, ozf = (t.detach().cpu().expand(N, 1, 1, 1).contiguous() for t in (zn, zf))
    oimg, s_ = bo.blend_forward(T(f["pix_to_face"]), T(f["dists"]), T(f["zbuf"]), T(f["colors"]), T(f["noise_r"]),
                                T(f["noise_a"]), T(f["sigma"]), T(f["gamma"]), T(f["alpha"]), float(f["eps"]),
                                T(f["background"]), ozn, ozf)
    og = bo.blend_backward(T(f["grad_image"]), s_)
    assert_close(img, oimg, name="image")
    assert_close(z.grad, og["zbuf"], name="zbuf")
    for name, leaf, ref in (("znear", zn, og["znear"]), ("zfar", zf, og["zfar"])):
        assert leaf.grad is not None and leaf.grad.shape == leaf.shape, name
        assert float(ref.abs().max()) > 0, name
        assert_close(leaf.grad, ref.sum() if scalar else ref, rtol=1e-4, atol_rel=1e-6, name=name)


def test_aggregate_plane_gradients_match_oracle(device):
    N, H, W, K, Sa = 2, 9, 11, 16, 8
    f = _synthetic(N, H, W, K, 4, Sa, seed=43)
    zn, zf = _planes(N, False, device)
    z = torch.tensor(f["zbuf"], device=device, requires_grad=True)
    prob = torch.rand((N, H, W, K), generator=torch.Generator().manual_seed(2)) * 0.9 + 0.05
    pr = prob.to(device).requires_grad_(True)
    mask = torch.tensor(f["pix_to_face"], device=device) >= 0
    gW = torch.randn((N, H, W, K + 1), generator=torch.Generator().manual_seed(3))
    g, a = (torch.tensor(float(f[k]), requires_grad=True) for k in ("gamma", "alpha"))
    Wt = perturbed_aggregate(z, zf, zn, pr, mask, g, a, Sa, eps=float(f["eps"]),
                             noise=Noise.injected(noise_a=torch.tensor(f["noise_a"], device=device)))
    (Wt * gW.to(device)).sum().backward()
    T = lambda x: torch.from_numpy(np.asarray(x))
    out = bo.aggregate_forward_backward(T(f["zbuf"]), zf.detach().cpu(), zn.detach().cpu(), prob, mask.cpu(),
                                        T(f["noise_a"]), T(f["gamma"]), T(f["alpha"]), float(f["eps"]), gW,
                                        planes=True)
    assert_close(Wt, out[0], name="W")
    assert_close(z.grad, out[1], name="zbuf")
    assert_close(zn.grad, out[5], rtol=1e-4, atol_rel=1e-6, name="znear")
    assert_close(zf.grad, out[6], rtol=1e-4, atol_rel=1e-6, name="zfar")


def test_soft_blend_plane_gradients_match_oracle(device):
    from test_gpu_softblend import _frags
    N, H, W, K = 2, 10, 8, 12
    sigma, gamma, alpha, eps, bg = 1e-3, 1e-2, 1.3, 1e-10, (0.1, 0.2, 0.3)
    p2f, d, z, cols, gimg, valid = _frags(N, H, W, K, 17, True, sigma)
    zn, zf = _planes(N, False, device)
    ozn, ozf = (t.detach().cpu().clone().requires_grad_(True) for t in (zn, zf))
    oimg, og = bo.soft_blend_forward_backward(p2f, d, z, cols, sigma, gamma, alpha, eps, bg, ozn, ozf, gimg)
    dd, zz, cc = (t.to(device).requires_grad_(True) for t in (d, z, cols))
    s, gm, al = (torch.tensor(v, requires_grad=True) for v in (sigma, gamma, alpha))
    img = soft_blend(cc, p2f.to(device), dd, zz, s, gm, al, eps=eps, background=bg, znear=zn, zfar=zf)
    (img * gimg.to(device)).sum().backward()
    assert_close(img, oimg, name="image")
    # d zbuf of a pixel's nearest slot holds the softmax's fp32 shift residue (test_gpu_softblend),
    # which the plane sums carry too: the same 1e-4 of the largest term
    assert_close(zn.grad, og["znear"], rtol=1e-4, atol_rel=1e-4, name="znear")
    assert_close(zf.grad, og["zfar"], rtol=1e-4, atol_rel=1e-4, name="zfar")


def test_constant_planes_add_no_node(device):
    """Float planes, or tensors without grad: zbuf goes to the kernels as is (no link node)."""
    from pertrenderer_amd import blend
    z = torch.rand((1, 4, 4, 3), device=device, requires_grad=True)
    p2f = torch.zeros((1, 4, 4, 3), dtype=torch.int64, device=device)
    for zn, zf in ((1.0, 100.0), (torch.ones(1, 1, 1, 1, device=device), torch.full((1, 1, 1, 1), 100.0, device=device))):
        out, linked = blend.plane_link(z, zn, zf, p2f)
        assert out is z and not linked
    with torch.no_grad():
        zn = torch.ones((), device=device, requires_grad=True)
        out, linked = blend.plane_link(z, zn, 100.0, p2f)
        assert out is z and not linked


@pytest.mark.parametrize("shader_kind", ["simple", "phong"])
def test_background_gradient_matches_finite_difference(shader_kind, device):
    """A background colour tensor that requires grad (the reference's colour mix differentiates it:
    random_rasterizer.py:39-43, 52) takes the composition path, through MeshRenderer too.  The image
    is linear in the background for fixed draws, so d L / d bg equals the difference quotient of
    two renders with the same torch draws (one unit step per channel)."""
    import math
    import pertrenderer_amd as pa
    from pertrenderer_amd import noise
    from pertrenderer_amd.renderer import (FoVPerspectiveCameras, MeshRasterizer, PointLights,
                                           RasterizationSettings, look_at_view_transform)
    from pertrenderer_amd.renderer.renderer import MeshRenderer
    from test_gpu_shading import _scene
    mesh, _, _, _, mats, _, _, _ = _scene(device, "vertex")
    R, T = look_at_view_transform(2.2, 25.0, 40.0, device=device)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    rs = RasterizationSettings(image_size=32, blur_radius=math.log(1e4 - 1) * 1e-3, faces_per_pixel=8)
    sr, sa = pa.GaussianRast(nb_samples=4, sigma=1e-3), pa.GaussianAgg(nb_samples=4, gamma=1e-2)
    if shader_kind == "simple":
        shader = pa.RandomSimpleShader(device=device, cameras=cams, smoothrast=sr, smoothagg=sa)
    else:
        shader = pa.RandomPhongShader(device=device, cameras=cams, lights=PointLights(device=device),
                                      materials=mats, smoothrast=sr, smoothagg=sa)
    renderer = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs), shader)
    G = torch.rand((1, 32, 32, 4), device=device, generator=torch.Generator(device).manual_seed(8))
    old = noise.get_noise_source()
    noise.set_noise_source("torch")
    try:
        def render(bg):
            torch.manual_seed(13)
            return renderer(mesh, blend_params=pa.random_rasterizer.BlendParams(1e-4, 1e-4, bg))
        bg = torch.tensor([0.2, 0.3, 0.4], device=device, requires_grad=True)
        img = render(bg)
        (gbg,) = torch.autograd.grad((img * G).sum(), bg)
        with torch.no_grad():
            base = render(bg.detach())
            assert_close(img.detach(), base, name="image (composition vs fused)")
            fd = torch.stack([((render(bg.detach() + torch.eye(3, device=device)[c]) - base) * G).sum()
                              for c in range(3)])
    finally:
        noise.set_noise_source(old)
    assert float(fd.abs().max()) > 0
    assert_close(gbg, fd, rtol=1e-4, atol_rel=1e-5, name="d background")
