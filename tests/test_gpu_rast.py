"""GPU parity of the native rasterizer / interpolation against the C oracle
(oracle/rast_oracle.c; PyTorch3D 0.4.0 semantics, parity unpinned by the reference).
Forward outputs are compared bit-exactly (same fp32 operation order on both sides);
the backward sums float atomics in arbitrary order and is compared with a tolerance."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, assert_close
from oracle import rast_ref
from pertrenderer_amd.renderer import (FoVPerspectiveCameras, MeshRasterizer, Meshes, RasterizationSettings,
                                       interpolate_face_attributes, load_obj, look_at_view_transform,
                                       rasterize_meshes)

pytestmark = pytest.mark.gpu


def _soup(F, seed, zmin=0.5, spread=1.2, size=0.4):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-spread, spread, (F, 1, 2))
    xy = c + rng.uniform(-size, size, (F, 3, 2))
    z = rng.uniform(zmin, 5.0, (F, 3, 1))
    fv = np.concatenate([xy, z], -1).astype(np.float32)
    fv[: F // 10, :, 2] -= 6.0  # some faces behind the camera
    return fv


def _run_native(fv, first, nf, H, W, K, blur, persp, clip, cull, dev):
    from pertrenderer_amd.renderer.rasterizer import _RasterizeFn
    fvt = torch.tensor(fv, device=dev, requires_grad=True)
    out = _RasterizeFn.apply(fvt, torch.tensor(first, device=dev), torch.tensor(nf, device=dev), H, W, K, blur,
                             persp, clip, cull)
    return fvt, out


@pytest.mark.parametrize("cfg", [
    dict(H=37, W=41, K=8, blur=0.0, persp=False, clip=False, cull=False),
    dict(H=32, W=32, K=20, blur=5e-3, persp=False, clip=True, cull=False),
    dict(H=24, W=40, K=5, blur=2e-3, persp=True, clip=True, cull=True),
    dict(H=16, W=16, K=70, blur=5e-2, persp=False, clip=True, cull=False),
])
def test_rasterizer_forward_matches_oracle_bitwise(cfg, device):
    fv = np.concatenate([_soup(150, 1), _soup(90, 2)])
    first, nf = np.array([0, 150]), np.array([150, 90])
    _, (p2f, zbuf, bary, dists) = _run_native(fv, first, nf, cfg["H"], cfg["W"], cfg["K"], cfg["blur"],
                                              cfg["persp"], cfg["clip"], cfg["cull"], device)
    rp, rz, rb, rd = rast_ref.rast_fwd(fv, first, nf, cfg["H"], cfg["W"], cfg["K"], cfg["blur"], cfg["persp"],
                                       cfg["clip"], cfg["cull"])
    assert (rp >= 0).sum() > 100
    np.testing.assert_array_equal(p2f.cpu().numpy(), rp)
    np.testing.assert_array_equal(zbuf.detach().cpu().numpy(), rz)
    np.testing.assert_array_equal(dists.detach().cpu().numpy(), rd)
    np.testing.assert_array_equal(bary.detach().cpu().numpy(), rb)


@pytest.mark.parametrize("persp,clip", [(False, False), (False, True), (True, True)])
def test_rasterizer_backward_matches_oracle(persp, clip, device):
    fv = _soup(120, 3)
    first, nf = np.array([0]), np.array([120])
    H = W = 32
    K = 10
    blur = 4e-3
    fvt, (p2f, zbuf, bary, dists) = _run_native(fv, first, nf, H, W, K, blur, persp, clip, False, device)
    g = np.random.default_rng(4)
    gz = g.standard_normal(zbuf.shape).astype(np.float32)
    gb = g.standard_normal(bary.shape).astype(np.float32)
    gd = g.standard_normal(dists.shape).astype(np.float32)
    loss = (zbuf * torch.tensor(gz, device=device)).sum() + (bary * torch.tensor(gb, device=device)).sum() \
        + (dists * torch.tensor(gd, device=device)).sum()
    loss.backward()
    ref = rast_ref.rast_bwd(fv, p2f.cpu().numpy(), gz, gb, gd, persp, clip)
    assert_close(fvt.grad, ref, rtol=1e-4, atol_rel=1e-5, name="grad_face_verts")


def test_interpolation_matches_oracle_and_backward(device):
    rng = np.random.default_rng(5)
    F, D = 300, 4
    p2f = rng.integers(-1, F, (2, 9, 11, 6))
    bary = rng.uniform(0, 1, p2f.shape + (3,)).astype(np.float32)
    attr = rng.standard_normal((F, 3, D)).astype(np.float32)
    b = torch.tensor(bary, device=device, requires_grad=True)
    a = torch.tensor(attr, device=device, requires_grad=True)
    out = interpolate_face_attributes(torch.tensor(p2f, device=device), b, a)
    np.testing.assert_array_equal(out.detach().cpu().numpy(), rast_ref.interp(p2f, bary, attr))
    gout = torch.randn_like(out)
    (out * gout).sum().backward()
    # reference gradients by autograd on the numpy-equivalent torch expression (CPU)
    bc = torch.tensor(bary, requires_grad=True)
    ac = torch.tensor(attr, requires_grad=True)
    m = torch.tensor(p2f) >= 0
    fa = ac[torch.tensor(np.where(p2f >= 0, p2f, 0))]
    oc = ((bc[..., :, None] * fa).sum(-2)) * m[..., None]
    (oc * gout.cpu()).sum().backward()
    assert_close(b.grad, bc.grad, rtol=1e-5, name="grad_bary")
    assert_close(a.grad, ac.grad, rtol=1e-4, atol_rel=1e-5, name="grad_attr")


def test_mesh_rasterizer_sphere_matches_oracle(device):
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    mesh = Meshes([verts.to(device)], [faces.verts_idx.to(device)])
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=device)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    sigma = 1e-3
    rs = RasterizationSettings(image_size=64, blur_radius=np.log(1.0 / 1e-4 - 1.0) * sigma, faces_per_pixel=50,
                               perspective_correct=False)
    frag = MeshRasterizer(cameras=cams, raster_settings=rs)(mesh)
    ms = MeshRasterizer(cameras=cams, raster_settings=rs).transform(mesh)
    fv = ms.verts_packed()[ms.faces_packed()].detach().cpu().numpy()
    rp, rz, rb, rd = rast_ref.rast_fwd(fv, [0], [faces.verts_idx.shape[0]], 64, 64, 50, rs.blur_radius,
                                       False, True, False)
    np.testing.assert_array_equal(frag.pix_to_face.cpu().numpy(), rp)
    np.testing.assert_array_equal(frag.zbuf.cpu().numpy(), rz)
    np.testing.assert_array_equal(frag.dists.cpu().numpy(), rd)
    full = (rp >= 0).sum(-1)
    assert full.max() == 50  # the blur radius fills all K slots near the sphere
