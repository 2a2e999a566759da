"""The native autograd Functions run detached native backwards: they are marked once_differentiable,
so a second differentiation through them raises instead of silently returning gradients that
cannot be differentiated again (a create_graph=True backward still gives the first-order values)."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, assert_close

pytestmark = pytest.mark.gpu


def _frame():
    import pertrenderer_amd as pa
    from pertrenderer_amd.renderer import (FoVPerspectiveCameras, MeshRasterizer, Meshes, RasterizationSettings,
                                           load_obj, look_at_view_transform)
    dev = torch.device("cuda:0")
    v, f, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    verts = v.to(dev).requires_grad_(True)
    mesh = Meshes([verts], [f.verts_idx.to(dev)])
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=dev)
    cams = FoVPerspectiveCameras(R=R, T=T, device=dev)
    rs = RasterizationSettings(image_size=32, blur_radius=np.log(1e4 - 1) * 1e-3, faces_per_pixel=8)
    frag = MeshRasterizer(cameras=cams, raster_settings=rs)(mesh)
    sig, gam, alp = (torch.tensor(v, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
    colors = torch.rand(frag.pix_to_face.shape + (3,), device=dev, requires_grad=True)
    img = pa.perturbed_blend(colors, frag.pix_to_face, frag.dists, frag.zbuf, sig, gam, alp, 4, 4,
                             background=(0.0, 0.0, 0.0))
    return verts, colors, img


def test_second_order_raises():
    verts, colors, img = _frame()
    loss = (img[..., :3] ** 2).mean()
    gv, gc = torch.autograd.grad(loss, (verts, colors), create_graph=True)
    assert torch.isfinite(gv).all() and gv.abs().sum() > 0
    with pytest.raises(RuntimeError, match="once_differentiable"):
        (gc.sum() + gv.sum()).backward()


def test_first_order_unchanged_by_create_graph():
    torch.manual_seed(0)
    from pertrenderer_amd import set_noise_source
    set_noise_source("torch")
    try:
        torch.manual_seed(5)
        verts, colors, img = _frame()
        g1 = torch.autograd.grad((img[..., :3] ** 2).mean(), (verts, colors))
        torch.manual_seed(5)
        verts2, colors2, img2 = _frame()
        g2 = torch.autograd.grad((img2[..., :3] ** 2).mean(), (verts2, colors2), create_graph=True)
    finally:
        set_noise_source("philox")
    assert torch.equal(img, img2)
    assert torch.equal(g1[1], g2[1].detach())
    assert_close(g2[0].detach(), g1[0])  # the rasterizer backward sums with float atomics
