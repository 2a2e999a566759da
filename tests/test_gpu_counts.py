"""The rasterizer's valid-prefix counts (PRRastArgs.pix_count, attached to pix_to_face) let the
blend kernels skip every fragment read at padded slots.  Results must not change: the counts
path is compared bit for bit (up to the sign of a zero gradient at a padded slot; scalar
gradients to fp32 summation order) with the same call on a count-less copy of pix_to_face,
under injected noise.  (With Philox noise the
counts path also draws the padded agg slots jointly: tests/test_gpu_blend.py checks that
draw against the per-slot one.)"""
import os

import numpy as np
import pytest
import torch

import pertrenderer_amd as pa
from conftest import ROOT, assert_close
from pertrenderer_amd import Noise
from pertrenderer_amd.renderer import (FoVPerspectiveCameras, MeshRasterizer, Meshes, RasterizationSettings,
                                       load_obj, look_at_view_transform)
from pertrenderer_amd.renderer.rasterizer import valid_counts

pytestmark = pytest.mark.gpu


def _frags(device, size=48, K=30):
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    mesh = Meshes([verts.to(device)], [faces.verts_idx.to(device)])
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=device)
    rs = RasterizationSettings(image_size=size, blur_radius=9.2e-3, faces_per_pixel=K)
    frag = MeshRasterizer(cameras=FoVPerspectiveCameras(R=R, T=T, device=device), raster_settings=rs)(mesh)
    return mesh, frag


def _same(a, b):
    """Bitwise equal except that -0.0 == +0.0 (a padded slot's zero gradient)."""
    return a.shape == b.shape and bool(((a == b) | (a.isnan() & b.isnan())).all())


def _injected(frag, S, seed):
    N, H, W, K = frag.pix_to_face.shape
    g = torch.Generator().manual_seed(seed)
    dev = frag.pix_to_face.device
    return Noise.injected(torch.randn((S, N, H, W, K), generator=g).to(dev),
                          torch.randn((S, N, H, W, K + 1), generator=g).to(dev))


def _run(fn, p2f, leaves):
    """fn(*leaves[:-3], p2f, *leaves[-3:]) -> image; returns the image and every leaf's gradient."""
    leaves = [t.detach().clone().requires_grad_(True) for t in leaves]
    img = fn(*leaves[:-3], p2f, *leaves[-3:])
    g = torch.randn(img.shape, generator=torch.Generator().manual_seed(3)).to(img.device)
    (img * g).sum().backward()
    return img.detach(), [t.grad for t in leaves]


def test_counts_attached_and_correct(device):
    _, frag = _frags(device)
    c = valid_counts(frag.pix_to_face)
    assert c is not None and c.dtype == torch.int32
    np.testing.assert_array_equal(c.cpu().numpy(), (frag.pix_to_face >= 0).sum(-1).cpu().numpy())
    frag.pix_to_face.add_(0)  # an in-place change drops them
    assert valid_counts(frag.pix_to_face) is None


def test_fused_blend_counts_path_is_bit_identical(device):
    _, frag = _frags(device)
    N, H, W, K = frag.pix_to_face.shape
    cols = torch.rand((N, H, W, K, 3), generator=torch.Generator().manual_seed(0)).to(device)
    sc = [torch.tensor(v, device=device) for v in (1e-3, 1e-2, 1.0)]
    noise = _injected(frag, 8, 11)

    def fn(c, d, z, p2f, s, g, a):
        return pa.perturbed_blend(c, p2f, d, z, s, g, a, 8, 8, background=(0.1, 0.2, 0.3), noise=noise)

    leaves = [cols, frag.dists, frag.zbuf, *sc]
    i1, g1 = _run(fn, frag.pix_to_face, leaves)
    i2, g2 = _run(fn, frag.pix_to_face.clone(), leaves)
    assert torch.equal(i1, i2)
    for a, b in zip(g1[:-3], g2[:-3]):
        assert _same(a, b)
    for a, b in zip(g1[-3:], g2[-3:]):  # scalar partials: valid slots land on other threads
        assert_close(a, b, rtol=1e-5, name="scalar")


def test_vertex_blend_counts_path_is_bit_identical(device):
    mesh, frag = _frags(device)
    vc = torch.rand((mesh.verts_packed().shape[0], 3), generator=torch.Generator().manual_seed(1)).to(device)
    faces = mesh.faces_packed()
    sc = [torch.tensor(v, device=device) for v in (1e-3, 1e-2, 1.0)]
    noise = _injected(frag, 8, 21)

    def fn(v, b, d, z, p2f, s, g, a):
        return pa.perturbed_blend_vertex(v, faces, p2f, b, d, z, s, g, a, 8, 8, background=(0.0, 0.0, 0.0),
                                         noise=noise)

    leaves = [vc, frag.bary_coords, frag.dists, frag.zbuf, *sc]
    i1, g1 = _run(fn, frag.pix_to_face, leaves)
    i2, g2 = _run(fn, frag.pix_to_face.clone(), leaves)
    assert torch.equal(i1, i2)
    assert_close(g1[0], g2[0], rtol=1e-5, atol_rel=1e-5, name="d vert colours")  # float atomics: summation order
    for a, b in zip(g1[1:-3], g2[1:-3]):
        assert _same(a, b)
    for a, b in zip(g1[-3:], g2[-3:]):
        assert_close(a, b, rtol=1e-5, name="scalar")
