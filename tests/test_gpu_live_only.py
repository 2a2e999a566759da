"""A direct ``shader(fragments, mesh)`` call returns the reference's exact zeros in the padded rows of
d dists / d zbuf / d bary, in Philox mode (the default), for both perturbed shaders.

The reference multiplies by the fragments' mask (random_rasterizer.py:46-47, smoothagg.py:198,
smoothrast.py:55-56), so a padded slot's gradient is 0.  The native backward may leave those rows
unwritten (PR_BLEND_LIVE_ONLY / PR_SHADE_LIVE_ONLY) only when MeshRenderer's handshake
(``takes_valid_only`` -> ``_pr_valid_only``) says the fragments' one consumer is its own rasterizer
backward.  The caching allocator is poisoned with NaNs first, so rows that are not written show up.
The valid rows must be bitwise the live-only path's (same Philox keys via torch.manual_seed)."""
import math

import pytest
import torch

import pertrenderer_amd as pa
from pertrenderer_amd import noise
from pertrenderer_amd.renderer import MeshRasterizer, PointLights, RasterizationSettings
from test_gpu_shading import _scene

pytestmark = pytest.mark.gpu


def _poison(shape, device, copies=6):
    """Fill and free blocks of the gradient buffers' sizes: empty_like then reuses NaN memory."""
    N, H, W, K = shape
    bufs = []
    for _ in range(copies):
        bufs.append(torch.full((N, H, W, K), float("nan"), device=device))
        bufs.append(torch.full((N, H, W, K, 3), float("nan"), device=device))
    torch.cuda.synchronize()
    del bufs


def _render_grads(shader, rast, mesh, G, seed, **kw):
    frag = rast(mesh)
    _poison(tuple(frag.pix_to_face.shape), frag.pix_to_face.device)
    torch.manual_seed(seed)  # Philox keys come from the CPU generator (noise.draw_pair)
    img = shader(frag, mesh, **kw)
    gd, gz, gb = torch.autograd.grad((img * G).sum(), [frag.dists, frag.zbuf, frag.bary_coords])
    return frag, img.detach(), gd, gz, gb


@pytest.mark.parametrize("shader_kind,kind", [("phong", "uv"), ("phong", "vertex"), ("simple", "vertex")])
def test_direct_shader_call_zeroes_padded_rows(shader_kind, kind, device):
    assert noise.get_noise_source() == "philox"
    mesh, _, _, cams, mats, verts, _, extra = _scene(device, kind)
    lights = PointLights(device=device, location=[[0.5, 2.0, -2.0]])
    rs = RasterizationSettings(image_size=48, blur_radius=math.log(1e4 - 1) * 1e-3, faces_per_pixel=12)
    rast = MeshRasterizer(cameras=cams, raster_settings=rs)
    sr, sa = pa.GaussianRast(sigma=1e-3, nb_samples=4), pa.GaussianAgg(nb_samples=4, gamma=1e-2)
    cls = pa.RandomPhongShader if shader_kind == "phong" else pa.RandomSimpleShader
    shader = cls(device=device, cameras=cams, lights=lights, materials=mats, smoothrast=sr, smoothagg=sa)
    G = torch.rand((1, 48, 48, 4), device=device, generator=torch.Generator(device).manual_seed(7))

    frag, img, gd, gz, gb = _render_grads(shader, rast, mesh, G, 11)
    pad = frag.pix_to_face < 0
    assert 0 < int(pad.sum()) < pad.numel() and int((~pad).sum()) > 500
    for name, g in (("dists", gd), ("zbuf", gz), ("bary", gb)):
        assert bool(torch.isfinite(g).all()), name
        rows = g[pad]
        assert bool((rows == 0).all()), (name, int((rows != 0).sum()))
    assert float(gd[~pad].abs().max()) > 0 and float(gb[~pad].abs().max()) > 0

    # the renderer-internal live-only path (what MeshRenderer's handshake turns on) on the same keys:
    # the image and every valid row bit for bit
    frag2, img2, gd2, gz2, gb2 = _render_grads(shader, rast, mesh, G, 11, _pr_valid_only=True)
    assert torch.equal(frag2.pix_to_face, frag.pix_to_face)
    assert torch.equal(img2, img)
    for name, a, b in (("dists", gd, gd2), ("zbuf", gz, gz2), ("bary", gb, gb2)):
        assert torch.equal(a[~pad], b[~pad]), name
