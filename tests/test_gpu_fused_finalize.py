"""The blend backward's fused scalar reduction (PRBlendFwdArgs.sync: the backward's last workgroup
forms d sigma / d gamma / d alpha from the per-block partials, no blend_finalize_kernel) against
the separate finalize kernel: the same reduction in the same order, so the scalars are bitwise
equal -- on the bench frame, with and without the segment plan, for texel and vertex colours, and
for a second backward of the same forward (the arrival counters reset themselves)."""
import contextlib
import os

import pytest
import torch

import pertrenderer_amd as pa
import pertrenderer_amd.blend as pb

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def fused(on, seg=False):
    old, old_seg = pb._FUSED_FINALIZE, os.environ.get("PR_BLEND_SEG")
    pb._FUSED_FINALIZE = on
    os.environ["PR_BLEND_SEG"] = "1" if seg else "0"
    try:
        yield
    finally:
        pb._FUSED_FINALIZE = old
        if old_seg is None:
            os.environ.pop("PR_BLEND_SEG", None)
        else:
            os.environ["PR_BLEND_SEG"] = old_seg


def _frame(device, size=192):
    import bench
    wl = bench.Workload(device, image_size=size, K=50, samples=8)
    from pertrenderer_amd.renderer import Rotate, so3_exponential_map
    R = so3_exponential_map(wl.log_rot)
    mesh = wl.base.update_padded(Rotate(R).transform_points(wl.base.verts_padded()))
    return mesh, wl.renderer.rasterizer(mesh, cameras=wl.cameras)


def _grads(device, mesh, frag, vertex, twice=False):
    sig, gam, alp = (torch.tensor(v, device=device, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
    nz = pa.blend.Noise.philox(seed_r=3, seed_a=4)
    vc = mesh.textures.verts_features_packed().detach()
    if vertex:
        img = pa.blend.perturbed_blend_vertex(vc, mesh.faces_packed(), frag.pix_to_face, frag.bary_coords,
                                              frag.dists, frag.zbuf, sig, gam, alp, 8, 8, noise=nz)
    else:
        from pertrenderer_amd.renderer.interp import interpolate_vertex_attributes
        tex = interpolate_vertex_attributes(frag.pix_to_face, frag.bary_coords, vc, mesh.faces_packed())
        img = pa.blend.perturbed_blend(tex, frag.pix_to_face, frag.dists, frag.zbuf, sig, gam, alp, 8, 8, noise=nz)
    g = torch.randn(img.shape, device=device, generator=torch.Generator(device).manual_seed(1))
    out = torch.autograd.grad(img, (sig, gam, alp), g, retain_graph=twice)
    if twice:
        again = torch.autograd.grad(img, (sig, gam, alp), g)
        for x, y in zip(out, again):
            assert torch.equal(x, y)
    return torch.stack(out)


@pytest.mark.parametrize("vertex", [True, False])
@pytest.mark.parametrize("seg", [False, True])
def test_fused_finalize_is_bitwise(device, vertex, seg):
    mesh, frag = _frame(device)
    with fused(True, seg):
        a = _grads(device, mesh, frag, vertex, twice=True)
    with fused(False, seg):
        b = _grads(device, mesh, frag, vertex)
    assert torch.isfinite(a).all() and a.abs().sum() > 0
    assert torch.equal(a, b), (a, b)
