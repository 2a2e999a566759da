"""The blend kernels' empty-block shortcut (pr_blend.hip: a workgroup none of whose pixels has a
valid slot writes the background / zero gradients directly) against the full phases.

On the bench frame (sphere_642 at 256^2, K = 50, Sr = Sa = 8) most workgroups cover background
only.  With Philox noise the forward image, the winners and every gradient (d dists, d zbuf,
d bary, the smoothing scalars; d vertex colours up to its float-atomic summation order) must be
bitwise equal with the shortcut on
(default) and off (PR_BLEND_EMPTY=0), for the Gaussian pair with variance reduction (the
shortcut's case) and for GaussianAgg_wovr (no baseline: the backward keeps the full path).
"""
import os

import pytest
import torch

import pertrenderer_amd as pa

pytestmark = pytest.mark.gpu


def _run(device, agg_vr, seed=5):
    import bench
    wl = bench.Workload(device, image_size=128, K=50, samples=8)
    from pertrenderer_amd.renderer import Rotate, so3_exponential_map
    R = so3_exponential_map(wl.log_rot)
    mesh = wl.base.update_padded(Rotate(R).transform_points(wl.base.verts_padded()))
    frag = wl.renderer.rasterizer(mesh, cameras=wl.cameras)
    dists = frag.dists.detach().requires_grad_(True)
    zbuf = frag.zbuf.detach().requires_grad_(True)
    bary = frag.bary_coords.detach().requires_grad_(True)
    vc = mesh.textures.verts_features_packed().detach().requires_grad_(True)
    sig, gam, alp = (torch.tensor(v, device=device, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
    noise = pa.blend.Noise.philox(seed_r=11 + seed, seed_a=23 + seed)
    img = pa.blend.perturbed_blend_vertex(vc, mesh.faces_packed(), frag.pix_to_face, bary, dists, zbuf, sig, gam,
                                          alp, 8, 8, background=(0.2, 0.4, 0.6), noise=noise, agg_vr=agg_vr)
    g = torch.randn(img.shape, device=device, generator=torch.Generator(device).manual_seed(3))
    img.backward(g)
    torch.cuda.synchronize()
    return [img.detach(), dists.grad, zbuf.grad, bary.grad, vc.grad, sig.grad, gam.grad, alp.grad]


@pytest.mark.parametrize("agg_vr", [True, False])
def test_empty_block_shortcut_is_bitwise(device, agg_vr):
    old = os.environ.get("PR_BLEND_EMPTY")
    try:
        torch.manual_seed(0)
        os.environ["PR_BLEND_EMPTY"] = "1"
        a = _run(device, agg_vr)
        os.environ["PR_BLEND_EMPTY"] = "0"
        b = _run(device, agg_vr)
    finally:
        if old is None:
            os.environ.pop("PR_BLEND_EMPTY", None)
        else:
            os.environ["PR_BLEND_EMPTY"] = old
    names = ("image", "d dists", "d zbuf", "d bary", "d vertex colours", "d sigma", "d gamma", "d alpha")
    for x, y, n in zip(a, b, names):
        if n == "d vertex colours":  # float atomics across slots: summation order varies run to run
            assert float((x - y).abs().max()) <= 1e-5 * float(y.abs().max()), n
        else:
            assert torch.equal(x, y), n
    # the frame has background-only workgroups (the shortcut ran) and foreground ones
    assert float((a[0][..., 3] == 0).float().mean()) > 0.3 and float((a[0][..., 3] > 0).float().mean()) > 0.1
