"""The fused perturbed blend at BASELINE cfg 4's full size: the 16-mesh batch (alternating
sphere_642 / cube2, seeded rotations) at 512 x 512, faces_per_pixel = 150, nb_samples = 64, with
TexturesVertex colours fused in (the bench's cfg-4 path), forward and backward.  The CPU oracle
cannot run this batch in seconds, so size-independent properties stand in for it (the oracle
parity of the same kernels is tests/test_gpu_blend.py, test_gpu_headline_parity.py):
  * repeated runs are bitwise identical (image and every gradient);
  * the backward is linear in the upstream gradient (1e-5 of the maximum);
  * alpha = 1 - prod(1 - P) with P from the standalone Heaviside on the same Philox key;
  * the 64 samples as 8 shards of 8 (one per GPU of the node, multidevice.sharded_blend's exact
    mode, logical shards on one device) reproduce the one-shard image bit for bit and its
    gradients at 1e-5, and the one-shard composition matches the fused kernel pair at 1e-5."""
import pytest
import torch

from conftest import assert_close
from pertrenderer_amd import Noise, perturbed_blend, perturbed_blend_vertex, perturbed_heaviside
from test_gpu_fullsize import SIGMA, _batch, _fragments

pytestmark = pytest.mark.gpu
SIZE, K, S, GAMMA = 512, 150, 64, 1e-2
SEEDS = (31, 32)


@pytest.fixture(scope="module")
def cfg4(device):
    mesh, cams = _batch(device)
    with torch.no_grad():
        frag = _fragments(mesh, cams, SIZE, K)
    g = torch.Generator(device).manual_seed(4)
    vcol = torch.rand((mesh.verts_packed().shape[0], 3), device=device, generator=g)
    gimg = [torch.randn((16, SIZE, SIZE, 4), device=device, generator=g) for _ in range(2)]
    assert int((frag.pix_to_face >= 0).sum()) > 10_000_000
    return mesh, frag, vcol, gimg


def _vertex_blend(mesh, frag, vcol, gimg):
    d = frag.dists.detach().clone().requires_grad_(True)
    z = frag.zbuf.detach().clone().requires_grad_(True)
    b = frag.bary_coords.detach().clone().requires_grad_(True)
    s, gm, al = (torch.tensor(v, requires_grad=True) for v in (SIGMA, GAMMA, 1.0))
    img = perturbed_blend_vertex(vcol, mesh.faces_packed(), frag.pix_to_face, b, d, z, s, gm, al, S, S,
                                 background=(0.0, 0.0, 0.0), noise=Noise.philox(seed_r=SEEDS[0], seed_a=SEEDS[1]))
    if gimg is None:
        return img.detach(), None
    (img * gimg).sum().backward()
    torch.cuda.synchronize()
    return img.detach(), dict(dists=d.grad, zbuf=z.grad, bary=b.grad, sigma=s.grad, gamma=gm.grad, alpha=al.grad)


def test_cfg4_blend_is_deterministic(cfg4):
    mesh, frag, vcol, gimg = cfg4
    i1, g1 = _vertex_blend(mesh, frag, vcol, gimg[0])
    i2, g2 = _vertex_blend(mesh, frag, vcol, gimg[0])
    assert torch.equal(i1, i2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k
    assert float(i1[..., 3].max()) > 0.5 and float(g1["dists"].abs().max()) > 0


def test_cfg4_blend_backward_is_linear_in_upstream_gradient(cfg4):
    mesh, frag, vcol, gimg = cfg4
    _, ga = _vertex_blend(mesh, frag, vcol, gimg[0])
    _, gb = _vertex_blend(mesh, frag, vcol, gimg[1])
    _, gs = _vertex_blend(mesh, frag, vcol, 2.0 * gimg[0] - 0.5 * gimg[1])
    for k in ("dists", "zbuf", "bary"):
        ref = 2.0 * ga[k] - 0.5 * gb[k]
        scale = float(ref.abs().max())
        assert scale > 0, k
        assert float((gs[k] - ref).abs().max()) <= 1e-5 * scale, k


def test_cfg4_alpha_matches_heaviside_with_same_key(cfg4):
    mesh, frag, vcol, _ = cfg4
    img, _ = _vertex_blend(mesh, frag, vcol, None)
    valid = frag.pix_to_face >= 0
    d = torch.where(valid, frag.dists, torch.zeros_like(frag.dists))
    P = perturbed_heaviside(d, torch.tensor(SIGMA), S, noise=Noise.philox(seed_r=SEEDS[0])) * valid
    alpha = 1.0 - torch.prod(1.0 - P, dim=-1)
    assert_close(img[..., 3], alpha, name="alpha")


def test_cfg4_eight_sample_shards_reproduce_the_estimator(cfg4, device):
    """multidevice.sharded_blend over 8 logical shards of 8 samples (exact mode: P summed over the
    rast shards before the agg shards) against 1 shard of 64, and that against the fused kernels."""
    from pertrenderer_amd.multidevice import sharded_blend
    mesh, frag, vcol, gimg = cfg4
    from pertrenderer_amd.renderer.interp import interpolate_vertex_attributes
    colors = interpolate_vertex_attributes(frag.pix_to_face, frag.bary_coords, vcol, mesh.faces_packed()).detach()
    # pix_to_face without the rasterizer's valid-prefix counts: with them attached, the fused
    # Philox backward draws a pixel's masked agg slots jointly (same distribution, different
    # draws -- DESIGN.md §4), while the standalone aggregate op draws every slot
    p2f = frag.pix_to_face.clone()
    outs = []
    for devices in ([device], [device] * 8, None):
        d = frag.dists.detach().clone().requires_grad_(True)
        z = frag.zbuf.detach().clone().requires_grad_(True)
        s, gm, al = (torch.tensor(v, requires_grad=True) for v in (SIGMA, GAMMA, 1.0))
        if devices is None:  # the fused kernel pair, same keys
            img = perturbed_blend(colors, p2f, d, z, s, gm, al, S, S, background=(0.0, 0.0, 0.0),
                                  noise=Noise.philox(seed_r=SEEDS[0], seed_a=SEEDS[1]))
        else:
            import pertrenderer_amd.noise as nz
            keys = iter(SEEDS)
            orig = nz.draw_key
            nz.draw_key = lambda generator=None: next(keys)  # the same two keys as the fused call
            try:
                img = sharded_blend(colors, p2f, d, z, s, gm, al, S, S, devices=devices,
                                    background=(0.0, 0.0, 0.0))
            finally:
                nz.draw_key = orig
        (img * gimg[0]).sum().backward()
        torch.cuda.synchronize()
        outs.append((img.detach(), d.grad, z.grad, torch.stack([s.grad, gm.grad, al.grad])))
        del img, d, z
    one, eight, fused = outs
    assert torch.equal(eight[0], one[0])
    for i, name in ((1, "d dists"), (2, "d zbuf")):
        assert_close(eight[i], one[i], name=name + " (8 shards)")
        assert_close(one[i], fused[i], name=name + " (composition vs fused)")
    assert_close(one[0], fused[0], name="image (composition vs fused)")
    assert_close(eight[3], one[3], rtol=2e-5, name="d sigma/gamma/alpha (8 shards)")
