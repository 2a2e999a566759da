"""Parity at BASELINE.json's full batch sizes (cfg 3: 16 x 256^2, K=100, S=16; cfg 4: 16 x
512^2, K=150, S=64), where the CPU oracles cannot run the whole batch in seconds:
* rasterizer: two images of the cfg-4 batch (a sphere and a cube) against the C oracle,
  bit-exact; structure of all 16 (valid prefix = the attached counts, depth order, face
  ids inside each mesh's range) checked on the GPU;
* blend (Philox): size-independent properties -- sample shards partition the
  Heaviside estimator exactly, the backward is linear in the upstream gradient, repeated
  runs are bitwise identical, and alpha = 1 - prod(1 - P) against the standalone
  Heaviside with the same keys."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import rast_ref
from pertrenderer_amd import Noise, perturbed_blend, perturbed_heaviside
from pertrenderer_amd.renderer import (FoVPerspectiveCameras, MeshRasterizer, Meshes, RasterizationSettings,
                                       load_obj, look_at_view_transform, random_rotations)
from pertrenderer_amd.renderer.project import project_faces
from pertrenderer_amd.renderer.rasterizer import valid_counts

pytestmark = pytest.mark.gpu
SIGMA = 1e-3
BLUR = float(np.log(1.0 / 1e-4 - 1.0) * SIGMA)


def _batch(device, n=16):
    """16 meshes alternating sphere_642 / cube2, each rotated by a seeded
    random rotation."""
    sph, sf, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    cub, cf, _ = load_obj(os.path.join(ROOT, "tests", "golden", "cube2.obj"))
    torch.manual_seed(1)
    Rs = random_rotations(n)
    vl, fl = [], []
    for i in range(n):
        v, f = (sph, sf) if i % 2 == 0 else (cub * 0.6, cf)
        vl.append((v @ Rs[i].T).to(device))
        fl.append(f.verts_idx.to(device))
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=device)
    return Meshes(vl, fl), FoVPerspectiveCameras(R=R, T=T, device=device)


def _fragments(mesh, cams, size, K, **kw):
    rs = RasterizationSettings(image_size=size, blur_radius=BLUR, faces_per_pixel=K, perspective_correct=False, **kw)
    return MeshRasterizer(cameras=cams, raster_settings=rs)(mesh)


@pytest.mark.parametrize("bin_size,mfpb", [(8, None), (64, 200)])
def test_cfg4_coarse_bins_do_not_change_fragments(bin_size, mfpb, device):
    """The whole cfg 4 batch: PyTorch3D's default bins (32 px at 512^2), 8-px bins and 64-px bins
    whose 200-face capacity overflows (those tiles cull the whole mesh) all give the naive path's
    fragments bit for bit."""
    size, K = 512, 150
    mesh, cams = _batch(device)
    with torch.no_grad():
        ref = _fragments(mesh, cams, size, K, bin_size=0)
        for f in (_fragments(mesh, cams, size, K), _fragments(mesh, cams, size, K, bin_size=bin_size,
                                                               max_faces_per_bin=mfpb)):
            assert torch.equal(f.pix_to_face, ref.pix_to_face)
            assert torch.equal(valid_counts(f.pix_to_face), valid_counts(ref.pix_to_face))
            for a, b in ((f.zbuf, ref.zbuf), (f.bary_coords, ref.bary_coords), (f.dists, ref.dists)):
                assert torch.equal(a.view(torch.int32), b.view(torch.int32))


def test_cfg4_rasterizer_batch(device):
    size, K = 512, 150
    mesh, cams = _batch(device)
    with torch.no_grad():
        frag = _fragments(mesh, cams, size, K)
    p2f, zbuf = frag.pix_to_face, frag.zbuf
    assert p2f.shape == (16, size, size, K)
    # structure of the whole batch (on the GPU)
    cnt = valid_counts(p2f)
    assert cnt is not None and cnt.shape == (16, size, size)
    ks = torch.arange(K, device=device)
    valid = p2f >= 0
    assert torch.equal(valid, ks < cnt[..., None].long())
    zn = torch.where(valid, zbuf, torch.full_like(zbuf, float("inf")))
    assert bool((zn[..., 1:] >= zn[..., :-1]).all())
    first = mesh.mesh_to_faces_packed_first_idx().view(-1, 1, 1, 1)
    nf = mesh.num_faces_per_mesh().view(-1, 1, 1, 1)
    inside = (p2f >= first) & (p2f < first + nf)
    assert bool(torch.where(valid, inside, torch.ones_like(inside)).all())
    assert int(cnt.max()) > 50  # the blur radius fills far more than cfg 2's K somewhere
    # two images against the C oracle, bit-exact
    fv_all = project_faces(mesh.verts_packed(), mesh.faces_packed(), mesh.mesh_to_faces_packed_first_idx(),
                           mesh.num_faces_per_mesh(), cams.world_to_view_matrix(), cams.projection_matrix())
    for n in (0, 1):
        f0, f1 = int(first[n]), int(first[n] + nf[n])
        fv = fv_all[f0:f1].cpu().numpy()
        rp, rz, rb, rd = rast_ref.rast_fwd(fv, [0], [f1 - f0], size, size, K, BLUR, False, True, False)
        got = p2f[n].cpu().numpy()
        np.testing.assert_array_equal(np.where(got >= 0, got - f0, -1), rp[0])
        np.testing.assert_array_equal(zbuf[n].cpu().numpy(), rz[0])
        np.testing.assert_array_equal(frag.dists[n].cpu().numpy(), rd[0])
        np.testing.assert_array_equal(frag.bary_coords[n].cpu().numpy(), rb[0])


@pytest.fixture(scope="module")
def cfg3(device):
    size, K, S = 256, 100, 16
    mesh, cams = _batch(device)
    with torch.no_grad():
        frag = _fragments(mesh, cams, size, K)
    g = torch.Generator().manual_seed(3)
    colors = torch.rand((16, size, size, K, 3), generator=g).to(device)
    gimg = [torch.randn((16, size, size, 4), generator=g).to(device) for _ in range(2)]
    return frag, colors, gimg, S


def _blend(frag, colors, S, gimg, seed=(21, 22)):
    d = frag.dists.detach().clone().requires_grad_(True)
    z = frag.zbuf.detach().clone().requires_grad_(True)
    c = colors.clone().requires_grad_(True)
    s, gm, al = (torch.tensor(v, requires_grad=True) for v in (SIGMA, 1e-2, 1.0))
    img = perturbed_blend(c, frag.pix_to_face, d, z, s, gm, al, S, S, background=(0.0, 0.0, 0.0),
                          noise=Noise.philox(seed_r=seed[0], seed_a=seed[1]))
    if gimg is not None:
        (img * gimg).sum().backward()
        return img.detach(), dict(dists=d.grad, zbuf=z.grad, colors=c.grad, sigma=s.grad, gamma=gm.grad,
                                  alpha=al.grad)
    return img.detach(), None


def test_cfg3_blend_is_deterministic(cfg3):
    frag, colors, gimg, S = cfg3
    i1, g1 = _blend(frag, colors, S, gimg[0])
    i2, g2 = _blend(frag, colors, S, gimg[0])
    assert torch.equal(i1, i2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


def test_cfg3_blend_backward_is_linear_in_upstream_gradient(cfg3):
    frag, colors, gimg, S = cfg3
    _, ga = _blend(frag, colors, S, gimg[0])
    _, gb = _blend(frag, colors, S, gimg[1])
    _, gs = _blend(frag, colors, S, 2.0 * gimg[0] - 0.5 * gimg[1])
    for k in ("dists", "zbuf", "colors"):
        ref = 2.0 * ga[k] - 0.5 * gb[k]
        scale = float(ref.abs().max())
        assert scale > 0, k
        err = float((gs[k] - ref).abs().max())
        assert err <= 1e-5 * scale, (k, err, scale)


def test_cfg3_alpha_matches_heaviside_with_same_keys(cfg3):
    """Image alpha = 1 - prod_k (1 - P_k) with P from the standalone Heaviside (same Philox keys)."""
    frag, colors, _, S = cfg3
    img, _ = _blend(frag, colors, S, None)
    valid = frag.pix_to_face >= 0
    d = torch.where(valid, frag.dists, torch.zeros_like(frag.dists))
    P = perturbed_heaviside(d, torch.tensor(SIGMA), S, noise=Noise.philox(seed_r=21)) * valid
    alpha = 1.0 - torch.prod(1.0 - P, dim=-1)
    torch.testing.assert_close(img[..., 3], alpha, rtol=1e-5, atol=1e-6)


def test_cfg4_heaviside_sample_shards_partition_the_estimator(device):
    """cfg 4's 64 samples as 8 shards of 8 (one per GPU of the node): the mean of the shard
    estimates equals the 64-sample estimate exactly (P = count / S)."""
    g = torch.Generator().manual_seed(4)
    d = ((torch.rand((16, 512, 512, 150), generator=g) - 0.5) * 8 * SIGMA).to(device)
    s = torch.tensor(SIGMA)
    full = perturbed_heaviside(d, s, 64, noise=Noise.philox(seed_r=99))
    acc = torch.zeros_like(full)
    for r in range(8):
        acc += perturbed_heaviside(d, s, 8, noise=Noise.philox(seed_r=99, offset_r=8 * r))
    torch.testing.assert_close(acc / 8, full, rtol=0, atol=0)
