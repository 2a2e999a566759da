"""GPU parity of the native rasterizer / interpolation against the C oracle
(oracle/rast_oracle.c; PyTorch3D 0.4.0 semantics, parity unpinned by the reference).
Forward outputs are compared bit-exactly (same fp32 operation order on both sides); the
default backward computes each slot with the oracle's operations but sums faces with float
atomics in arbitrary order, so it is compared at the 1e-5 bar (conftest.assert_close); its
deterministic mode is the oracle bit for bit (tests/test_gpu_deterministic.py)."""
import contextlib
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, assert_close
from oracle import rast_ref
from pertrenderer_amd.renderer import (FoVPerspectiveCameras, MeshRasterizer, Meshes, RasterizationSettings,
                                       interpolate_face_attributes, load_obj, look_at_view_transform,
                                       rasterize_meshes)

from pertrenderer_amd.renderer.interp import interpolate_vertex_attributes
from pertrenderer_amd.renderer.project import project_faces

pytestmark = pytest.mark.gpu


def test_native_projection_matches_transform_path(device):
    """pr_project_* == MeshRasterizer.transform + verts[faces] (PyTorch3D Transform3d math), fwd and bwd."""
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    v = verts.to(device).requires_grad_(True)
    mesh = Meshes([v], [faces.verts_idx.to(device)])
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=device)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    fv = project_faces(mesh.verts_packed(), mesh.faces_packed(), mesh.mesh_to_faces_packed_first_idx(),
                       mesh.num_faces_per_mesh(), cams.world_to_view_matrix(), cams.projection_matrix())
    ms = MeshRasterizer(cameras=cams).transform(mesh)
    ref = ms.verts_packed()[ms.faces_packed()]
    torch.testing.assert_close(fv, ref, rtol=1e-5, atol=1e-6)
    g = torch.randn_like(fv)
    (gv,) = torch.autograd.grad((fv * g).sum(), v)
    (gr,) = torch.autograd.grad((ref * g).sum(), v)
    assert_close(gv, gr, name="d verts")  # 1e-5 relative (conftest)


def test_vertex_interpolation_matches_face_gather(device):
    rng = np.random.default_rng(7)
    V, F = 50, 80
    faces = torch.tensor(rng.integers(0, V, (F, 3)), device=device)
    p2f = torch.tensor(rng.integers(-1, F, (1, 6, 7, 5)), device=device)
    bary = torch.rand((1, 6, 7, 5, 3), device=device, requires_grad=True)
    vattr = torch.randn((V, 3), device=device, requires_grad=True)
    out = interpolate_vertex_attributes(p2f, bary, vattr, faces)
    ref = interpolate_face_attributes(p2f, bary, vattr[faces])
    torch.testing.assert_close(out, ref, rtol=0, atol=0)
    g = torch.randn_like(out)
    ga = torch.autograd.grad((out * g).sum(), (bary, vattr))
    gr = torch.autograd.grad((ref * g).sum(), (bary, vattr))
    torch.testing.assert_close(ga[0], gr[0], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(ga[1], gr[1], rtol=1e-5, atol=1e-5)


def _soup(F, seed, zmin=0.5, spread=1.2, size=0.4):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-spread, spread, (F, 1, 2))
    xy = c + rng.uniform(-size, size, (F, 3, 2))
    z = rng.uniform(zmin, 5.0, (F, 3, 1))
    fv = np.concatenate([xy, z], -1).astype(np.float32)
    fv[: F // 10, :, 2] -= 6.0  # some faces behind the camera
    return fv


def _run_native(fv, first, nf, H, W, K, blur, persp, clip, cull, dev, bins=(0, 0)):
    from pertrenderer_amd.renderer.rasterizer import _rasterize
    fvt = torch.tensor(fv, device=dev, requires_grad=True)
    out = _rasterize(fvt, torch.tensor(first, device=dev), torch.tensor(nf, device=dev), H, W, K, blur,
                     persp, clip, cull, bins)
    return fvt, out


@pytest.mark.parametrize("cfg", [
    dict(H=37, W=41, K=8, blur=0.0, persp=False, clip=False, cull=False),
    dict(H=32, W=32, K=20, blur=5e-3, persp=False, clip=True, cull=False),
    dict(H=24, W=40, K=5, blur=2e-3, persp=True, clip=True, cull=True),
    dict(H=16, W=16, K=70, blur=5e-2, persp=False, clip=True, cull=False),
    # K = 1; and K > 128 (8 face slices on 4x2 tiles), on sizes that leave partial border tiles:
    # the compacted fragment pass's edge cases (empty pixels between full ones, partial tiles)
    dict(H=29, W=35, K=1, blur=5e-3, persp=False, clip=True, cull=False),
    dict(H=21, W=27, K=140, blur=8e-2, persp=False, clip=True, cull=False),
])
@pytest.mark.parametrize("bins", [(0, 0), (8, 10000), (16, 6)])
def test_rasterizer_forward_matches_oracle_bitwise(cfg, bins, device):
    """bins: no coarse bins; 8-pixel bins; 16-pixel bins of capacity 6, so that most bins overflow
    and their tiles fall back to the whole mesh.  The fragments are the same bits every way."""
    fv = np.concatenate([_soup(150, 1), _soup(90, 2)])
    first, nf = np.array([0, 150]), np.array([150, 90])
    _, (p2f, zbuf, bary, dists) = _run_native(fv, first, nf, cfg["H"], cfg["W"], cfg["K"], cfg["blur"],
                                              cfg["persp"], cfg["clip"], cfg["cull"], device, bins)
    rp, rz, rb, rd = rast_ref.rast_fwd(fv, first, nf, cfg["H"], cfg["W"], cfg["K"], cfg["blur"], cfg["persp"],
                                       cfg["clip"], cfg["cull"])
    assert (rp >= 0).sum() > 100
    np.testing.assert_array_equal(p2f.cpu().numpy(), rp)
    # the attached valid-prefix counts
    from pertrenderer_amd.renderer.rasterizer import valid_counts
    np.testing.assert_array_equal(valid_counts(p2f).cpu().numpy(), (rp >= 0).sum(-1))
    np.testing.assert_array_equal(zbuf.detach().cpu().numpy(), rz)
    np.testing.assert_array_equal(dists.detach().cpu().numpy(), rd)
    np.testing.assert_array_equal(bary.detach().cpu().numpy(), rb)


def _extreme_soup(seed):
    """Faces with corners on pixel centres (zero edge functions and projections), huge corners (a mesh
    partly behind the camera projects to such), very long edges and slivers: the forward's fast
    certain-reject stage must keep every pixel the exact test takes (pr_rast.hip dist_margin)."""
    rng = np.random.default_rng(seed)
    c = lambda i: -1.0 + (2 * i + 1) / 32.0  # pixel-centre NDC coordinate of a 32-pixel axis (exact)
    faces = []
    for _ in range(24):  # axis-aligned right triangles with corners on pixel centres
        i, j, w, h = rng.integers(0, 28), rng.integers(0, 28), rng.integers(1, 6), rng.integers(1, 6)
        faces.append([[c(i), c(j), 1.0], [c(i + w), c(j), 1.5], [c(i), c(j + h), 2.0]])
    for _ in range(16):  # huge corners crossing the image
        a = rng.uniform(-1, 1, 2)
        faces.append([[a[0], a[1], 1.0], [a[0] + 3e6, a[1] - 2e6, 2.0], [a[0] - 2e6, a[1] + 4e6, 1.5]])
    for _ in range(16):  # one very long edge
        a = rng.uniform(-1, 1, 2)
        faces.append([[a[0], a[1], 1.0], [a[0] + 5e5, a[1] + 0.3, 2.0], [a[0] + 0.2, a[1] + 0.4, 1.5]])
    for _ in range(24):  # slivers: tiny area, long edges
        a, d = rng.uniform(-0.8, 0.8, 2), rng.uniform(-1, 1, 2)
        e = rng.uniform(2e-8, 2e-6)
        faces.append([[a[0], a[1], 1.0], [a[0] + d[0], a[1] + d[1], 1.2], [a[0] + d[0] / 2 + e, a[1] + d[1] / 2, 0.8]])
    return np.asarray(faces, dtype=np.float32)


@pytest.mark.parametrize("blur,clip", [(0.0, False), (2e-3, True), (5e-2, True)])
def test_rasterizer_forward_extreme_faces_bitwise(blur, clip, device):
    """(A fixed 1e-3 blur band around the fast distance, rounds 1-4, failed here at blur 2e-3.)"""
    fv = np.concatenate([_extreme_soup(3), _soup(60, 4)])
    first, nf = np.array([0]), np.array([len(fv)])
    _, (p2f, zbuf, bary, dists) = _run_native(fv, first, nf, 32, 32, 24, blur, False, clip, False, device)
    rp, rz, rb, rd = rast_ref.rast_fwd(fv, first, nf, 32, 32, 24, blur, False, clip, False)
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
    assert_close(fvt.grad, ref, name="grad_face_verts")


@pytest.mark.parametrize("F,H,K,size", [(400, 16, 50, 0.5), (900, 20, 120, 0.9), (60, 40, 8, 0.2)])
def test_rasterizer_backward_dense_tiles(F, H, K, size, device):
    """Tiles with more valid slots than one backward round (1024) and more distinct faces than the
    tile-local transpose holds (128: the global-atomic overflow path), plus a sparse case; two meshes."""
    fv = np.concatenate([_soup(F, 11, spread=0.6, size=size), _soup(F // 2, 12, spread=0.6, size=size)])
    first, nf = np.array([0, F]), np.array([F, F // 2])
    blur = 2e-2
    fvt, (p2f, zbuf, bary, dists) = _run_native(fv, first, nf, H, H, K, blur, False, True, False, device)
    pc = p2f.cpu().numpy()
    g = np.random.default_rng(13)
    gz = g.standard_normal(zbuf.shape).astype(np.float32)
    gb = g.standard_normal(bary.shape).astype(np.float32)
    gd = g.standard_normal(dists.shape).astype(np.float32)
    loss = (zbuf * torch.tensor(gz, device=device)).sum() + (bary * torch.tensor(gb, device=device)).sum() \
        + (dists * torch.tensor(gd, device=device)).sum()
    loss.backward()
    ref = rast_ref.rast_bwd(fv, pc, gz, gb, gd, False, True)
    assert_close(fvt.grad, ref, name="grad_face_verts")
    if K >= 50:
        per_tile = (pc[0, :8, :8] >= 0).sum()
        faces_tile = len(np.unique(pc[0, :8, :8][pc[0, :8, :8] >= 0]))
        assert per_tile > 1024 and faces_tile > 128, (per_tile, faces_tile)


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
    assert_close(a.grad, ac.grad, name="grad_attr")


@pytest.mark.parametrize("size,K,dist_cam", [(64, 50, 2.7), (24, 16, 2.7), (40, 8, 6.7), (16, 150, 2.7)])
def test_mesh_rasterizer_sphere_matches_oracle(size, K, dist_cam, device):
    """Includes tiles whose culled face list exceeds one 512-face round (small images) and K=150 (cfg 4)."""
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    mesh = Meshes([verts.to(device)], [faces.verts_idx.to(device)])
    R, T = look_at_view_transform(dist_cam, 30.0, 120.0, device=device)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    sigma = 1e-3
    rs = RasterizationSettings(image_size=size, blur_radius=np.log(1.0 / 1e-4 - 1.0) * sigma, faces_per_pixel=K,
                               perspective_correct=False)
    frag = MeshRasterizer(cameras=cams, raster_settings=rs)(mesh)
    fv = project_faces(mesh.verts_packed(), mesh.faces_packed(), mesh.mesh_to_faces_packed_first_idx(),
                       mesh.num_faces_per_mesh(), cams.world_to_view_matrix(),
                       cams.projection_matrix()).cpu().numpy()
    rp, rz, rb, rd = rast_ref.rast_fwd(fv, [0], [faces.verts_idx.shape[0]], size, size, K, rs.blur_radius,
                                       False, True, False)
    np.testing.assert_array_equal(frag.pix_to_face.cpu().numpy(), rp)
    np.testing.assert_array_equal(frag.zbuf.cpu().numpy(), rz)
    np.testing.assert_array_equal(frag.dists.cpu().numpy(), rd)
    np.testing.assert_array_equal(frag.bary_coords.cpu().numpy(), rb)
    assert (rp >= 0).sum(-1).max() == min(K, 56)  # the blur radius fills all K slots somewhere (<= 56 here)


@pytest.mark.parametrize("size,K", [(256, 50), (24, 16), (64, 100)])
def test_two_wave_tiles_match_one_wave_bitwise(size, K, device, monkeypatch):
    """PR_RAST_DUO=1 (rast_fwd_kernel NW = 2: two waves per 4x4 tile, each walking alternate
    chunks of the sorted face list into its own K-queue, the output pass merging them) gives the
    one-wave kernel's fragments and valid counts bit for bit -- the cfg 2 frame, small images whose
    lists take several rounds, and K = 100 (cfg 3)."""
    from pertrenderer_amd.renderer.rasterizer import valid_counts
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    mesh = Meshes([verts.to(device)], [faces.verts_idx.to(device)])
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=device)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    rs = RasterizationSettings(image_size=size, blur_radius=np.log(1.0 / 1e-4 - 1.0) * 1e-3, faces_per_pixel=K,
                               perspective_correct=False)
    out = []
    for duo in ("0", "1"):
        monkeypatch.setenv("PR_RAST_DUO", duo)
        f = MeshRasterizer(cameras=cams, raster_settings=rs)(mesh)
        out.append((f.pix_to_face, f.zbuf, f.bary_coords, f.dists, valid_counts(f.pix_to_face)))
    for x, y in zip(*out):
        assert torch.equal(x, y)
    assert (out[0][0] >= 0).sum() > 0


def test_mesh_batch_with_one_camera_matches_single_meshes(device):
    """One camera broadcast over a batch of different meshes (PyTorch3D semantics): each image of
    the batch equals the single-mesh render, with pix_to_face offset by the mesh's first face."""
    sph, sf, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    cub, cf, _ = load_obj(os.path.join(ROOT, "tests", "golden", "cube2.obj"))
    vl = [sph.to(device), cub.to(device) * 0.5, sph.to(device) * 0.8]
    fl = [sf.verts_idx.to(device), cf.verts_idx.to(device), sf.verts_idx.to(device)]
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=device)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    rs = RasterizationSettings(image_size=40, blur_radius=9.2e-3, faces_per_pixel=12)
    rast = MeshRasterizer(cameras=cams, raster_settings=rs)
    batch = rast(Meshes(vl, fl))
    first = 0
    for i in range(3):
        single = rast(Meshes([vl[i]], [fl[i]]))
        p = single.pix_to_face[0]
        np.testing.assert_array_equal(batch.pix_to_face[i].cpu().numpy(), torch.where(p >= 0, p + first, p).cpu().numpy())
        np.testing.assert_array_equal(batch.zbuf[i].cpu().numpy(), single.zbuf[0].cpu().numpy())
        np.testing.assert_array_equal(batch.dists[i].cpu().numpy(), single.dists[0].cpu().numpy())
        first += fl[i].shape[0]
    assert (batch.pix_to_face >= 0).sum() > 100


def test_fused_projection_rasterizer_matches_separate_ops(device):
    """pr_project_rast_fwd (MeshRasterizer's fast path) == pr_project_fwd + pr_rast_fwd: fragments
    bit for bit; d verts through the pre-zeroed accumulators == through the memset path (float
    atomics: summation order), including a second backward (retain_graph)."""
    from pertrenderer_amd.renderer.rasterizer import _rasterize
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=device)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    rs = RasterizationSettings(image_size=48, blur_radius=9.2e-3, faces_per_pixel=20)
    g = torch.Generator().manual_seed(5)
    gz, gb, gd = (torch.randn(s, generator=g).to(device) for s in ((1, 48, 48, 20), (1, 48, 48, 20, 3), (1, 48, 48, 20)))
    v1 = verts.to(device).requires_grad_(True)
    m1 = Meshes([v1], [faces.verts_idx.to(device)])
    fr = MeshRasterizer(cameras=cams, raster_settings=rs)(m1)
    loss1 = (fr.zbuf * gz).sum() + (fr.bary_coords * gb).sum() + (fr.dists * gd).sum()
    loss1.backward(retain_graph=True)
    g1 = v1.grad.clone()
    v1.grad = None
    loss1.backward()
    g1b = v1.grad.clone()
    v2 = verts.to(device).requires_grad_(True)
    m2 = Meshes([v2], [faces.verts_idx.to(device)])
    fv = project_faces(m2.verts_packed(), m2.faces_packed(), m2.mesh_to_faces_packed_first_idx(),
                       m2.num_faces_per_mesh(), cams.world_to_view_matrix(), cams.projection_matrix())
    p2f, zbuf, bary, dists = _rasterize(fv, m2.mesh_to_faces_packed_first_idx(), m2.num_faces_per_mesh(), 48, 48, 20,
                                        9.2e-3, False, True, False)
    for a, b in ((fr.pix_to_face, p2f), (fr.zbuf, zbuf), (fr.bary_coords, bary), (fr.dists, dists)):
        assert torch.equal(a, b)
    ((zbuf * gz).sum() + (bary * gb).sum() + (dists * gd).sum()).backward()
    assert_close(g1, v2.grad, name="d verts")
    assert_close(g1b, v2.grad, name="d verts (second backward)")


@pytest.mark.parametrize("bin_size,mfpb", [(8, None), (16, 300), (None, None)])
def test_rasterizer_large_mesh_bins_match_oracle(bin_size, mfpb, device):
    """An 81 920-face sphere (sphere_642 subdivided 3x) through MeshRasterizer at 64x64, K=20 with
    blur: PyTorch3D's bins for this size (8 px, capacity max(10000, F/5)), 16-px bins with a
    300-face capacity that the central bins overflow, and the naive path (None) -- all bit-exact
    against the C oracle."""
    import meshgen
    from pertrenderer_amd.renderer.rasterizer import valid_counts
    v, f = meshgen.fine_sphere(3)
    assert f.shape[0] == 81920
    mesh = Meshes([torch.tensor(v, device=device)], [torch.tensor(f, device=device)])
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=device)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    H, K, blur = 64, 20, 2e-4
    rs = RasterizationSettings(image_size=H, blur_radius=blur, faces_per_pixel=K, bin_size=bin_size,
                               max_faces_per_bin=mfpb)
    with torch.no_grad():
        frag = MeshRasterizer(cameras=cams, raster_settings=rs)(mesh)
    fv = project_faces(mesh.verts_packed(), mesh.faces_packed(), mesh.mesh_to_faces_packed_first_idx(),
                       mesh.num_faces_per_mesh(), cams.world_to_view_matrix(), cams.projection_matrix())
    rp, rz, rb, rd = rast_ref.rast_fwd(fv.cpu().numpy(), [0], [f.shape[0]], H, H, K, blur, False, True, False)
    assert (rp >= 0).sum(-1).max() == K  # deep pixels: the K-truncation is exercised
    np.testing.assert_array_equal(frag.pix_to_face.cpu().numpy(), rp)
    np.testing.assert_array_equal(valid_counts(frag.pix_to_face).cpu().numpy(), (rp >= 0).sum(-1))
    np.testing.assert_array_equal(frag.zbuf.cpu().numpy(), rz)
    np.testing.assert_array_equal(frag.dists.cpu().numpy(), rd)
    np.testing.assert_array_equal(frag.bary_coords.cpu().numpy(), rb)


@pytest.mark.parametrize("layer", ["c++", "python"])
def test_device_blur_radius_matches_float_and_replays(layer, device):
    """RasterizationSettings.blur_radius as a one-element float32 device tensor
    (PRRastArgs.blur_radius_dev, ABI 18): fragments equal the float threshold's bit for bit; a
    captured forward replays with the value last written into the tensor (pose_opt's graph mode
    lowers the blur in place instead of capturing again)."""
    from pertrenderer_amd import host_layer
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    mesh = Meshes([verts.to(device)], [faces.verts_idx.to(device)])
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=device)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    b1, b2 = 9.2e-3, 2.1e-3

    def run(blur):
        rs = RasterizationSettings(image_size=64, blur_radius=blur, faces_per_pixel=20, perspective_correct=False)
        return MeshRasterizer(cameras=cams, raster_settings=rs)(mesh)

    ctx = host_layer.disabled() if layer == "python" else contextlib.nullcontext()
    with ctx:
        ref1, ref2 = run(b1), run(b2)
        bt = torch.tensor(b1, dtype=torch.float32, device=device)
        got = run(bt)
        for x, y in zip(got, ref1):
            assert torch.equal(x, y)
        assert not torch.equal(ref1.pix_to_face, ref2.pix_to_face)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            run(bt)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = run(bt)
        bt.fill_(b2)
        g.replay()
        torch.cuda.synchronize()
        for x, y in zip(out, ref2):
            assert torch.equal(x, y)
