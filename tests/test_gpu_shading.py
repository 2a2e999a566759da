"""Native Phong shading (pr_shade_fwd / pr_shade_bwd) against the PyTorch3D phong_shading
composition (renderer.shading.phong_shading_reference: the same formulas as torch ops, PyTorch3D's
op order) evaluated in float64, for the three texel sources: given texels, TexturesVertex and
TexturesUV (bilinear map lookup).  Gradients: vertex positions (through both the shading and the
rasterizer's barycentrics), vertex colours, UV maps, the light position and the camera centre --
the parameters eval.py's check_differentiability optimises (eval.py:693-725)."""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

from conftest import ROOT, assert_close
from pertrenderer_amd.renderer import (FoVPerspectiveCameras, Materials, MeshRasterizer, Meshes, PointLights,
                                       RasterizationSettings, TexturesUV, TexturesVertex, load_obj,
                                       look_at_view_transform)
from pertrenderer_amd.renderer import shading as sh
from pertrenderer_amd.renderer.renderer import DirectionalLights

pytestmark = pytest.mark.gpu


def _interp64(p2f, bary, attr, faces):
    """interpolate_face_attributes in float64 torch (0 on padded slots)."""
    mask = (p2f >= 0)[..., None]
    fa = attr[faces[p2f.clamp(min=0)]]  # (...,3,D)
    out = (bary[..., 0:1] * fa[..., 0, :] + bary[..., 1:2] * fa[..., 1, :]) + bary[..., 2:3] * fa[..., 2, :]
    return out * mask


def _uv_sample64(p2f, bary, tex, dtype=torch.float64):
    uv = _interp64(p2f, bary, torch.cat([tex.verts_uvs_list()[0]]).to(dtype), tex.faces_uvs_list()[0])
    N, Ho, Wo, K = p2f.shape
    maps = tex.maps_padded().to(dtype)
    m = torch.flip(maps.permute(0, 3, 1, 2), [2])
    g = uv.reshape(N, Ho, Wo * K, 2) * 2.0 - 1.0
    t = Fn.grid_sample(m, g, align_corners=True, padding_mode="border")
    return t.reshape(N, 3, Ho, Wo, K).permute(0, 2, 3, 4, 1)


def _reference64(mesh, frag, lights, cams, mats, texels, dtype=torch.float64):
    d = lambda t: t.to(dtype)
    verts, faces = d(mesh.verts_packed()), mesh.faces_packed()
    # area-weighted vertex normals in float64 (Meshes.verts_normals_packed)
    fv = verts[faces]
    n = torch.zeros_like(verts)
    n = n.index_add(0, faces[:, 1], torch.cross(fv[:, 2] - fv[:, 1], fv[:, 0] - fv[:, 1], dim=1))
    n = n.index_add(0, faces[:, 2], torch.cross(fv[:, 0] - fv[:, 2], fv[:, 1] - fv[:, 2], dim=1))
    n = n.index_add(0, faces[:, 0], torch.cross(fv[:, 1] - fv[:, 0], fv[:, 2] - fv[:, 0], dim=1))
    vn = Fn.normalize(n, eps=1e-6, dim=1)
    p2f, bary = frag.pix_to_face, d(frag.bary_coords)
    coords, normals = _interp64(p2f, bary, verts, faces), _interp64(p2f, bary, vn, faces)
    N = coords.shape[0]
    e = lambda t: d(t).expand(N, -1) if t.shape[0] == 1 else d(t)
    if isinstance(lights, DirectionalLights):
        direction = sh._bc(e(lights.location), coords).expand_as(coords)
    else:
        direction = sh._bc(e(lights.location), coords) - coords
    diffuse = sh._diffuse(normals, e(lights.diffuse_color), direction)
    specular = sh._specular(coords, normals, direction, e(cams.get_camera_center()), e(lights.specular_color),
                            e(mats.shininess.reshape(-1, 1)).reshape(-1))
    ambient = sh._bc(e(mats.ambient_color * lights.ambient_color), coords)
    return (ambient + sh._bc(e(mats.diffuse_color), coords) * diffuse) * d(texels) \
        + sh._bc(e(mats.specular_color), coords) * specular


def _scene(device, kind, light_kind="point", size=48, K=12, uv_shift=0.0):
    torch.manual_seed(3)
    if kind == "uv":
        from pertrenderer_amd.pose_opt import load_cube
        mesh = load_cube(device)
        tex = mesh.textures
        verts = mesh.verts_packed().clone()
        faces = mesh.faces_packed()
        maps = tex.maps_padded().clone().requires_grad_(True)
        Hm, Wm = maps.shape[1:3]
        # uv_shift (texels): moves the cube's per-face constant UVs (all three corners of a face
        # share one UV, at y = 0.5 of the map: a texel row exactly) off the texel grid
        shift = torch.tensor([uv_shift / (Wm - 1), uv_shift / (Hm - 1)], device=device)
        tex = TexturesUV(maps, [tex.faces_uvs_list()[0]], [tex.verts_uvs_list()[0] + shift])
        extra = maps
    else:
        v, f, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
        verts, faces = v.to(device), f.verts_idx.to(device)
        extra = torch.rand((verts.shape[0], 3), device=device).requires_grad_(True)
        tex = TexturesVertex([extra])
    verts = (verts - verts.mean(0)).requires_grad_(True)
    mesh = Meshes([verts], [faces], tex)
    R, T = look_at_view_transform(2.2 if kind != "uv" else 3.0, 25.0, 40.0, device=device)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    loc = torch.tensor([[0.5, 2.0, -2.0]] if light_kind == "point" else [[0.3, 1.0, 0.4]], device=device,
                       requires_grad=True)
    lights = (PointLights(device=device, location=loc) if light_kind == "point"
              else DirectionalLights(device=device, direction=loc))
    lights.location = loc  # keep the leaf (PointLights stores a reshaped view)
    mats = Materials(device=device, shininess=32)
    rs = RasterizationSettings(image_size=size, blur_radius=math.log(1e4 - 1) * 1e-3, faces_per_pixel=K)
    frag = MeshRasterizer(cameras=cams, raster_settings=rs)(mesh)
    return mesh, frag, lights, cams, mats, verts, loc, extra


def _grads(out, G, leaves):
    gs = torch.autograd.grad((out * G).sum(), leaves, allow_unused=True, retain_graph=True)
    return [torch.zeros_like(l) if g is None else g for g, l in zip(gs, leaves)]


def _close(a, b, rtol, name):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    scale = float(b.abs().max())
    err = float((a - b).abs().max())
    assert err <= rtol * max(scale, 1e-12), (name, err, scale)


@pytest.mark.parametrize("kind,light_kind", [("vertex", "point"), ("uv", "point"), ("given", "point"),
                                             ("vertex", "directional")])
def test_native_shading_matches_float64_reference(kind, light_kind, device):
    mesh, frag, lights, cams, mats, verts, loc, extra = _scene(device, kind, light_kind)
    valid = (frag.pix_to_face >= 0).sum()
    assert valid > 500
    if kind == "given":
        texels = mesh.sample_textures(frag).detach().requires_grad_(True)
        out = sh.phong_shading(mesh, frag, lights, cams, mats, texels)
        leaves = [verts, loc, texels]
        ref_tex = texels
    else:
        out = sh.textured_phong_shading(mesh, frag, lights, cams, mats)
        leaves = [verts, loc, extra]
        ref_tex = (_uv_sample64(frag.pix_to_face, frag.bary_coords.double(), mesh.textures) if kind == "uv"
                   else _interp64(frag.pix_to_face, frag.bary_coords.double(), extra.double(), mesh.faces_packed()))
    ref = _reference64(mesh, frag, lights, cams, mats, ref_tex)
    _close(out, ref, 5e-6, "colors")  # fp32 kernel vs the fp64 composition
    G = torch.randn(out.shape, device=device, generator=torch.Generator(device).manual_seed(5))
    # only valid slots carry gradient in the renderer (the blend's weights are 0 elsewhere)
    G = G * (frag.pix_to_face >= 0)[..., None]
    got = _grads(out, G, leaves)
    exp = _grads(ref, G.double(), leaves)
    for name, a, b in zip(("verts", "light", "texture"), got, exp):
        _close(a, b, 2e-4, name)


def test_native_shading_camera_gradient(device):
    """d colour / d camera centre through the specular term (camera parameters with grad take the
    transform path of MeshRasterizer: eval.py's camera check)."""
    mesh, frag, lights, cams, mats, verts, loc, extra = _scene(device, "vertex")
    T = cams.T.clone().requires_grad_(True)
    cams.T = T
    out = sh.textured_phong_shading(mesh, frag, lights, cams, mats)
    ref = _reference64(mesh, frag, lights, cams, mats,
                       _interp64(frag.pix_to_face, frag.bary_coords.double(), extra.double(), mesh.faces_packed()))
    G = torch.randn(out.shape, device=device) * (frag.pix_to_face >= 0)[..., None]
    (ga,) = torch.autograd.grad((out * G).sum(), [T], retain_graph=True)
    (gb,) = torch.autograd.grad((ref * G.double()).sum(), [T])
    _close(ga, gb, 2e-4, "camera T")
    assert float(ga.abs().sum()) > 0


@pytest.mark.parametrize("layer", ["python", "c++"])
def test_renderer_uses_native_shading(device, layer):
    """RandomPhongShader / HardPhongShader route TexturesUV and TexturesVertex through pr_shade, in
    the Python Functions and in the C++ autograd layer (host_layer.py)."""
    import pertrenderer_amd.renderer.shading as shm
    from pertrenderer_amd import _native as nat
    from pertrenderer_amd import host_layer
    from pertrenderer_amd.renderer import HardPhongShader
    mesh, frag, lights, cams, mats, *_ = _scene(device, "uv")
    calls = []
    if layer == "c++":
        ext = host_layer.get()
        assert ext is not None, host_layer.error()

        class Counting:
            def __getattr__(self, name):
                fn = getattr(ext, name)
                if name != "shade":
                    return fn
                return lambda *a: calls.append(a[-3]) or fn(*a)  # (..., mode, directional, live_only)

        orig_get = host_layer.get
        try:
            host_layer.get = lambda: Counting()
            HardPhongShader(device=device, cameras=cams, lights=lights)(frag, mesh)
        finally:
            host_layer.get = orig_get
        assert calls == [nat.PR_TEX_UV]
        return
    orig = shm._ShadeFn.apply
    try:
        shm._ShadeFn.apply = lambda *a: calls.append(a[-1]["mode"]) or orig(*a)
        with host_layer.disabled():
            HardPhongShader(device=device, cameras=cams, lights=lights)(frag, mesh)
    finally:
        shm._ShadeFn.apply = orig
    assert calls == [nat.PR_TEX_UV]


@pytest.mark.parametrize("kind", ["vertex", "uv"])
def test_native_shading_matches_float32_composition(kind, device):
    """At the reference's own precision: the same torch composition in float32 (PyTorch3D's
    phong_shading op order), with the deterministic-order backward (torch.use_deterministic_
    algorithms: per-vertex / per-texel sums in slot order).  Colours and the shading's own
    gradients (barycentrics, vertices, light, vertex colours / texture map) at the 1e-5 bar; the
    fragments are fixed inputs here (the rasterizer backward has its own bitwise oracle tests:
    composed with it, ulp-level d bary differences are amplified by the 1 / face-area factors)."""
    from pertrenderer_amd.renderer.rasterizer import Fragments
    old = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)  # the reference's grid_sample backward has none
    try:
        # the cube's UVs sit on a texel row (see _scene): shifted off it, so that d bary is compared
        mesh, frag, lights, cams, mats, verts, loc, extra = _scene(device, kind, uv_shift=0.3)
        b = frag.bary_coords.detach().clone().requires_grad_(True)
        fr = Fragments(frag.pix_to_face, frag.zbuf.detach(), b, frag.dists.detach())
        vd = verts.detach().clone().requires_grad_(True)
        m = Meshes([vd], [mesh.faces_packed()], mesh.textures)
        out = sh.textured_phong_shading(m, fr, lights, cams, mats)
        ref_tex = (_uv_sample64(fr.pix_to_face, b, m.textures, torch.float32) if kind == "uv"
                   else _interp64(fr.pix_to_face, b, extra, m.faces_packed()))
        ref = _reference64(m, fr, lights, cams, mats, ref_tex, dtype=torch.float32)
        assert_close(out, ref, name="colors")
        G = torch.randn(out.shape, device=device, generator=torch.Generator(device).manual_seed(5))
        G = G * (frag.pix_to_face >= 0)[..., None]
        leaves = [b, vd, loc, extra]
        names = ("bary", "verts", "light", "texture" if kind == "uv" else "vertex colours")
        got, exp = _grads(out, G, leaves), _grads(ref, G, leaves)
        if kind == "uv":
            # bilinear sampling is not differentiable on texel grid lines: a slot whose map
            # coordinate lies within 1e-4 texel of one takes a one-sided derivative there, and
            # which side depends on the last ulp of its coordinate (torch's grid_sample
            # contracts to FMAs); those slots' d bary are left out, every other value is compared
            tex = m.textures
            uv = _interp64(fr.pix_to_face, b.detach().double(), tex.verts_uvs_list()[0].double(),
                           tex.faces_uvs_list()[0])
            Hm, Wm = tex.maps_padded().shape[1:3]
            ix, iy = uv[..., 0] * (Wm - 1), uv[..., 1] * (Hm - 1)
            edge = lambda c: (c - c.round()).abs() < 1e-4
            keep = ~(edge(ix) | edge(iy))
            assert float(keep[fr.pix_to_face >= 0].float().mean()) > 0.9
            got[0], exp[0] = got[0] * keep[..., None], exp[0] * keep[..., None]
            # d bary through the map is a sum of terms scaled by the bilinear derivative's (Wm - 1)
            # = 974 texels per unit u that cancel to values ~1e-2 of them: fp32 rounding of those
            # terms (ulp ~1e-5 of the final value) differs with the operation order, the
            # reference's own included.  So d bary is held to the reference's own float32 error:
            # against the float64 composition, the native values' worst and RMS errors may be at
            # most twice those of torch's float32 composition
            ref64 = _reference64(m, fr, lights, cams, mats,
                                 _uv_sample64(fr.pix_to_face, b, m.textures, torch.float64), dtype=torch.float64)
            e64 = _grads(ref64, G.double(), [b])[0].detach().double() * keep[..., None]
            err_nat, err_ref = got[0].double() - e64, exp[0].double() - e64
            floor = 1e-7 * float(e64.abs().max())
            assert float(err_nat.abs().max()) <= 2.0 * float(err_ref.abs().max()) + floor
            assert float(err_nat.norm()) <= 2.0 * float(err_ref.norm()) + floor
            names, got, exp = names[1:], got[1:], exp[1:]
        for name, x, y in zip(names, got, exp):
            assert_close(x, y, name=name)
    finally:
        torch.use_deterministic_algorithms(old)


@pytest.mark.parametrize("counts", [True, False])
def test_tiny_frames_shade_as_one_frame(device, counts):
    """Frames of a few slots: a 2048-slot chunk of the shading kernels then spans more images than
    its LDS table of per-image padded terms holds (pr_shade.hip pad_table), so padded slots take
    the direct path.  The 48x48 frame cut into 576 frames of 2x2 pixels (the same light, camera and
    materials on every row) shades bit for bit as the one frame, forward and backward, with the
    valid-prefix counts attached or not."""
    from pertrenderer_amd.renderer.rasterizer import Fragments, valid_counts
    mesh, frag, lights, cams, mats, verts, loc, extra = _scene(device, "vertex")
    N, H, W, K = frag.pix_to_face.shape
    b = frag.bary_coords.detach().clone().requires_grad_(True)
    one = Fragments(frag.pix_to_face, frag.zbuf.detach(), b, frag.dists.detach())
    assert valid_counts(one.pix_to_face) is not None
    out1 = sh.textured_phong_shading(mesh, one, lights, cams, mats)
    n = H * W // 4
    p2f = frag.pix_to_face.reshape(n, 2, 2, K).clone()
    if counts:
        c = valid_counts(frag.pix_to_face).reshape(n, 2, 2)
        p2f._pr_valid_counts = (p2f._version, c)
    bt = b.reshape(n, 2, 2, K, 3)
    tiny = Fragments(p2f, frag.zbuf.detach().reshape(n, 2, 2, K), bt, frag.dists.detach().reshape(n, 2, 2, K))
    assert (valid_counts(tiny.pix_to_face) is not None) == counts
    outn = sh.textured_phong_shading(mesh, tiny, lights, cams, mats)
    assert torch.equal(outn.reshape(out1.shape), out1)
    G = torch.randn(out1.shape, device=device, generator=torch.Generator(device).manual_seed(9))
    g1 = torch.autograd.grad((out1 * G).sum(), [b, extra], retain_graph=True)
    gn = torch.autograd.grad((outn * G.reshape(outn.shape)).sum(), [b, extra])
    assert torch.equal(g1[0], gn[0])
    # float atomics: the per-vertex sums' order differs (entries that cancel keep an absolute error)
    torch.testing.assert_close(g1[1], gn[1], rtol=1e-5, atol=1e-6 * float(g1[1].abs().max()))


@pytest.mark.parametrize("kind", ["vertex", "uv"])
def test_pixel_block_kernels_match_the_slot_kernels(kind, device, monkeypatch):
    """With the valid-prefix counts attached the shading forward runs as pixel blocks (padded slots
    written as 16-byte stores of the image's colour pattern, live slots enumerated from the counts'
    prefix, pr_shade.hip shade_fwd_pix_kernel); PR_SHADE_PIX=0 forces the per-wave chunk kernel.
    Colours bit for bit (and the backward, one kernel for both, on them); on a batch of 3 frames
    whose pixel blocks straddle image boundaries (48^2 pixels = 36 blocks of 64)."""
    from pertrenderer_amd.renderer.rasterizer import Fragments, valid_counts
    mesh, frag, lights, cams, mats, verts, loc, extra = _scene(device, kind)
    assert valid_counts(frag.pix_to_face) is not None
    N = 3
    p2f = frag.pix_to_face.expand(N, -1, -1, -1).contiguous()
    p2f._pr_valid_counts = (p2f._version, valid_counts(frag.pix_to_face).expand(N, -1, -1).contiguous())
    b = frag.bary_coords.detach().expand(N, -1, -1, -1, -1).contiguous().requires_grad_(True)
    fr = Fragments(p2f, frag.zbuf.detach().expand(N, -1, -1, -1), b, frag.dists.detach().expand(N, -1, -1, -1))
    if kind == "uv":
        tex = mesh.textures
        maps = tex.maps_padded().expand(N, -1, -1, -1).contiguous().detach().requires_grad_(True)
        m = Meshes([verts] * N, [mesh.faces_packed()] * N,
                   TexturesUV(maps, tex.faces_uvs_list() * N, tex.verts_uvs_list() * N))
        leaf = maps
    else:
        m = Meshes([verts] * N, [mesh.faces_packed()] * N, TexturesVertex([extra] * N))
        leaf = extra
    F = mesh.faces_packed().shape[0]
    # frame i's faces are the i-th copy in the packed mesh
    fr = Fragments(p2f.where(p2f < 0, p2f + F * torch.arange(N, device=device).view(N, 1, 1, 1)), fr.zbuf, b,
                   fr.dists)
    fr.pix_to_face._pr_valid_counts = (fr.pix_to_face._version, p2f._pr_valid_counts[1])
    G = torch.randn((N,) + tuple(frag.pix_to_face.shape[1:]) + (3,), device=device,
                    generator=torch.Generator(device).manual_seed(2))
    runs = []
    for pix in ("1", "0"):
        monkeypatch.setenv("PR_SHADE_PIX", pix)
        out = sh.textured_phong_shading(m, fr, lights, cams, mats)
        runs.append((out,) + tuple(torch.autograd.grad((out * G).sum(), [b, verts, leaf])))
    (o1, gb1, gv1, gt1), (o0, gb0, gv0, gt0) = runs
    assert torch.equal(o1, o0)
    assert torch.equal(gb1, gb0)
    for x, y in ((gv1, gv0), (gt1, gt0)):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6 * float(y.abs().max()))


def test_forward_zeroed_accumulators_once(device):
    """The C++ layer's shading forward zeroes the backward's small accumulators (d verts, d normals,
    d vertex colours, d light; pr_shade_fwd + PR_GRAD_PREZEROED, no memsets in the backward): a
    second backward of the same graph (retain_graph) zeroes its own and gives the same gradients,
    and both agree with the Python layer's (zeroed by the backward call)."""
    from pertrenderer_amd import host_layer
    assert host_layer.get() is not None, host_layer.error()
    mesh, frag, lights, cams, mats, verts, loc, extra = _scene(device, "vertex")
    out = sh.textured_phong_shading(mesh, frag, lights, cams, mats)
    G = torch.randn(out.shape, device=device, generator=torch.Generator(device).manual_seed(4))
    leaves = [verts, loc, extra]
    g1 = torch.autograd.grad((out * G).sum(), leaves, retain_graph=True)
    g2 = torch.autograd.grad((out * G).sum(), leaves)
    with host_layer.disabled():
        mesh2, frag2, lights2, cams2, mats2, verts2, loc2, extra2 = _scene(device, "vertex")
        out2 = sh.textured_phong_shading(mesh2, frag2, lights2, cams2, mats2)
        g3 = torch.autograd.grad((out2 * G).sum(), [verts2, loc2, extra2])
    assert torch.equal(out, out2)
    for a, b, c in zip(g1, g2, g3):
        assert float(a.abs().sum()) > 0
        tol = dict(rtol=1e-5, atol=1e-6 * float(c.abs().max()))  # float atomics: order differs
        torch.testing.assert_close(a, b, **tol)
        torch.testing.assert_close(a, c, **tol)


@pytest.mark.parametrize("shader_kind,kind,pair,K", [
    ("phong", "uv", "gaussian", 12), ("phong", "vertex", "gaussian", 12), ("simple", "vertex", "gaussian", 12),
    # eval.py's "softras" renderer (SoftRast + SoftAgg): K <= 64 runs the 16-lane kernels, K > 64 the
    # one-thread-per-pixel ones, both on fragments whose padding was never written
    ("phong", "uv", "soft", 12), ("phong", "uv", "soft", 80), ("phong", "vertex", "soft", 80)])
def test_renderer_valid_only_fragments_match_full(shader_kind, kind, pair, K, device):
    """MeshRenderer hands a shader that reads each pixel's valid prefix only (takes_valid_only) fragments
    whose padding is left unwritten (PR_RAST_VALID_ONLY): the image is the full-fragment render's bit for
    bit, the gradients agree to float-atomic order.  (Renders compared after a first one: with
    fixed_noise=True the reference reseeds after the rast draw (smoothagg.py:18-19 after smoothrast.py:21),
    so call 1's rast noise comes from the caller's generator and every later call repeats call 2 --
    the reference's semantics, pinned by tests/test_noise_pair.py.)"""
    import pertrenderer_amd as pa
    from pertrenderer_amd.renderer.renderer import MeshRenderer
    mesh, _, _, cams, mats, verts, _, extra = _scene(device, kind)
    lights = PointLights(device=device, location=[[0.5, 2.0, -2.0]])
    rs = RasterizationSettings(image_size=48, blur_radius=math.log(1e4 - 1) * 1e-3, faces_per_pixel=K)
    rast = MeshRasterizer(cameras=cams, raster_settings=rs)
    if pair == "soft":
        sr, sa = pa.SoftRast(sigma=1e-3), pa.SoftAgg(gamma=1e-2)
    else:
        sr, sa = pa.GaussianRast(sigma=1e-3), pa.GaussianAgg(nb_samples=4, gamma=1e-2, fixed_noise=True)
    cls = pa.RandomPhongShader if shader_kind == "phong" else pa.RandomSimpleShader
    shader = cls(device=device, cameras=cams, lights=lights, materials=mats, smoothrast=sr, smoothagg=sa)
    assert shader.takes_valid_only(mesh)
    G = torch.rand((1, 48, 48, 4), device=device)
    renderer = MeshRenderer(rast, shader)
    with torch.no_grad():
        renderer(mesh)
    img_v = renderer(mesh)
    g_v = _grads(img_v, G, [verts, extra])
    shader.takes_valid_only = lambda *a, **k: False  # the same render with PyTorch3D's full fragments
    img_f = renderer(mesh)
    g_f = _grads(img_f, G, [verts, extra])
    assert torch.equal(img_v, img_f)
    for a, b, name in zip(g_v, g_f, ("verts", "texture")):
        _close(a, b, 1e-5, name)
