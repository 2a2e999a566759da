"""RandomPhongShader with its shading fused into the blend's forward (PR_BLEND_PHONG; backward:
PR_BLEND_COLOR_SPARSE then pr_shade_bwd) against the unfused composition it replaces
(random_rasterizer.py:99-116: sample_textures -> phong_shading -> smooth_rgb_blend, here pr_shade_fwd/bwd
-> the texel blend pr_blend_* with colour mode 1).

Same Monte-Carlo draws (injected reference noise, or the same Philox keys): the image, d dists,
d zbuf and d bary are bit-identical (every slot colour and d colour is computed with the same
operations, pr_phong.h); the float-atomic sums -- vertex positions (through the shading and the
vertex normals), the UV map or vertex colours, the light and the camera -- agree to fp32 summation
order (conftest.assert_close, 1e-5 relative); the smoothing scalars too."""
import math

import pytest
import torch

import pertrenderer_amd as pa
import pertrenderer_amd.random_rasterizer as rr
from conftest import assert_close
from pertrenderer_amd import host_layer, noise
from pertrenderer_amd.renderer import (FoVPerspectiveCameras, MeshRasterizer, PointLights, RasterizationSettings,
                                       look_at_view_transform)
from pertrenderer_amd.renderer.renderer import DirectionalLights, MeshRenderer
from test_gpu_shading import _scene

pytestmark = pytest.mark.gpu


def _render(kind, light_kind, fused, source, device, K=12, size=48, via_renderer=False, seed=11):
    mesh, _, _, _, mats, verts, _, extra = _scene(device, kind)
    R, T = look_at_view_transform(2.2 if kind != "uv" else 3.0, 25.0, 40.0, device=device)
    T = T.clone().requires_grad_(True)  # camera centre gradient through the shading
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    loc = torch.tensor([[0.5, 2.0, -2.0]] if light_kind == "point" else [[0.3, 1.0, 0.4]], device=device,
                       requires_grad=True)
    lights = (PointLights(device=device, location=loc) if light_kind == "point"
              else DirectionalLights(device=device, direction=loc))
    lights.location = loc
    rs = RasterizationSettings(image_size=size, blur_radius=math.log(1e4 - 1) * 1e-3, faces_per_pixel=K)
    rast = MeshRasterizer(cameras=cams, raster_settings=rs)
    sr = pa.GaussianRast(nb_samples=8, sigma=1e-3)
    sa = pa.GaussianAgg(nb_samples=8, gamma=1e-2)
    shader = pa.RandomPhongShader(device=device, cameras=cams, lights=lights, materials=mats, smoothrast=sr,
                                  smoothagg=sa, blend_params=pa.random_rasterizer.BlendParams(1e-4, 1e-4, (0.2, 0.3, 0.4)))
    G = torch.rand((1, size, size, 4), device=device, generator=torch.Generator(device).manual_seed(5))
    old, old_src = rr.FUSE_PHONG, noise.get_noise_source()
    rr.FUSE_PHONG = fused
    noise.set_noise_source(source)
    try:
        torch.manual_seed(seed)
        if via_renderer:
            img = MeshRenderer(rast, shader)(mesh)
            frag_leaves = []
        else:
            frag = rast(mesh)
            torch.manual_seed(seed)
            img = shader(frag, mesh)
            frag_leaves = [frag.dists, frag.zbuf, frag.bary_coords]
        leaves = frag_leaves + [verts, extra, loc, T, sr.sigma, sa.gamma, sa.alpha]
        gs = torch.autograd.grad((img * G).sum(), leaves, allow_unused=True)
    finally:
        rr.FUSE_PHONG = old
        noise.set_noise_source(old_src)
    gs = [torch.zeros_like(l) if g is None else g for g, l in zip(gs, leaves)]
    return img.detach(), gs, len(frag_leaves)


@pytest.mark.parametrize("kind,light_kind", [("uv", "point"), ("vertex", "point"), ("vertex", "directional")])
@pytest.mark.parametrize("source", ["torch", "philox"])
def test_fused_phong_matches_shade_then_blend(kind, light_kind, source, device):
    img_f, g_f, nf = _render(kind, light_kind, True, source, device)
    img_u, g_u, _ = _render(kind, light_kind, False, source, device)
    assert float((img_f[..., 3] > 0).float().mean()) > 0.05  # the mesh covers the frame
    assert torch.equal(img_f, img_u)
    names = ["d dists", "d zbuf", "d bary"][:nf] + ["verts", "texture", "light", "camera T", "sigma", "gamma",
                                                   "alpha"]
    for name, a, b in zip(names, g_f, g_u):
        if name.startswith("d "):
            assert torch.equal(a, b), name  # per-slot, same operations
        else:
            assert float(b.abs().max()) > 0, name
            assert_close(a, b, rtol=1e-5, atol_rel=1e-6, name=name)


def test_fused_phong_through_mesh_renderer_valid_only(device):
    """MeshRenderer's handshake (valid-prefix fragments, live-only backward) with the fused shading:
    the image equals the unfused renderer's bit for bit, the pose-side gradients at 1e-5."""
    img_f, g_f, _ = _render("uv", "point", True, "philox", device, via_renderer=True)
    img_u, g_u, _ = _render("uv", "point", False, "philox", device, via_renderer=True)
    assert torch.equal(img_f, img_u)
    for name, a, b in zip(("verts", "texture", "light", "camera T"), g_f, g_u):
        assert_close(a, b, rtol=1e-5, atol_rel=1e-6, name=name)


def test_fused_phong_host_layers_agree(device):
    """The C++ autograd node (host_layer) and the Python Function launch the same kernels."""
    assert host_layer.get() is not None, host_layer.error()
    img_c, g_c, nf = _render("uv", "point", True, "philox", device)
    with host_layer.disabled():
        img_p, g_p, _ = _render("uv", "point", True, "philox", device)
    assert torch.equal(img_c, img_p)
    for i, (a, b) in enumerate(zip(g_c, g_p)):
        if i < nf:
            assert torch.equal(a, b)
        else:
            assert_close(a, b, rtol=1e-5, atol_rel=1e-6, name=str(i))


def test_fused_phong_runs_no_shading_pass(device, tmp_path):
    """The fused forward shades inside the blend kernel: no shading pass over every slot
    (shade_fwd_*) runs; the backward is the blend kernel then the shading backward."""
    import json
    from torch.profiler import ProfilerActivity, profile
    _render("uv", "point", True, "philox", device)  # warm
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        _render("uv", "point", True, "philox", device)
        torch.cuda.synchronize()
    tr = str(tmp_path / "trace.json")
    prof.export_chrome_trace(tr)
    names = [e.get("name", "") for e in json.load(open(tr))["traceEvents"]
             if e.get("ph") == "X" and e.get("cat") == "kernel"]
    assert any("blend_fwd_kernel" in n for n in names) and any("blend_bwd_kernel" in n for n in names), names
    assert not any("shade_fwd" in n for n in names), [n for n in names if "shade_" in n]
    assert any("shade_bwd" in n for n in names), names


def _render_batch(fused, device, size=40, K=10, seed=23):
    """Two vertex-coloured meshes (sphere, shifted / scaled sphere) in one batch, each with its own
    camera pose and point light: the shade arguments are indexed per image."""
    import os
    from conftest import ROOT
    from pertrenderer_amd.renderer import Materials, Meshes, TexturesVertex, load_obj
    torch.manual_seed(4)
    v, f, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    v, f = v.to(device), f.verts_idx.to(device)
    v = v - v.mean(0)
    verts = [v.clone().requires_grad_(True), (0.7 * v + 0.1).requires_grad_(True)]
    cols = [torch.rand((v.shape[0], 3), device=device).requires_grad_(True) for _ in range(2)]
    mesh = Meshes(verts, [f, f], TexturesVertex(cols))
    R, T = look_at_view_transform(2.4, torch.tensor([25.0, -10.0]), torch.tensor([40.0, 160.0]), device=device)
    T = T.clone().requires_grad_(True)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    loc = torch.tensor([[0.5, 2.0, -2.0], [-1.0, 0.5, 2.5]], device=device, requires_grad=True)
    lights = PointLights(device=device, location=loc)
    lights.location = loc
    rs = RasterizationSettings(image_size=size, blur_radius=math.log(1e4 - 1) * 1e-3, faces_per_pixel=K)
    rast = MeshRasterizer(cameras=cams, raster_settings=rs)
    sr = pa.GaussianRast(nb_samples=8, sigma=1e-3)
    sa = pa.GaussianAgg(nb_samples=8, gamma=1e-2)
    shader = pa.RandomPhongShader(device=device, cameras=cams, lights=lights, materials=Materials(device=device),
                                  smoothrast=sr, smoothagg=sa,
                                  blend_params=pa.random_rasterizer.BlendParams(1e-4, 1e-4, (0.2, 0.3, 0.4)))
    G = torch.rand((2, size, size, 4), device=device, generator=torch.Generator(device).manual_seed(6))
    old, old_src = rr.FUSE_PHONG, noise.get_noise_source()
    rr.FUSE_PHONG = fused
    noise.set_noise_source("philox")
    try:
        torch.manual_seed(seed)
        img = MeshRenderer(rast, shader)(mesh)
        leaves = verts + cols + [loc, T, sr.sigma, sa.gamma, sa.alpha]
        gs = torch.autograd.grad((img * G).sum(), leaves, allow_unused=True)
    finally:
        rr.FUSE_PHONG = old
        noise.set_noise_source(old_src)
    return img.detach(), [torch.zeros_like(l) if g is None else g for g, l in zip(gs, leaves)]


def test_fused_phong_batch_per_image_camera_and_light(device):
    """N = 2 with per-image poses and lights: the fused forward shades each slot with its own
    image's camera and light; image bitwise, every gradient at 1e-5 against the unfused path."""
    img_f, g_f = _render_batch(True, device)
    img_u, g_u = _render_batch(False, device)
    for n in range(2):  # both meshes are on screen
        assert float((img_f[n, ..., 3] > 0).float().mean()) > 0.05, n
    assert torch.equal(img_f, img_u)
    names = ["verts 0", "verts 1", "colours 0", "colours 1", "light", "camera T", "sigma", "gamma", "alpha"]
    for name, a, b in zip(names, g_f, g_u):
        assert float(b.abs().max()) > 0, name
        assert_close(a, b, rtol=1e-5, atol_rel=1e-6, name=name)
    # per-image rows of the light / camera gradients are distinct (not one image's sum broadcast)
    assert not torch.equal(g_f[4][0], g_f[4][1]) and not torch.equal(g_f[5][0], g_f[5][1])


def test_fused_phong_deterministic_mode_is_bitwise(device):
    """torch.use_deterministic_algorithms(True): the shading backward sums in slot order on both
    paths, which see bit-identical d colours, so every gradient is bit-identical too -- and the
    fused path is run-to-run reproducible."""
    old = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True)
    try:
        img_f, g_f, _ = _render("uv", "point", True, "philox", device, via_renderer=True)
        img_f2, g_f2, _ = _render("uv", "point", True, "philox", device, via_renderer=True)
        img_u, g_u, _ = _render("uv", "point", False, "philox", device, via_renderer=True)
    finally:
        torch.use_deterministic_algorithms(old)
    assert torch.equal(img_f, img_u) and torch.equal(img_f, img_f2)
    for name, a, a2, b in zip(("verts", "texture", "light", "camera T", "sigma", "gamma", "alpha"), g_f, g_f2, g_u):
        assert torch.equal(a, a2), name
        assert torch.equal(a, b), name
