"""eval.py's check_differentiability flows (eval.py:693-725 -> optimize_scene_params :411-470):
gradients of a rendered loss w.r.t. the light location, the camera (elev / azim through
look_at_view_transform: the MeshRasterizer path with camera gradients), TexturesUV maps and
TexturesVertex colours, on the GPU, against central differences.

Noise is the reference's own draw (``set_noise_source("torch")``), reseeded before every render,
so the perturbed renderer is a fixed function of its inputs.  Its Monte-Carlo weights are
piecewise constant in the geometry, so the geometry gradient (camera) is checked on the
deterministic SoftRast + SoftAgg renderer (eval.py's "softras", made smooth enough for finite
differences: see the camera test); the colour-side gradients (light,
textures) on the perturbed GaussianRast + GaussianAgg renderer, where the weights do not depend on
the colours and the image is smooth in those parameters (linear in the texels)."""
import math
import os

import pytest
import torch

import pertrenderer_amd as pa
from conftest import ROOT
from pertrenderer_amd import random_rasterizer as rr
from pertrenderer_amd.renderer import (BlendParams, Meshes, MeshRasterizer, MeshRenderer, OpenGLPerspectiveCameras,
                                       PointLights, RasterizationSettings, TexturesUV, TexturesVertex, load_obj,
                                       look_at_view_transform)

pytestmark = pytest.mark.gpu
IMSIZE = 48


@pytest.fixture
def torch_noise():
    old = pa.noise.get_noise_source()
    pa.set_noise_source("torch")
    yield
    pa.set_noise_source(old)


def _sphere(device, colors):
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    v = verts - verts.mean(0)
    v = v / (2 * v.abs().max())
    return Meshes(verts=[v.to(device)], faces=[faces.verts_idx.to(device)], textures=TexturesVertex(colors[None]))


def _renderer(device, kind, sigma, gamma, nb=8):
    rast, agg = {"gaussian": (pa.GaussianRast(sigma=sigma), pa.GaussianAgg(gamma=gamma, nb_samples=nb)),
                 "softras": (pa.SoftRast(sigma=sigma), pa.SoftAgg(gamma=gamma))}[kind]
    settings = RasterizationSettings(image_size=IMSIZE, blur_radius=math.log(1e4 - 1) * sigma, faces_per_pixel=50,
                                     max_faces_per_bin=50000, perspective_correct=False)
    R, T = look_at_view_transform(dist=2.7, elev=30.0, azim=120.0, device=device)
    cam = OpenGLPerspectiveCameras(device=device, R=R, T=T)
    lights = PointLights(device=device, location=[[0.0, 2.0, -2.0]])
    shader = rr.RandomPhongShader(device=device, cameras=cam, lights=lights, smoothrast=rast, smoothagg=agg,
                                  blend_params=BlendParams(sigma, gamma, (0.0, 0.0, 0.0)))
    return MeshRenderer(MeshRasterizer(cameras=cam, raster_settings=settings), shader), cam, lights


def _loss(renderer, mesh, G, seed=5, **kw):
    torch.manual_seed(seed)  # the same reference draws at every evaluation
    img = renderer(mesh, **kw)
    return (img[..., :3].double() * G).sum()


def _central(f, x, d, h):
    """Central difference with one Richardson step: (4 D(h/2) - D(h)) / 3, O(h^4)."""
    with torch.no_grad():
        D = lambda t: float((f(x + t * d) - f(x - t * d)) / (2 * t))
        return (4.0 * D(0.5 * h) - D(h)) / 3.0


def _check(ad, fd, rtol):
    assert math.isfinite(ad) and abs(ad - fd) <= rtol * max(abs(fd), 1e-6), (ad, fd)


def _grid(device, n=3):
    """A flat n x n quad grid facing the camera: no face hides another, and with n = 3 (18
    faces) no pixel has more faces than K = 50 in reach (no K truncation)."""
    t = torch.linspace(-0.4, 0.4, n + 1)
    yy, xx = torch.meshgrid(t, t, indexing="ij")
    verts = torch.stack([xx.flatten(), yy.flatten(), torch.zeros((n + 1) ** 2)], -1)
    i = torch.arange(n)
    a = (i[:, None] * (n + 1) + i[None, :]).flatten()
    faces = torch.cat([torch.stack([a, a + 1, a + n + 2], -1), torch.stack([a, a + n + 2, a + n + 1], -1)])
    g = torch.Generator().manual_seed(4)
    col = torch.rand(((n + 1) ** 2, 3), generator=g)
    return Meshes(verts=[verts.to(device)], faces=[faces.to(device)], textures=TexturesVertex(col[None].to(device)))


def test_light_location_gradient(device, torch_noise):
    """On a flat grid (constant normal: no diffuse terminator crossing the image, the specular
    max(0, .)^64 is smooth at 0), so finite differences converge."""
    mesh = _grid(device)
    renderer, _, _ = _renderer(device, "gaussian", 1e-3, 1e-2)
    R, T = look_at_view_transform(dist=2.0, elev=15.0, azim=10.0, device=device)
    cam = OpenGLPerspectiveCameras(device=device, R=R, T=T)
    G = torch.randn((1, IMSIZE, IMSIZE, 3), generator=torch.Generator().manual_seed(0),
                    dtype=torch.float64).to(device)
    f = lambda loc: _loss(renderer, mesh, G, cameras=cam, lights=PointLights(device=device, location=loc))
    loc = torch.tensor([[0.3, 1.0, 2.0]], device=device, requires_grad=True)
    f(loc).backward()
    for d in ([[1.0, 0.0, 0.0]], [[0.0, 1.0, 0.0]], [[0.6, -0.48, 0.64]]):
        d = torch.tensor(d, device=device)
        _check(float((loc.grad * d).sum()), _central(f, loc.detach(), d, 2e-2), 5e-3)


def test_vertex_colour_gradient(device, torch_noise):
    g = torch.Generator().manual_seed(1)
    base = torch.rand((642, 3), generator=g).to(device)
    renderer, cam, lights = _renderer(device, "gaussian", 1e-3, 1e-2)
    G = torch.randn((1, IMSIZE, IMSIZE, 3), generator=g, dtype=torch.float64).to(device)
    # eval.py:450: TexturesVertex(verts_features=rgb.clamp(0, 1)) on the optimised colours
    f = lambda rgb: _loss(renderer, _sphere(device, rgb.clamp(min=0.0, max=1.0)), G, cameras=cam, lights=lights)
    rgb = (0.1 + 0.8 * base).requires_grad_(True)
    f(rgb).backward()
    d = torch.randn((642, 3), generator=g).to(device)
    _check(float((rgb.grad * d).sum()), _central(f, rgb.detach(), d, 1e-2), 2e-3)


def test_uv_map_gradient(device, torch_noise):
    from pertrenderer_amd import pose_opt
    mesh = pose_opt.load_cube(device)
    v = mesh.verts_packed()
    v = (v - v.mean(0)) / (v - v.mean(0)).abs().max()
    tex = mesh.textures
    g = torch.Generator().manual_seed(2)
    renderer, _, lights = _renderer(device, "gaussian", 1e-3, 1e-2)
    R, T = look_at_view_transform(dist=6.7, elev=30.0, azim=120.0, device=device)
    cam = OpenGLPerspectiveCameras(device=device, R=R, T=T)
    G = torch.randn((1, IMSIZE, IMSIZE, 3), generator=g, dtype=torch.float64).to(device)

    def f(maps):
        m = Meshes(verts=[v], faces=[mesh.faces_packed()],
                   textures=TexturesUV(maps=maps, faces_uvs=tex.faces_uvs_list(), verts_uvs=tex.verts_uvs_list()))
        return _loss(renderer, m, G, cameras=cam, lights=lights)

    maps = tex.maps_padded().detach().clone().requires_grad_(True)
    f(maps).backward()
    assert maps.grad is not None and maps.grad.abs().sum() > 0
    d = torch.randn(maps.shape, generator=g).to(device)
    _check(float((maps.grad * d).sum()), _central(f, maps.detach(), d, 1e-2), 2e-3)


def test_camera_gradient_soft_renderer(device):
    """d loss / d (elev, azim) through look_at_view_transform, the camera-gradient path of
    MeshRasterizer (transform + rasterizer backward) and the soft blend, vs central differences
    in degrees.  The soft renderer drops a face where its P reaches exp(-blur/sigma): with
    eval.py's blur factor ln(1e4 - 1) that is a 1e-4 jump per (pixel, face) crossing, which
    swamps any finite difference; here blur = 25 sigma (jumps ~1e-11) on a flat grid (no face
    behind another, so no K truncation)."""
    mesh = _grid(device)
    sigma, gamma = 3e-3, 1e-2
    settings = RasterizationSettings(image_size=IMSIZE, blur_radius=25.0 * sigma, faces_per_pixel=50,
                                     perspective_correct=False)
    lights = PointLights(device=device, location=[[0.0, 2.0, 2.0]])
    G = torch.randn((1, IMSIZE, IMSIZE, 3), generator=torch.Generator().manual_seed(3),
                    dtype=torch.float64).to(device)

    def f(ea):
        R, T = look_at_view_transform(dist=2.0, elev=ea[0:1], azim=ea[1:2], device=device)
        cam = OpenGLPerspectiveCameras(device=device, R=R, T=T)
        shader = rr.RandomPhongShader(device=device, cameras=cam, lights=lights, smoothrast=pa.SoftRast(sigma=sigma),
                                      smoothagg=pa.SoftAgg(gamma=gamma),
                                      blend_params=BlendParams(sigma, gamma, (0.0, 0.0, 0.0)))
        r = MeshRenderer(MeshRasterizer(cameras=cam, raster_settings=settings), shader)
        return _loss(r, mesh, G, cameras=cam, lights=lights)

    ea = torch.tensor([15.0, 10.0], device=device, requires_grad=True)
    f(ea).backward()
    assert ea.grad is not None and ea.grad.abs().sum() > 0
    # (degrees: a 0.01 step moves the image by ~1e-4 NDC; much larger steps cross the blur
    # cut-off of faces and stop being a derivative)
    for d in (torch.tensor([0.0, 1.0]), torch.tensor([0.6, 0.8])):
        d = d.to(device)
        _check(float((ea.grad * d).sum()), _central(f, ea.detach(), d, 1e-2), 2e-2)
