"""Diagnostic: vertex gradients of the soft renderer through MeshRasterizer's fast path (camera
without grad: native projection) and its transform path (camera with grad), which must agree;
and the camera-angle gradient against central differences."""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pertrenderer_amd as pa  # noqa: E402
from pertrenderer_amd import random_rasterizer as rr  # noqa: E402
from pertrenderer_amd.renderer import (BlendParams, Meshes, MeshRasterizer, MeshRenderer,  # noqa: E402
                                       OpenGLPerspectiveCameras, PointLights, RasterizationSettings,
                                       TexturesVertex, load_obj, look_at_view_transform)

dev = torch.device("cuda:0")
S = 48
MESH = os.environ.get("DIAG_MESH", "sphere")
if MESH == "sphere":
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    v0 = verts - verts.mean(0)
    v0 = (v0 / (2 * v0.abs().max())).to(dev)
    f0 = faces.verts_idx.to(dev)
else:  # flat n x n grid in z = 0
    n = 3
    t = torch.linspace(-0.4, 0.4, n + 1)
    yy, xx = torch.meshgrid(t, t, indexing="ij")
    v0 = torch.stack([xx.flatten(), yy.flatten(), torch.zeros((n + 1) ** 2)], -1).to(dev)
    i = torch.arange(n)
    a = (i[:, None] * (n + 1) + i[None, :]).flatten()
    f0 = torch.cat([torch.stack([a, a + 1, a + n + 2], -1), torch.stack([a, a + n + 2, a + n + 1], -1)]).to(dev)
g = torch.Generator().manual_seed(3)
col = torch.rand((v0.shape[0], 3), generator=g).to(dev)
G = torch.randn((1, S, S, 3), generator=g, dtype=torch.float64).to(dev)
sigma = float(sys.argv[1]) if len(sys.argv) > 1 else 1e-2
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
BF = float(os.environ.get("DIAG_BLUR", math.log(1e4 - 1)))
settings = RasterizationSettings(image_size=S, blur_radius=BF * sigma, faces_per_pixel=K,
                                 perspective_correct=False)
lights = PointLights(device=dev, location=[[0.0, 2.0, 2.0]])
DIST, EL, AZ = (2.0, 15.0, 10.0) if MESH != "sphere" else (2.7, 20.0, 100.0)


def render(v, R, T):
    cam = OpenGLPerspectiveCameras(device=dev, R=R, T=T)
    shader = rr.RandomPhongShader(device=dev, cameras=cam, lights=lights, smoothrast=pa.SoftRast(sigma=sigma),
                                  smoothagg=pa.SoftAgg(gamma=1e-2), blend_params=BlendParams(sigma, 1e-2, (0, 0, 0)))
    r = MeshRenderer(MeshRasterizer(cameras=cam, raster_settings=settings), shader)
    img = r(Meshes(verts=[v], faces=[f0], textures=TexturesVertex(col[None])), cameras=cam, lights=lights)
    return (img[..., :3].double() * G).sum()


R, T = look_at_view_transform(dist=DIST, elev=EL, azim=AZ, device=dev)
v = v0.clone().requires_grad_(True)
render(v, R, T).backward()
ga = v.grad.clone()
v = v0.clone().requires_grad_(True)
Rg = R.clone().requires_grad_(True)
render(v, Rg, T).backward()
gb = v.grad.clone()
print("verts grad fast vs transform path: max|a| %.4e max|a-b| %.4e" % (ga.abs().max(), (ga - gb).abs().max()))
d = torch.randn(v0.shape, generator=g).to(dev)
with torch.no_grad():
    for h in (1e-2, 3e-3, 1e-3, 3e-4, 1e-4):
        fd = float((render(v0 + h * d, R, T) - render(v0 - h * d, R, T)) / (2 * h))
        print("verts FD h=%g: %.5f  autograd fast %.5f transform %.5f" % (h, fd, float((ga * d).sum()),
                                                                          float((gb * d).sum())))
ea = torch.tensor([EL, AZ], device=dev, requires_grad=True)
R2, T2 = look_at_view_transform(dist=DIST, elev=ea[0:1], azim=ea[1:2], device=dev)
render(v0, R2, T2).backward()
print("d/d(elev, azim) autograd", ea.grad.tolist())
with torch.no_grad():
    for h in (0.3, 0.1, 1e-2, 3e-3, 1e-3):
        out = []
        for e in (torch.tensor([1.0, 0.0], device=dev), torch.tensor([0.0, 1.0], device=dev)):
            p, m = ea.detach() + h * e, ea.detach() - h * e
            Rp, Tp = look_at_view_transform(dist=DIST, elev=p[0:1], azim=p[1:2], device=dev)
            Rm, Tm = look_at_view_transform(dist=DIST, elev=m[0:1], azim=m[1:2], device=dev)
            out.append(float((render(v0, Rp, Tp) - render(v0, Rm, Tm)) / (2 * h)))
        print("FD h=%g:" % h, out)
