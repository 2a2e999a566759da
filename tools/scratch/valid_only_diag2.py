"""Scratch: MeshRenderer renders with and without valid-only fragments."""
import sys, os, math, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import test_gpu_shading as T
import pertrenderer_amd as pa
from pertrenderer_amd.renderer import PointLights, MeshRasterizer, RasterizationSettings
from pertrenderer_amd.renderer.renderer import MeshRenderer
dev = torch.device("cuda:0")
kind = sys.argv[1] if len(sys.argv) > 1 else "vertex"
mesh, _, _, cams, mats, verts, _, extra = T._scene(dev, kind)
lights = PointLights(device=dev, location=[[0.5, 2.0, -2.0]])
rs = RasterizationSettings(image_size=48, blur_radius=math.log(1e4 - 1) * 1e-3, faces_per_pixel=12)
rast = MeshRasterizer(cameras=cams, raster_settings=rs)
sr, sa = pa.GaussianRast(sigma=1e-3), pa.GaussianAgg(nb_samples=4, gamma=1e-2, fixed_noise=True)
shader = (pa.RandomPhongShader if kind == "uv" else pa.RandomSimpleShader)(device=dev, cameras=cams, lights=lights, materials=mats, smoothrast=sr, smoothagg=sa)
r = MeshRenderer(rast, shader)
with torch.no_grad():
    r(mesh)  # first call (lazy state: differs from later calls with or without valid-only)
    v1 = r(mesh); v2 = r(mesh)
    shader.takes_valid_only = lambda *a, **k: False
    f1 = r(mesh); f2 = r(mesh)
d = lambda a, b: float((a - b).abs().max())
print("vo-vo", d(v1, v2), "full-full", d(f1, f2), "vo-full", d(v1, f1), "pixels differing", int(((v1 - f1).abs() > 1e-6).any(-1).sum()))
frag = rast(mesh)
print("valid slots", int((frag.pix_to_face >= 0).sum()), flush=True)
