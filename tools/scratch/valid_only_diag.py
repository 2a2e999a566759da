"""Scratch: valid-only vs full fragments render diagnostics."""
import sys, os, math, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import test_gpu_shading as T
import pertrenderer_amd as pa
from pertrenderer_amd.renderer import PointLights, MeshRasterizer, RasterizationSettings
from pertrenderer_amd.renderer.renderer import MeshRenderer
dev = torch.device("cuda:0")
for shader_kind, kind in (("phong", "uv"), ("simple", "vertex")):
    mesh, _, _, cams, mats, verts, _, extra = T._scene(dev, kind)
    lights = PointLights(device=dev, location=[[0.5, 2.0, -2.0]])
    rs = RasterizationSettings(image_size=48, blur_radius=math.log(1e4 - 1) * 1e-3, faces_per_pixel=12)
    rast = MeshRasterizer(cameras=cams, raster_settings=rs)
    sr, sa = pa.GaussianRast(sigma=1e-3), pa.GaussianAgg(nb_samples=4, gamma=1e-2, fixed_noise=True)
    cls = pa.RandomPhongShader if shader_kind == "phong" else pa.RandomSimpleShader
    shader = cls(device=dev, cameras=cams, lights=lights, materials=mats, smoothrast=sr, smoothagg=sa)
    f1 = shader(rast(mesh), mesh); f2 = shader(rast(mesh), mesh)
    v1 = MeshRenderer(rast, shader)(mesh); v2 = MeshRenderer(rast, shader)(mesh)
    print(shader_kind, kind, "full-full", float((f1 - f2).abs().max()), "vo-vo", float((v1 - v2).abs().max()),
          "vo-full", float((v1 - f1).abs().max()), flush=True)
