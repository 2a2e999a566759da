"""Diagnostic: where does the native Phong kernel's d bary / d verts part from the fp32 torch
composition (tests/test_gpu_shading.py::_reference64 in float32)?"""
import sys
sys.path.insert(0, "tests")
import torch
import test_gpu_shading as T
from pertrenderer_amd.renderer import shading as sh

dev = torch.device("cuda:0")
torch.use_deterministic_algorithms(True)
mesh, frag, lights, cams, mats, verts, loc, extra = T._scene(dev, "vertex")
from pertrenderer_amd.renderer.rasterizer import Fragments
b = frag.bary_coords.detach().clone().requires_grad_(True)
fr = Fragments(frag.pix_to_face, frag.zbuf.detach(), b, frag.dists.detach())
vd = verts.detach().clone().requires_grad_(True)
from pertrenderer_amd.renderer import Meshes, TexturesVertex
m2 = Meshes([vd], [mesh.faces_packed()], TexturesVertex([extra.detach()]))
out = sh.textured_phong_shading(m2, fr, lights, cams, mats)
ref = T._reference64(m2, fr, lights, cams, mats, T._interp64(fr.pix_to_face, b, extra.detach(), m2.faces_packed()),
                     dtype=torch.float32)
G = torch.randn(out.shape, device=dev, generator=torch.Generator(dev).manual_seed(5)) * (frag.pix_to_face >= 0)[..., None]
ga = torch.autograd.grad((out * G).sum(), [b, vd], retain_graph=True)
gr = torch.autograd.grad((ref * G).sum(), [b, vd])
for name, x, y in zip(("bary", "verts(shading only)"), ga, gr):
    d = (x - y).abs()
    sc = y.abs().max()
    rel = d / (1e-5 * y.abs() + 1e-6 * sc)
    print(name, "max|e|", float(sc), "worst/tol", float(rel.max()), "n bad", int((rel > 1).sum()))
    if name == "bary":
        idx = torch.nonzero(rel.reshape(-1, 3).max(-1).values > 1).reshape(-1)[:10]
        print("bad slots", idx.tolist())
        print("out", out.reshape(-1, 3)[idx].tolist())
        print("ga", x.reshape(-1, 3)[idx].tolist())
        print("gr", y.reshape(-1, 3)[idx].tolist())
print("colour diff max", float((out - ref).abs().max()))
