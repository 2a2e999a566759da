"""Diagnostic: native TexturesUV Phong d bary vs the fp32 torch composition at the slots where they
part (tests/test_gpu_shading.py::test_native_shading_matches_float32_composition[uv])."""
import sys
sys.path.insert(0, "tests")
import torch
import test_gpu_shading as T
from pertrenderer_amd.renderer import Meshes, shading as sh
from pertrenderer_amd.renderer.rasterizer import Fragments

dev = torch.device("cuda:0")
torch.use_deterministic_algorithms(True, warn_only=True)
mesh, frag, lights, cams, mats, verts, loc, extra = T._scene(dev, "uv")
b = frag.bary_coords.detach().clone().requires_grad_(True)
fr = Fragments(frag.pix_to_face, frag.zbuf.detach(), b, frag.dists.detach())
m = Meshes([verts.detach()], [mesh.faces_packed()], mesh.textures)
out = sh.textured_phong_shading(m, fr, lights, cams, mats)
ref_tex = T._uv_sample64(fr.pix_to_face, b, m.textures, torch.float32)
ref = T._reference64(m, fr, lights, cams, mats, ref_tex, dtype=torch.float32)
G = torch.randn(out.shape, device=dev, generator=torch.Generator(dev).manual_seed(5)) * (frag.pix_to_face >= 0)[..., None]
(ga,) = torch.autograd.grad((out * G).sum(), [b], retain_graph=True)
(gr,) = torch.autograd.grad((ref * G).sum(), [b], retain_graph=True)
(gt,) = torch.autograd.grad((ref_tex * G).sum(), [b])
rel = (ga - gr).abs() / (1e-5 * gr.abs() + 1e-6 * gr.abs().max())
bad = torch.nonzero(rel.amax(-1) > 1)[:8]
tex = m.textures
uv = T._interp64(fr.pix_to_face, b.detach(), tex.verts_uvs_list()[0], tex.faces_uvs_list()[0])
for idx in bad.tolist():
    n, y, x, k = idx
    print(idx, "p2f", int(fr.pix_to_face[n, y, x, k]), "uv", uv[n, y, x, k].tolist(), "bary", b[n, y, x, k].tolist())
    print("   native", ga[n, y, x, k].tolist(), "ref", gr[n, y, x, k].tolist(), "ref tex-part", gt[n, y, x, k].tolist())
    print("   out", out[n, y, x, k].tolist(), "ref", ref[n, y, x, k].tolist())
print("maps", tex.maps_padded().shape)
