"""One pixel of tests/test_gpu_pipeline_ref.py's frame, stage by stage: GPU (native) vs the CPU
oracle composition -- fragments, texels, Phong colours, vertex normals, image.  Diagnostic only."""
import math
import sys

import torch

sys.path.insert(0, ".")
import pertrenderer_amd as pa  # noqa: E402
from oracle import pipeline_ref as pr  # noqa: E402
from pertrenderer_amd import pose_opt  # noqa: E402
from pertrenderer_amd.renderer import Rotate, so3_exponential_map  # noqa: E402
from pertrenderer_amd.renderer.shading import textured_phong_shading  # noqa: E402

H, K, SIGMA = 64, 50, 1e-3
py, px = int(sys.argv[1]) if len(sys.argv) > 1 else 30, int(sys.argv[2]) if len(sys.argv) > 2 else 36
dev = torch.device("cuda:0")
pa.set_noise_source("torch")
torch.manual_seed(0)
gpu = pose_opt.Scene(dev, H)
cpu = pose_opt.Scene(torch.device("cpu"), H)
target, R_true = gpu.target()
_, (renderer,) = pose_opt.init_renderers(gpu, R_true, sigma=SIGMA, gamma=1e-2, nb_samples=8, noise_type=("gaussian",))
log_rot0 = pose_opt.so3_log_map(R_true @ so3_exponential_map(torch.tensor([[0.2, -0.15, 0.1]], device=dev)))
with torch.no_grad():
    R = so3_exponential_map(log_rot0)
    mg = gpu.meshes.update_padded(Rotate(R).transform_points(gpu.meshes.verts_padded()))
    Rc = so3_exponential_map(log_rot0.cpu())
    mc = cpu.meshes.update_padded(Rotate(Rc).transform_points(cpu.meshes.verts_padded()))
    print("verts equal", torch.equal(mg.verts_packed().cpu(), mc.verts_packed()))
    ng, nc = mg.verts_normals_packed().cpu(), mc.verts_normals_packed()
    print("normals equal", torch.equal(ng, nc), "max diff", (ng - nc).abs().max().item())
    frag = renderer.rasterizer(mg, cameras=gpu.cameras[0])
    cam = cpu.cameras[0]
    view = cam.get_world_to_view_transform().transform_points(mc.verts_packed()[None])
    ndc = cam.get_projection_transform().transform_points(view)
    screen = torch.cat([ndc[..., :2], view[..., 2:3]], -1)[0]
    blur = math.log(1.0 / 1e-4 - 1.0) * SIGMA
    p2f, zbuf, bary, dists = pr.RastRef.apply(screen[mc.faces_packed()], H, H, K, blur, blur > 0.0)
    sl = (0, py, px)
    for name, a, b in (("p2f", frag.pix_to_face, p2f), ("zbuf", frag.zbuf, zbuf), ("bary", frag.bary_coords, bary),
                       ("dists", frag.dists, dists)):
        a = a[sl].cpu()
        print(name, "equal", torch.equal(a, b[sl]), "max diff", (a.float() - b[sl].float()).abs().max().item())
    colors_g = textured_phong_shading(mg, frag, gpu.lights, gpu.cameras[0], renderer.shader.materials).cpu()
    tex = cpu.meshes.textures
    texels = pr.sample_uv(p2f, bary, tex.faces_uvs_list()[0], tex.verts_uvs_list()[0], tex.maps_padded())
    colors_c = pr.phong(p2f, bary, mc.verts_packed(), mc.faces_packed(), nc, texels, cpu.lights.location[0],
                        cam.get_camera_center()[0])
    cnt = int((p2f[sl] >= 0).sum())
    d = (colors_g[sl][:cnt] - colors_c[sl][:cnt]).abs()
    print("valid slots", cnt, "colors max diff", d.max().item(), "per slot", d.max(-1).values.tolist())
    colors_n = pr.phong(p2f, bary, mc.verts_packed(), mc.faces_packed(), ng, texels, cpu.lights.location[0],
                        cam.get_camera_center()[0])
    print("oracle colours with GPU normals: max diff vs GPU", (colors_g[sl][:cnt] - colors_n[sl][:cnt]).abs().max().item())
    k = int(d.max(-1).values.argmax())
    print("worst slot", k, "gpu", colors_g[sl][k].tolist(), "cpu", colors_c[sl][k].tolist(), "face", int(p2f[sl][k]))
