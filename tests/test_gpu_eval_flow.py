"""experiments/eval.py's cube pose-optimisation flow written against the reference's own
import surface (pytorch3d.* through the shim, randomras.* through the alias): textured
cube (eval.py:727-757), HardPhongShader target render (eval.py:762-785), then a few
optimisation steps of the rotation through RandomPhongShader(GaussianRast, GaussianAgg)
(eval.py:343-370).  Checks: textured target renders, the smoothed loss drops, and
texture sampling agrees with a numpy bilinear restatement."""
import math
import os

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _load_cube(device):
    from pytorch3d.io import load_obj
    from pytorch3d.renderer import Textures
    from pytorch3d.structures import Meshes
    d = os.path.join(ROOT, "tests", "golden")
    with np.load(os.path.join(d, "cube_p.npz")) as f:
        pos_idx, pos, col_idx, col = f.values()
    vtx_col = torch.from_numpy(col.astype(np.float32))
    green = vtx_col[3, :].clone()
    vtx_col[3, :] = vtx_col[0, :]
    vtx_col[0, :] = green
    verts, faces, aux = load_obj(os.path.join(d, "cube2.obj"))
    img = aux.texture_images["cube"]
    l = img.size()[1] // 6
    for i in range(6):
        img[:, i * l:(i + 1) * l, :] = vtx_col[i, :][None, None].repeat(img.size()[0], l, 1)
    tex = Textures(verts_uvs=aux.verts_uvs[None], faces_uvs=faces.textures_idx[None], maps=img[None])
    mesh = Meshes(verts=[verts], faces=[faces.verts_idx], textures=tex).to(device)
    return mesh, vtx_col


def test_cube_pose_optimisation_through_reference_imports(device):
    from pytorch3d.renderer import (BlendParams, HardPhongShader, MeshRasterizer, MeshRenderer,
                                    OpenGLPerspectiveCameras, PointLights, RasterizationSettings,
                                    look_at_view_transform)
    from pytorch3d.transforms import Rotate, so3_exponential_map, so3_log_map, so3_relative_angle
    from randomras.random_rasterizer import RandomPhongShader
    from randomras.smoothagg import GaussianAgg
    from randomras.smoothrast import GaussianRast

    torch.manual_seed(0)
    mesh, vtx_col = _load_cube(device)
    verts = mesh.verts_packed()
    center = verts.mean(0)
    scale = max((verts - center).abs().max(0)[0])
    mesh.offset_verts_(-center.expand(verts.shape[0], 3))
    mesh.scale_verts_(1.0 / float(scale))
    R, T = look_at_view_transform(dist=6.7, elev=torch.tensor([30.0]), azim=torch.tensor([120.0]))
    cam = OpenGLPerspectiveCameras(device=device, R=R.to(device), T=T.to(device), fov=60)
    lights = PointLights(device=device, location=[[0.0, 2.0, -2.0]])
    imsize = 64
    hard = MeshRenderer(MeshRasterizer(cameras=cam, raster_settings=RasterizationSettings(
        image_size=imsize, blur_radius=0.0, faces_per_pixel=1, max_faces_per_bin=100000)),
        HardPhongShader(device=device, blend_params=BlendParams(background_color=(0.0, 0.0, 0.0))))
    R_true = so3_exponential_map(torch.tensor([[0.3, -0.5, 0.2]], device=device))
    meshes = mesh.extend(1)
    target = hard(meshes.update_padded(Rotate(R_true).transform_points(meshes.verts_padded())),
                  cameras=cam, lights=lights)[..., :3].detach()
    covered = target.sum(-1) > 0
    assert covered.float().mean() > 0.05 and not torch.isnan(target).any()

    sigma, gamma = 1e-3, 1e-2
    rast = GaussianRast(nb_samples=8, sigma=sigma)
    agg = GaussianAgg(nb_samples=8, gamma=gamma)
    rs = RasterizationSettings(image_size=imsize, blur_radius=math.log(1.0 / 1e-4 - 1.0) * sigma,
                               faces_per_pixel=16, max_faces_per_bin=100000)
    renderer = MeshRenderer(MeshRasterizer(cameras=cam, raster_settings=rs),
                            RandomPhongShader(device=device, cameras=cam, lights=lights, smoothrast=rast,
                                              smoothagg=agg, blend_params=BlendParams(sigma, gamma, (0.0, 0.0, 0.0))))
    log_rot = (so3_log_map(R_true) + torch.tensor([[0.25, -0.2, 0.15]], device=device)).requires_grad_(True)
    opt = torch.optim.Adam([log_rot], lr=0.05)
    losses = []
    for _ in range(25):
        opt.zero_grad()
        Rc = so3_exponential_map(log_rot)
        img = renderer(meshes.update_padded(Rotate(Rc).transform_points(meshes.verts_padded())), cameras=cam,
                       lights=lights)
        loss = ((img[..., :3] - target) ** 2).mean()
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    err0 = float(so3_relative_angle(so3_exponential_map(log_rot.detach() * 0 + so3_log_map(R_true)
                                                        + torch.tensor([[0.25, -0.2, 0.15]], device=device)),
                                    R_true))
    err1 = float(so3_relative_angle(so3_exponential_map(log_rot.detach()), R_true))
    assert np.mean(losses[-5:]) < 0.8 * np.mean(losses[:3]), losses
    assert err1 < err0, (err0, err1)


def test_uv_texture_sampling_matches_numpy_bilinear(device):
    """TexturesUV.sample_textures on the GPU == bilinear sampling (align_corners=True, border,
    v flipped) of the map at the barycentric UVs, restated in numpy."""
    from pytorch3d.renderer import TexturesUV
    from pytorch3d.renderer.mesh import Fragments
    g = torch.Generator().manual_seed(1)
    Hm, Wm = 7, 9
    maps = torch.rand((1, Hm, Wm, 3), generator=g)
    vu = torch.rand((5, 2), generator=g) * 1.2 - 0.1
    fu = torch.tensor([[0, 1, 2], [2, 3, 4]])
    N, H, W, K = 1, 3, 4, 2
    p2f = torch.randint(-1, 2, (N, H, W, K), generator=g)
    bary = torch.rand((N, H, W, K, 3), generator=g)
    bary = bary / bary.sum(-1, keepdim=True)
    tex = TexturesUV(maps.to(device), fu[None].to(device), vu[None].to(device))
    out = tex.sample_textures(Fragments(p2f.to(device), None, bary.to(device), None)).cpu().numpy()
    m = maps[0].numpy()
    ref = np.zeros((N, H, W, K, 3), np.float32)
    for idx in np.ndindex(N, H, W, K):
        f = int(p2f[idx])
        uv = (bary[idx].numpy()[:, None] * vu[fu[max(f, 0)]].numpy()).sum(0) if f >= 0 else np.zeros(2)
        x = np.clip(uv[0] * (Wm - 1), 0, Wm - 1)
        y = np.clip((1.0 - uv[1]) * (Hm - 1), 0, Hm - 1)
        x0, y0 = int(np.floor(x)), int(np.floor(y))
        x1, y1 = min(x0 + 1, Wm - 1), min(y0 + 1, Hm - 1)
        fx, fy = x - x0, y - y0
        ref[idx] = ((1 - fx) * (1 - fy) * m[y0, x0] + fx * (1 - fy) * m[y0, x1] + (1 - fx) * fy * m[y1, x0]
                    + fx * fy * m[y1, x1])
    np.testing.assert_allclose(out, ref, rtol=1e-4, atol=1e-5)
