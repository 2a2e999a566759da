"""CPU oracle of eval.py's whole perturbed render (TEST INFRASTRUCTURE ONLY: imported by tests/
alone, never by the product).

One RandomPhongShader frame of experiments/eval.py (init_renderers :124-180, the cube of
load_cube :727-757) composed from the oracles, with autograd through each piece:
  * projection: the package's torch camera transforms (world -> view -> NDC, view z kept), as
    MeshRasterizer.transform does (PyTorch3D 0.4.0 rasterizer.py);
  * rasterization: the C oracle (oracle/rast_oracle.c) forward and backward, wrapped as one
    autograd Function;
  * TexturesUV sampling (PyTorch3D TexturesUV.sample_textures: interpolated UVs, map flipped
    vertically, grid_sample align_corners=True, padding "border") and Phong shading
    (PyTorch3D phong_shading / lighting.py diffuse + specular, PointLights and Materials
    defaults) restated here in torch;
  * the perturbed blend: oracle/blend_oracle.py's closed-form forward and backward
    (random_rasterizer.py:34-56, smoothrast.py, smoothagg.py), with the reference's own noise
    draws injected.
Parity of each piece is pinned elsewhere (tests/golden, the rasterizer KATs); this module pins
the composition: the GPU renderer and this one, fed the same draws, give the same images and
pose gradients, and the same pose-optimisation runs (tests/test_gpu_pipeline_ref.py)."""
import numpy as np
import torch
import torch.nn.functional as F

from oracle import blend_oracle as bo
from oracle import rast_ref

F32 = torch.float32


class RastRef(torch.autograd.Function):
    """rasterize_meshes on face_verts (F,3,3) of one mesh -> (p2f, zbuf, bary, dists)."""

    @staticmethod
    def forward(ctx, fv, H, W, K, blur, clip):
        f = fv.detach().numpy()
        p2f, zbuf, bary, dists = rast_ref.rast_fwd(f, [0], [f.shape[0]], H, W, K, blur, False, clip, False)
        ctx.save_for_backward(fv)
        ctx.p2f, ctx.clip = p2f, clip
        return (torch.from_numpy(p2f), torch.from_numpy(zbuf), torch.from_numpy(bary), torch.from_numpy(dists))

    @staticmethod
    def backward(ctx, g_p2f, gz, gb, gd):
        (fv,) = ctx.saved_tensors
        z = lambda g, shape: np.zeros(shape, np.float32) if g is None else g.detach().numpy()
        p2f = ctx.p2f
        out = rast_ref.rast_bwd(fv.detach().numpy(), p2f, z(gz, p2f.shape), z(gb, p2f.shape + (3,)),
                                z(gd, p2f.shape), False, ctx.clip)
        return torch.from_numpy(out), None, None, None, None, None


class BlendRef(torch.autograd.Function):
    """smooth_rgb_blend(colors, fragments, GaussianRast, GaussianAgg) with injected noise."""

    @staticmethod
    def forward(ctx, dists, zbuf, colors, sigma, gamma, alpha, p2f, noise_r, noise_a, bg, znear, zfar):
        img, saved = bo.blend_forward(p2f, dists.detach(), zbuf.detach(), colors.detach(), noise_r, noise_a,
                                      sigma.detach(), gamma.detach(), alpha.detach(), 1e-10, bg, znear, zfar)
        ctx.saved = saved
        return img

    @staticmethod
    def backward(ctx, gimg):
        g = bo.blend_backward(gimg.contiguous(), ctx.saved)
        return (g["dists"], g["zbuf"], g["colors"], g["sigma"].reshape(()), g["gamma"].reshape(()),
                g["alpha"].reshape(()), None, None, None, None, None, None)


def _interp(p2f, bary, face_attr):
    """interpolate_face_attributes: sum_i bary_i attr[f, i], 0 where p2f < 0 (PyTorch3D)."""
    mask = p2f >= 0
    fa = face_attr[torch.where(mask, p2f, torch.zeros_like(p2f))]            # (...,K,3,D)
    out = (bary[..., None] * fa).sum(-2)
    return out * mask[..., None]


def sample_uv(p2f, bary, faces_uvs, verts_uvs, maps):
    """TexturesUV.sample_textures: bilinear, align_corners, border padding, map flipped (UV (0,0)
    is the map's bottom-left) -> (N,H,W,K,C)."""
    uv = _interp(p2f, bary, verts_uvs[faces_uvs])                             # (N,H,W,K,2)
    N, H, W, K, _ = uv.shape
    grid = (uv * 2.0 - 1.0).reshape(N, H, W * K, 2)
    tex = maps.permute(0, 3, 1, 2).flip([2])                                  # (N,C,Hm,Wm), row 0 = v 0
    s = F.grid_sample(tex, grid, mode="bilinear", padding_mode="border", align_corners=True)
    return s.permute(0, 2, 3, 1).reshape(N, H, W, K, -1)


def phong(p2f, bary, verts, faces, vnormals, texels, light_loc, cam_center, ambient=0.5, diffuse_c=0.3,
          specular_c=0.2, shininess=64.0):
    """PyTorch3D phong_shading with PointLights(ambient 0.5, diffuse 0.3, specular 0.2) and
    default Materials (ones, shininess 64): (ambient + diffuse) * texels + specular."""
    coords = _interp(p2f, bary, verts[faces])
    normals = _interp(p2f, bary, vnormals[faces])
    direction = light_loc.reshape(1, 1, 1, 1, 3) - coords
    n = F.normalize(normals, p=2, dim=-1, eps=1e-6)
    d = F.normalize(direction, p=2, dim=-1, eps=1e-6)
    cos = (n * d).sum(-1)
    diff = diffuse_c * F.relu(cos)[..., None]
    view = F.normalize(cam_center.reshape(1, 1, 1, 1, 3) - coords, p=2, dim=-1, eps=1e-6)
    refl = -d + 2 * (cos[..., None] * n)
    a = F.relu((view * refl).sum(-1)) * (cos > 0).to(F32)
    spec = specular_c * torch.pow(a, shininess)[..., None]
    return (ambient + diff) * texels + spec


def render(mesh, camera, light_loc, tex, H, K, blur, sigma, gamma, alpha, noise_r, noise_a, background=(0.0, 0.0, 0.0)):
    """One RandomPhongShader(GaussianRast, GaussianAgg) frame of `mesh` (a CPU Meshes whose
    verts may carry the pose gradient) -> (1,H,H,4)."""
    verts = mesh.verts_packed()
    faces = mesh.faces_packed()
    view = camera.get_world_to_view_transform().transform_points(verts[None])
    ndc = camera.get_projection_transform().transform_points(view)
    screen = torch.cat([ndc[..., :2], view[..., 2:3]], -1)[0]
    p2f, zbuf, bary, dists = RastRef.apply(screen[faces], H, H, K, blur, blur > 0.0)
    faces_uvs, verts_uvs, maps = tex
    texels = sample_uv(p2f, bary, faces_uvs, verts_uvs, maps)
    colors = phong(p2f, bary, verts, faces, mesh.verts_normals_packed(), texels, light_loc,
                   camera.get_camera_center()[0])
    zn = torch.full((1, 1, 1, 1), float(camera.znear))
    zf = torch.full((1, 1, 1, 1), float(camera.zfar))
    return BlendRef.apply(dists, zbuf, colors, sigma, gamma, alpha, p2f, noise_r, noise_a,
                          torch.tensor(background, dtype=F32), zn, zf)
