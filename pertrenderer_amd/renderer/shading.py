"""Phong shading of per-slot texels (PyTorch3D phong_shading, used by
RandomPhongShader at random_rasterizer.py:103-110).  Pixel positions and normals
are interpolated on the native pr_interp kernels; the lighting is elementwise."""
import torch
import torch.nn.functional as Fn

from .interp import interpolate_vertex_attributes


def _bc(t, like):
    """(N,C) / (N,) per-batch parameters broadcast against (N,H,W,K,...) tensors."""
    t = t.to(like.device)
    if t.dim() == 2:
        return t.reshape((t.shape[0],) + (1,) * (like.dim() - 2) + (t.shape[-1],))
    return t.reshape((t.shape[0],) + (1,) * (like.dim() - 2))


def _diffuse(normals, color, direction):
    n = Fn.normalize(normals, p=2, dim=-1, eps=1e-6)
    d = Fn.normalize(direction, p=2, dim=-1, eps=1e-6)
    angle = Fn.relu(torch.sum(n * d, dim=-1))
    return _bc(color, normals) * angle[..., None]


def _specular(points, normals, direction, camera_position, color, shininess):
    n = Fn.normalize(normals, p=2, dim=-1, eps=1e-6)
    d = Fn.normalize(direction, p=2, dim=-1, eps=1e-6)
    cos_angle = torch.sum(n * d, dim=-1)
    mask = (cos_angle > 0).to(torch.float32)
    view = Fn.normalize(_bc(camera_position, points) - points, p=2, dim=-1, eps=1e-6)
    reflect = -d + 2 * (cos_angle[..., None] * n)
    alpha = Fn.relu(torch.sum(view * reflect, dim=-1)) * mask
    return _bc(color, points) * torch.pow(alpha, _bc(shininess, alpha))[..., None]


def phong_shading(meshes, fragments, lights, cameras, materials, texels):
    verts = meshes.verts_packed()
    faces = meshes.faces_packed()
    vnormals = meshes.verts_normals_packed()
    coords = interpolate_vertex_attributes(fragments.pix_to_face, fragments.bary_coords, verts, faces)
    normals = interpolate_vertex_attributes(fragments.pix_to_face, fragments.bary_coords, vnormals, faces)
    if hasattr(lights, "light_direction"):
        direction = lights.light_direction(coords)
    else:
        direction = _bc(lights.location, coords) - coords
    N = coords.shape[0]
    expand = lambda t: t.expand(N, -1) if t.shape[0] == 1 else t
    diffuse = _diffuse(normals, expand(lights.diffuse_color), direction)
    specular = _specular(coords, normals, direction, expand(cameras.get_camera_center()),
                         expand(lights.specular_color), expand(materials.shininess.reshape(-1)))
    ambient = _bc(expand(materials.ambient_color * lights.ambient_color), coords)
    diffuse = _bc(expand(materials.diffuse_color), coords) * diffuse
    specular = _bc(expand(materials.specular_color), coords) * specular
    return (ambient + diffuse) * texels + specular
