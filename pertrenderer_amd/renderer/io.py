"""Wavefront OBJ / MTL reader with PyTorch3D 0.4.0's ``load_obj`` return structure
(experiments/eval.py:224-237, 296-297, 746-755):

    verts (V,3), Faces(verts_idx, normals_idx, textures_idx, materials_idx),
    Properties(normals, verts_uvs, material_colors, texture_images, texture_atlas)

Polygons are fan-split.  Texture images (map_Kd) load through PIL as (H,W,3) float
in [0,1].  ``create_texture_atlas`` samples each face's UV triangle of its material's
texture on an R x R grid in the TexturesAtlas layout (textures.py).  Parity with
PyTorch3D's loader is unpinned (not installable here); the reference's own meshes
(data/objs/rubiks/cube2.obj + .mtl + .png, data/objs/sphere/sphere_642.obj) are the
test inputs."""
import os
from typing import NamedTuple, Optional

import numpy as np
import torch
import torch.nn.functional as F


class Faces(NamedTuple):
    verts_idx: torch.Tensor
    normals_idx: torch.Tensor
    textures_idx: torch.Tensor
    materials_idx: torch.Tensor


class Properties(NamedTuple):
    normals: Optional[torch.Tensor]
    verts_uvs: Optional[torch.Tensor]
    material_colors: Optional[dict]
    texture_images: Optional[dict]
    texture_atlas: Optional[torch.Tensor]


Aux = Properties  # earlier name


def _load_mtl(path, load_textures):
    colors, images, cur = {}, {}, None
    base = os.path.dirname(path)
    with open(path, "r") as fh:
        for line in fh:
            tok = line.split()
            if not tok or tok[0].startswith("#"):
                continue
            if tok[0] == "newmtl":
                cur = tok[1]
                colors[cur] = {}
            elif cur is not None and tok[0] in ("Ka", "Kd", "Ks"):
                key = {"Ka": "ambient_color", "Kd": "diffuse_color", "Ks": "specular_color"}[tok[0]]
                colors[cur][key] = torch.tensor([float(x) for x in tok[1:4]], dtype=torch.float32)
            elif cur is not None and tok[0] == "Ns":
                colors[cur]["shininess"] = torch.tensor([float(tok[1])], dtype=torch.float32)
            elif cur is not None and tok[0] == "map_Kd" and load_textures:
                from PIL import Image
                img = Image.open(os.path.join(base, tok[-1])).convert("RGB")
                images[cur] = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0)
    return colors, images


def _atlas(verts_uvs, faces_uvs, mat_idx, images, names, R, wrap):
    """(F,R,R,3) texel grids: texel (y, x) of face f is its material image sampled at the UV of
    barycentric (w0, w1) = ((x + 1/3)/R, (y + 1/3)/R) below the diagonal, mirrored above it."""
    Fn = faces_uvs.shape[0]
    atlas = torch.zeros((Fn, R, R, 3), dtype=torch.float32)
    ii, jj = torch.meshgrid(torch.arange(R), torch.arange(R), indexing="ij")   # (y, x)
    below = (ii + jj) <= R - 1
    w0 = torch.where(below, (jj + 1.0 / 3) / R, (R - jj - 1.0 / 3) / R)
    w1 = torch.where(below, (ii + 1.0 / 3) / R, (R - ii - 1.0 / 3) / R)
    w2 = 1.0 - w0 - w1
    for m, name in enumerate(names):
        sel = (mat_idx == m).nonzero().reshape(-1)
        if sel.numel() == 0 or name not in images:
            continue
        img = images[name]                                             # (H,W,3)
        tri = verts_uvs[faces_uvs[sel]]                                # (f,3,2)
        uv = (w0[None, ..., None] * tri[:, None, None, 0] + w1[None, ..., None] * tri[:, None, None, 1]
              + w2[None, ..., None] * tri[:, None, None, 2])           # (f,R,R,2)
        if wrap == "repeat":
            uv = uv - torch.floor(uv)
        elif wrap == "clamp":
            uv = uv.clamp(0.0, 1.0)
        grid = (uv * 2.0 - 1.0).reshape(1, -1, R * R, 2)
        m_img = torch.flip(img.permute(2, 0, 1)[None], [2])
        s = F.grid_sample(m_img, grid, align_corners=True, padding_mode="border")   # (1,3,f,R*R)
        atlas[sel] = s[0].permute(1, 2, 0).reshape(-1, R, R, 3)
    return atlas


def load_obj(path, load_textures=True, create_texture_atlas=False, texture_atlas_size=4,
             texture_wrap="repeat", device="cpu", path_manager=None):
    verts, uvs, normals = [], [], []
    fv, ft, fn, fm = [], [], [], []
    mtl_files, mat_names, cur_mat = [], [], -1
    with open(path, "r") as fh:
        for line in fh:
            tok = line.split()
            if not tok or tok[0].startswith("#"):
                continue
            if tok[0] == "v":
                verts.append([float(x) for x in tok[1:4]])
            elif tok[0] == "vt":
                uvs.append([float(x) for x in tok[1:3]])
            elif tok[0] == "vn":
                normals.append([float(x) for x in tok[1:4]])
            elif tok[0] == "mtllib":
                mtl_files.append(os.path.join(os.path.dirname(path), tok[1]))
            elif tok[0] == "usemtl":
                if tok[1] not in mat_names:
                    mat_names.append(tok[1])
                cur_mat = mat_names.index(tok[1])
            elif tok[0] == "f":
                idx = []
                for t in tok[1:]:
                    parts = t.split("/")
                    gi = lambda j, n: (int(parts[j]) - 1 if int(parts[j]) > 0 else n + int(parts[j])) \
                        if len(parts) > j and parts[j] else -1
                    idx.append((gi(0, len(verts)), gi(1, len(uvs)), gi(2, len(normals))))
                for k in range(1, len(idx) - 1):
                    tri = (idx[0], idx[k], idx[k + 1])
                    fv.append([t[0] for t in tri])
                    ft.append([t[1] for t in tri])
                    fn.append([t[2] for t in tri])
                    fm.append(cur_mat)
    colors, images = {}, {}
    for mf in mtl_files:
        if os.path.exists(mf):
            c, i = _load_mtl(mf, load_textures)
            colors.update(c)
            images.update(i)
    V = torch.tensor(verts, dtype=torch.float32)
    faces = Faces(torch.tensor(fv, dtype=torch.int64).reshape(-1, 3),
                  torch.tensor(fn, dtype=torch.int64).reshape(-1, 3),
                  torch.tensor(ft, dtype=torch.int64).reshape(-1, 3),
                  torch.tensor(fm, dtype=torch.int64))
    verts_uvs = torch.tensor(uvs, dtype=torch.float32).reshape(-1, 2)
    atlas = None
    if create_texture_atlas:
        atlas = _atlas(verts_uvs, faces.textures_idx, faces.materials_idx, images, mat_names,
                       int(texture_atlas_size), texture_wrap)
    to = lambda t: t.to(device) if torch.is_tensor(t) else t
    aux = Properties(to(torch.tensor(normals, dtype=torch.float32).reshape(-1, 3)), to(verts_uvs),
                     {k: {kk: to(vv) for kk, vv in v.items()} for k, v in colors.items()} or None,
                     {k: to(v) for k, v in images.items()} or None, to(atlas))
    return to(V), Faces(*[to(t) for t in faces]), aux


def load_objs_as_meshes(files, device="cpu", load_textures=True, create_texture_atlas=False,
                        texture_atlas_size=4, texture_wrap="repeat", path_manager=None):
    """Meshes from OBJ files with UV textures (first material's image) or an atlas."""
    from .mesh import Meshes
    from .textures import TexturesAtlas, TexturesUV
    verts, faces, maps, fuvs, vuvs, atlases = [], [], [], [], [], []
    for f in files:
        v, fc, aux = load_obj(f, load_textures, create_texture_atlas, texture_atlas_size, texture_wrap, device)
        verts.append(v)
        faces.append(fc.verts_idx)
        if create_texture_atlas:
            atlases.append(aux.texture_atlas)
        elif load_textures and aux.texture_images:
            maps.append(list(aux.texture_images.values())[0])
            fuvs.append(fc.textures_idx)
            vuvs.append(aux.verts_uvs)
    tex = None
    if atlases:
        tex = TexturesAtlas(atlases)
    elif maps and len(maps) == len(files):
        tex = TexturesUV(maps, fuvs, vuvs)
    return Meshes(verts, faces, tex)
