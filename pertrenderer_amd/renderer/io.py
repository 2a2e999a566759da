"""Minimal Wavefront OBJ reader (vertices, triangle faces, optional uv indices).

Enough for the reference's meshes (data/objs/rubiks/cube2.obj, data/objs/sphere/
sphere_642.obj, read at experiments/eval.py:297,347).  Polygons are fan-split."""
from typing import NamedTuple

import torch


class Faces(NamedTuple):
    verts_idx: torch.Tensor
    textures_idx: torch.Tensor
    normals_idx: torch.Tensor


class Aux(NamedTuple):
    verts_uvs: torch.Tensor
    normals: torch.Tensor


def load_obj(path, device="cpu"):
    verts, uvs, normals = [], [], []
    fv, ft, fn = [], [], []
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
    V = torch.tensor(verts, dtype=torch.float32, device=device)
    faces = Faces(torch.tensor(fv, dtype=torch.int64, device=device).reshape(-1, 3),
                  torch.tensor(ft, dtype=torch.int64, device=device).reshape(-1, 3),
                  torch.tensor(fn, dtype=torch.int64, device=device).reshape(-1, 3))
    aux = Aux(torch.tensor(uvs, dtype=torch.float32, device=device).reshape(-1, 2),
              torch.tensor(normals, dtype=torch.float32, device=device).reshape(-1, 3))
    return V, faces, aux
