"""Triangle-mesh batch and per-vertex textures (PyTorch3D ``Meshes`` / ``TexturesVertex``
subset used by experiments/eval.py and random_rasterizer.py:170).

Memory layout: vertices and faces are kept as per-mesh lists plus lazily built
packed views (faces_packed indexes verts_packed).  ``sample_textures`` runs the
native face-attribute interpolation (pr_interp_*).
"""
import torch

from . import interp as _interp

F32 = torch.float32


class TexturesVertex:
    """Per-vertex features interpolated with barycentrics (PyTorch3D TexturesVertex)."""

    def __init__(self, verts_features):
        if torch.is_tensor(verts_features):
            self._list = [f for f in verts_features] if verts_features.dim() == 3 else [verts_features]
        else:
            self._list = list(verts_features)

    def verts_features_list(self):
        return self._list

    def verts_features_packed(self):
        return torch.cat(self._list, dim=0)

    def verts_features_padded(self):
        V = max(f.shape[0] for f in self._list)
        out = self._list[0].new_zeros((len(self._list), V, self._list[0].shape[-1]))
        for i, f in enumerate(self._list):
            out[i, : f.shape[0]] = f
        return out

    def extend(self, N):
        return TexturesVertex([f for f in self._list for _ in range(N)])

    def clone(self):
        return TexturesVertex([f.clone() for f in self._list])

    def detach(self):
        return TexturesVertex([f.detach() for f in self._list])

    def to(self, device):
        return TexturesVertex([f.to(device) for f in self._list])

    def sample_textures(self, fragments, faces_packed=None, **kwargs):
        """(N,H,W,K,C) texels = sum_i bary_i * feature[face_i] (0 on padded slots)."""
        face_attr = self.verts_features_packed()[faces_packed]
        return _interp.interpolate_face_attributes(fragments.pix_to_face, fragments.bary_coords, face_attr)


class Meshes:
    """A batch of triangle meshes (lists of (V_i,3) verts and (F_i,3) int64 faces)."""

    def __init__(self, verts, faces, textures=None):
        if torch.is_tensor(verts):
            verts = [v for v in verts] if verts.dim() == 3 else [verts]
        if torch.is_tensor(faces):
            faces = [f for f in faces] if faces.dim() == 3 else [faces]
        if len(verts) != len(faces):
            raise ValueError("verts and faces must have the same batch size")
        self._verts = list(verts)
        self._faces = [f.to(torch.int64) for f in faces]
        self.textures = textures
        self.device = self._verts[0].device if self._verts else torch.device("cpu")
        self._packed = None

    def __len__(self):
        return len(self._verts)

    def isempty(self):
        return len(self._verts) == 0 or all(v.shape[0] == 0 for v in self._verts)

    # ---------------------------------------------------------------- views
    def verts_list(self):
        return self._verts

    def faces_list(self):
        return self._faces

    def num_verts_per_mesh(self):
        return torch.tensor([v.shape[0] for v in self._verts], dtype=torch.int64, device=self.device)

    def num_faces_per_mesh(self):
        return torch.tensor([f.shape[0] for f in self._faces], dtype=torch.int64, device=self.device)

    def mesh_to_faces_packed_first_idx(self):
        nf = self.num_faces_per_mesh()
        return torch.cumsum(nf, 0) - nf

    def mesh_to_verts_packed_first_idx(self):
        nv = self.num_verts_per_mesh()
        return torch.cumsum(nv, 0) - nv

    def verts_packed(self):
        return torch.cat(self._verts, dim=0)

    def faces_packed(self):
        if self._packed is None:
            offs, out = 0, []
            for v, f in zip(self._verts, self._faces):
                out.append(f.to(v.device) + offs)
                offs += v.shape[0]
            self._packed = torch.cat(out, dim=0)
        return self._packed

    def verts_padded(self):
        V = max(v.shape[0] for v in self._verts)
        out = self._verts[0].new_zeros((len(self._verts), V, 3))
        for i, v in enumerate(self._verts):
            out[i, : v.shape[0]] = v
        return out

    def faces_padded(self):
        Fm = max(f.shape[0] for f in self._faces)
        out = self._faces[0].new_full((len(self._faces), Fm, 3), -1)
        for i, f in enumerate(self._faces):
            out[i, : f.shape[0]] = f
        return out

    def verts_normals_packed(self):
        """Area-weighted vertex normals (PyTorch3D convention)."""
        v = self.verts_packed()
        f = self.faces_packed().to(v.device)
        fv = v[f]
        n = torch.zeros_like(v)
        # each corner's cross product is 2x the face area times its normal
        n = n.index_add(0, f[:, 1], torch.cross(fv[:, 2] - fv[:, 1], fv[:, 0] - fv[:, 1], dim=1))
        n = n.index_add(0, f[:, 2], torch.cross(fv[:, 0] - fv[:, 2], fv[:, 1] - fv[:, 2], dim=1))
        n = n.index_add(0, f[:, 0], torch.cross(fv[:, 1] - fv[:, 0], fv[:, 2] - fv[:, 0], dim=1))
        return torch.nn.functional.normalize(n, eps=1e-6, dim=1)

    # ------------------------------------------------------------- updates
    def _new(self, verts):
        m = Meshes(verts, self._faces, self.textures)
        return m

    def update_padded(self, new_verts_padded):
        return self._new([new_verts_padded[i, : v.shape[0]] for i, v in enumerate(self._verts)])

    def offset_verts(self, vert_offsets_packed):
        off = vert_offsets_packed
        if off.dim() == 1:
            off = off.expand(self.verts_packed().shape[0], 3)
        chunks = torch.split(off, [v.shape[0] for v in self._verts], dim=0)
        return self._new([v + o for v, o in zip(self._verts, chunks)])

    def offset_verts_(self, vert_offsets_packed):
        m = self.offset_verts(vert_offsets_packed)
        self._verts = m._verts
        return self

    def scale_verts(self, scale):
        s = scale if torch.is_tensor(scale) else torch.full((len(self),), float(scale))
        s = s.reshape(-1).expand(len(self))
        return self._new([v * float(s[i]) for i, v in enumerate(self._verts)])

    def scale_verts_(self, scale):
        m = self.scale_verts(scale)
        self._verts = m._verts
        return self

    def extend(self, N):
        tex = self.textures.extend(N) if self.textures is not None else None
        return Meshes([v.clone() for v in self._verts for _ in range(N)],
                      [f.clone() for f in self._faces for _ in range(N)], tex)

    def clone(self):
        return Meshes([v.clone() for v in self._verts], [f.clone() for f in self._faces],
                      self.textures.clone() if self.textures is not None else None)

    def detach(self):
        return Meshes([v.detach() for v in self._verts], self._faces,
                      self.textures.detach() if self.textures is not None else None)

    def to(self, device):
        return Meshes([v.to(device) for v in self._verts], [f.to(device) for f in self._faces],
                      self.textures.to(device) if self.textures is not None else None)

    def sample_textures(self, fragments):
        if self.textures is None:
            raise ValueError("Meshes has no textures")
        return self.textures.sample_textures(fragments, faces_packed=self.faces_packed())
