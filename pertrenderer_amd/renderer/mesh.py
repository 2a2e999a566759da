"""Triangle-mesh batch and per-vertex textures (PyTorch3D ``Meshes`` / ``TexturesVertex``
subset used by experiments/eval.py and random_rasterizer.py:170).

Layout: per-mesh vertex lists plus a shared, lazily built topology record (packed
faces, per-mesh face offsets/counts as device tensors).  Meshes derived by
``update_padded`` / ``offset_verts`` share the record, so a pose-optimisation step
builds no index tensor and does no host->device copy: it is safe to capture in a
HIP graph.  ``sample_textures`` runs the native face-attribute interpolation.
"""
import os

import torch

from . import interp as _interp

F32 = torch.float32


def gather_faces(values, faces_packed):
    """values[faces] as (F,3,C) via index_select (its backward is an index_add, no sort)."""
    F = faces_packed.shape[0]
    return values.index_select(0, faces_packed.reshape(-1)).reshape(F, 3, values.shape[-1])


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
        return self._list[0] if len(self._list) == 1 else torch.cat(self._list, dim=0)

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
        return _interp.interpolate_vertex_attributes(fragments.pix_to_face, fragments.bary_coords,
                                                     self.verts_features_packed(), faces_packed)


class _Topology:
    def __init__(self, faces, nverts, device):
        self.faces = faces
        self.nverts = list(nverts)
        self.nfaces = [f.shape[0] for f in faces]
        self.device = device
        self._packed = None
        self._idx = None
        self._csr = {}

    def faces_packed(self):
        if self._packed is None:
            offs, out = 0, []
            for nv, f in zip(self.nverts, self.faces):
                out.append(f.to(self.device) + offs)
                offs += nv
            self._packed = torch.cat(out, dim=0).contiguous()
        return self._packed

    def index_tensors(self):
        if self._idx is None:
            nf = torch.tensor(self.nfaces, dtype=torch.int64)
            first = torch.cumsum(nf, 0) - nf
            nv = torch.tensor(self.nverts, dtype=torch.int64)
            self._idx = dict(nfaces=nf.to(self.device), first=first.to(self.device), nverts=nv.to(self.device),
                             vfirst=(torch.cumsum(nv, 0) - nv).to(self.device))
        return self._idx

    def corner_csr(self, kind="gather"):
        """Vertex -> face-corner index (CSR) of the packed mesh: (start (V+1), corners (3F)) int64,
        the corners t = 3 f + i of vertex v at corners[start[v]:start[v+1]].  "gather": in
        increasing t (the order of the verts[faces] backward); "normals": PyTorch3D's normal
        accumulation order (corner 1 of every face, then corner 2, then corner 0: its three
        index_adds).  Built once per topology on the device (stable sort, no host sync), so the
        native projection / normals passes gather per vertex without atomics."""
        c = self._csr.get(kind)
        if c is None:
            f = self.faces_packed()
            F, V = f.shape[0], sum(self.nverts)
            t = torch.arange(3 * F, device=f.device).reshape(F, 3)
            perm = [1, 2, 0] if kind == "normals" else [0, 1, 2]
            keys = f[:, perm].t().reshape(-1) if kind == "normals" else f.reshape(-1)
            vals = t[:, perm].t().reshape(-1) if kind == "normals" else t.reshape(-1)
            order = torch.argsort(keys, stable=True)
            start = torch.searchsorted(keys[order].contiguous(), torch.arange(V + 1, device=f.device))
            c = self._csr[kind] = (start.contiguous(), vals[order].contiguous())
        return c


class Meshes:
    """A batch of triangle meshes (lists of (V_i,3) verts and (F_i,3) int64 faces)."""

    def __init__(self, verts, faces, textures=None, _topo=None):
        if torch.is_tensor(verts):
            verts = [v for v in verts] if verts.dim() == 3 else [verts]
        if _topo is None:
            if torch.is_tensor(faces):
                faces = [f for f in faces] if faces.dim() == 3 else [faces]
            if len(verts) != len(faces):
                raise ValueError("verts and faces must have the same batch size")
            dev = verts[0].device if verts else torch.device("cpu")
            _topo = _Topology([f.to(torch.int64) for f in faces], [v.shape[0] for v in verts], dev)
        self._verts = list(verts)
        self._topo = _topo
        self.textures = textures
        self.device = self._verts[0].device if self._verts else torch.device("cpu")

    def __len__(self):
        return len(self._verts)

    def isempty(self):
        return len(self._verts) == 0 or all(v.shape[0] == 0 for v in self._verts)

    # ---------------------------------------------------------------- views
    def verts_list(self):
        return self._verts

    def faces_list(self):
        return self._topo.faces

    def num_verts_per_mesh(self):
        return self._topo.index_tensors()["nverts"]

    def num_faces_per_mesh(self):
        return self._topo.index_tensors()["nfaces"]

    def mesh_to_faces_packed_first_idx(self):
        return self._topo.index_tensors()["first"]

    def mesh_to_verts_packed_first_idx(self):
        return self._topo.index_tensors()["vfirst"]

    def verts_packed(self):
        return self._verts[0] if len(self._verts) == 1 else torch.cat(self._verts, dim=0)

    def faces_packed(self):
        return self._topo.faces_packed()

    def corner_csr(self, kind="gather"):
        """Vertex -> face-corner CSR of the packed topology (_Topology.corner_csr); not PyTorch3D API."""
        return self._topo.corner_csr(kind)

    def verts_padded(self):
        if len(self._verts) == 1:
            return self._verts[0][None]  # a view: no copy kernel
        if all(v.shape[0] == self._verts[0].shape[0] for v in self._verts):
            return torch.stack(self._verts, 0)
        V = max(v.shape[0] for v in self._verts)
        out = self._verts[0].new_zeros((len(self._verts), V, 3))
        for i, v in enumerate(self._verts):
            out[i, : v.shape[0]] = v
        return out

    def faces_padded(self):
        faces = self._topo.faces
        Fm = max(f.shape[0] for f in faces)
        out = faces[0].new_full((len(faces), Fm, 3), -1)
        for i, f in enumerate(faces):
            out[i, : f.shape[0]] = f
        return out

    def verts_normals_packed(self):
        """Area-weighted vertex normals (PyTorch3D convention).  On the GPU one native kernel pair
        (pr_vert_normals_fwd/bwd) instead of ~20 torch kernels per direction (NATIVE_NORMALS)."""
        v = self.verts_packed()
        f = self.faces_packed()
        if NATIVE_NORMALS and v.is_cuda and v.dtype == torch.float32:
            from .. import host_layer
            ext = host_layer.get()
            if ext is not None:  # the C++ autograd layer (host_layer.py): same kernels
                return ext.vert_normals(v, f, *self._topo.corner_csr("normals"))
            return _VertNormalsFn.apply(v, f, *self._topo.corner_csr("normals"))
        fv = gather_faces(v, f)
        n = torch.zeros_like(v)
        # each corner's cross product is 2x the face area times its normal
        n = n.index_add(0, f[:, 1], torch.cross(fv[:, 2] - fv[:, 1], fv[:, 0] - fv[:, 1], dim=1))
        n = n.index_add(0, f[:, 2], torch.cross(fv[:, 0] - fv[:, 2], fv[:, 1] - fv[:, 2], dim=1))
        n = n.index_add(0, f[:, 0], torch.cross(fv[:, 1] - fv[:, 0], fv[:, 2] - fv[:, 0], dim=1))
        return torch.nn.functional.normalize(n, eps=1e-6, dim=1)

    # ------------------------------------------------------------- updates
    def _new(self, verts):
        return Meshes(verts, None, self.textures, _topo=self._topo)

    def update_padded(self, new_verts_padded):
        nv = self._topo.nverts
        if len(nv) == 1 and new_verts_padded.shape[1] == nv[0]:
            # a reshape, not a slice: its backward is a view (a slice's is a zero-fill + copy)
            return self._new([new_verts_padded.reshape(nv[0], new_verts_padded.shape[-1])])
        return self._new([new_verts_padded[i, : n] for i, n in enumerate(nv)])

    def offset_verts(self, vert_offsets_packed):
        off = vert_offsets_packed
        if off.dim() == 1:
            off = off.expand(sum(self._topo.nverts), 3)
        chunks = torch.split(off, self._topo.nverts, dim=0)
        return self._new([v + o for v, o in zip(self._verts, chunks)])

    def offset_verts_(self, vert_offsets_packed):
        self._verts = self.offset_verts(vert_offsets_packed)._verts
        return self

    def scale_verts(self, scale):
        s = scale if torch.is_tensor(scale) else torch.full((len(self),), float(scale))
        s = s.reshape(-1).expand(len(self))
        return self._new([v * float(s[i]) for i, v in enumerate(self._verts)])

    def scale_verts_(self, scale):
        self._verts = self.scale_verts(scale)._verts
        return self

    def extend(self, N):
        tex = self.textures.extend(N) if self.textures is not None else None
        return Meshes([v.clone() for v in self._verts for _ in range(N)],
                      [f.clone() for f in self._topo.faces for _ in range(N)], tex)

    def clone(self):
        return Meshes([v.clone() for v in self._verts], [f.clone() for f in self._topo.faces],
                      self.textures.clone() if self.textures is not None else None)

    def detach(self):
        return Meshes([v.detach() for v in self._verts], None,
                      self.textures.detach() if self.textures is not None else None, _topo=self._topo)

    def to(self, device):
        return Meshes([v.to(device) for v in self._verts], [f.to(device) for f in self._topo.faces],
                      self.textures.to(device) if self.textures is not None else None)

    def sample_textures(self, fragments):
        if self.textures is None:
            raise ValueError("Meshes has no textures")
        return self.textures.sample_textures(fragments, faces_packed=self.faces_packed())


# Meshes.verts_normals_packed on the native kernels when the mesh is on the GPU (PR_NATIVE_NORMALS=0 or False for
# the torch composition above; tests/test_gpu_normals.py compares the two)
NATIVE_NORMALS = os.environ.get("PR_NATIVE_NORMALS", "1") == "1"


class _VertNormalsFn(torch.autograd.Function):
    """verts -> area-weighted, normalised vertex normals (pr_vert_normals_fwd/bwd), gathered per
    vertex over the topology's corner CSR (deterministic, no atomics).  Its backward runs on the
    kernels' outputs, so it is once-differentiable: a double backward raises instead of returning
    silent zeros."""

    @staticmethod
    def forward(ctx, verts, faces, csr_start=None, csr_corners=None):
        from .. import _native as nat
        v = verts.detach().contiguous()
        f = nat.dense(faces, torch.int64)
        n = torch.empty_like(v)
        raw = torch.empty_like(v)
        a = nat.PRNormalsArgs()
        a.verts, a.faces, a.V, a.F = nat.ptr(v), nat.ptr(f), v.shape[0], f.shape[0]
        a.normals, a.raw = nat.ptr(n), nat.ptr(raw)
        a.vert_corner_start, a.vert_corners = nat.ptr(csr_start), nat.ptr(csr_corners)
        nat.call("pr_vert_normals_fwd", "pr_vert_normals_fwd", v, a)
        ctx.save_for_backward(v, f, raw)
        ctx.csr = (csr_start, csr_corners)
        return n

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        from .. import _native as nat
        v, f, raw = ctx.saved_tensors
        gc = nat.dense(g, torch.float32)
        graw, gv = torch.empty_like(v), torch.empty_like(v)
        a = nat.PRNormalsArgs()
        a.verts, a.faces, a.V, a.F = nat.ptr(v), nat.ptr(f), v.shape[0], f.shape[0]
        a.raw, a.grad_normals, a.grad_raw, a.grad_verts = nat.ptr(raw), nat.ptr(gc), nat.ptr(graw), nat.ptr(gv)
        a.vert_corner_start, a.vert_corners = nat.ptr(ctx.csr[0]), nat.ptr(ctx.csr[1])
        nat.call("pr_vert_normals_bwd", "pr_vert_normals_bwd", gc, a)
        return gv, None, None, None
