"""Fused world -> NDC projection + face gather (pr_project_fwd / pr_project_bwd).

Replaces, for the rasterizer input, MeshRasterizer.transform (world->view, view->NDC,
keep view z) and rasterize_meshes' ``verts[faces]`` gather: one kernel forward, one
scatter-add kernel backward (d verts), instead of ~30 small tensor kernels each way.
Used when the camera matrices need no gradient; otherwise MeshRasterizer keeps the
differentiable tensor path.
"""
import torch

from .. import _native as nat

F32 = torch.float32


def _per_mesh(m, N, name):
    """(N,4,4) float32 contiguous matrices, one per mesh (the kernels index mesh n's matrix at
    n*16): one camera broadcast over a batch of meshes, as PyTorch3D does."""
    m = m.detach().to(F32)
    if m.dim() != 3 or m.shape[1:] != (4, 4) or m.shape[0] not in (1, N):
        raise ValueError(f"{name} matrices must be (1,4,4) or (N={N},4,4), got {tuple(m.shape)}")
    return (m.expand(N, 4, 4) if m.shape[0] != N else m).contiguous()


class _ProjectFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, verts, faces, first, nfaces, w2v, proj, csr_start=None, csr_corners=None):
        nat.require_device(verts, faces, w2v, proj)
        v = nat.dense(verts, F32)
        f = nat.dense(faces, torch.int64)
        a = nat.PRProjectArgs()
        a.verts, a.faces, a.mesh_first_face, a.mesh_num_faces = nat.ptr(v), nat.ptr(f), nat.ptr(first), nat.ptr(nfaces)
        N = first.shape[0]
        m1, m2 = _per_mesh(w2v, N, "world_to_view"), _per_mesh(proj, N, "projection")
        a.world_to_view, a.proj = nat.ptr(m1), nat.ptr(m2)
        a.V, a.F, a.N = v.shape[0], f.shape[0], N
        fv = torch.empty((f.shape[0], 3, 3), dtype=F32, device=v.device)
        a.face_verts = nat.ptr(fv)
        nat.call("pr_project_fwd", "pr_project_fwd", fv, a)
        ctx.save_for_backward(v, f, first, nfaces, m1, m2)
        ctx.csr = (csr_start, csr_corners)
        return fv

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        v, f, first, nfaces, m1, m2 = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return (None,) * 8
        go = nat.dense(g, F32)
        gv = torch.empty_like(v)
        a = nat.PRProjectArgs()
        a.verts, a.faces, a.mesh_first_face, a.mesh_num_faces = nat.ptr(v), nat.ptr(f), nat.ptr(first), nat.ptr(nfaces)
        a.world_to_view, a.proj = nat.ptr(m1), nat.ptr(m2)
        a.V, a.F, a.N = v.shape[0], f.shape[0], first.shape[0]
        a.grad_face_verts, a.grad_verts = nat.ptr(go), nat.ptr(gv)
        a.vert_corner_start, a.vert_corners = nat.ptr(ctx.csr[0]), nat.ptr(ctx.csr[1])
        nat.call("pr_project_bwd", "pr_project_bwd", go, a)
        return (gv,) + (None,) * 7


def project_faces(verts_packed, faces_packed, mesh_first_face, mesh_num_faces, world_to_view, proj, csr=None):
    """(V,3) world verts -> (F,3,3) face corners (x_ndc, y_ndc, z_view); matrices (N,4,4) row-vector.
    csr: the topology's vertex -> corner index (Meshes.corner_csr()), for the deterministic
    per-vertex gather backward (else one float atomic per corner component)."""
    start, corners = csr if csr is not None else (None, None)
    return _ProjectFn.apply(verts_packed, faces_packed, mesh_first_face, mesh_num_faces, world_to_view, proj,
                            start, corners)
