"""Barycentric interpolation of per-face-corner or per-vertex attributes on the native
kernels (pr_interp_fwd / pr_interp_bwd): PyTorch3D interpolate_face_attributes
semantics, 0 on padded slots (pix_to_face < 0).  The per-vertex form gathers
attr[faces[f, i]] inside the kernel (no (F,3,D) gather tensor, no index backward)."""
import torch

from .. import _native as nat

F32 = torch.float32


class _InterpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, bary, attr, p2f, faces):
        nat.require_device(bary, attr, p2f)
        shape = tuple(p2f.shape)
        D = attr.shape[-1]
        p2f_c = nat.dense(p2f, torch.int64)
        b_c = nat.dense(bary, F32)
        fa = nat.dense(attr, F32)
        fc = None if faces is None else nat.dense(faces, torch.int64)
        out = torch.empty(shape + (D,), dtype=F32, device=b_c.device)
        a = nat.PRInterpArgs()
        a.pix_to_face, a.bary, a.face_attr = nat.ptr(p2f_c), nat.ptr(b_c), nat.ptr(fa)
        a.PK, a.D, a.out = p2f_c.numel(), D, nat.ptr(out)
        a.F = fc.shape[0] if fc is not None else fa.shape[0]
        a.faces, a.V = nat.ptr(fc), (fa.shape[0] if fc is not None else 0)
        nat.call("pr_interp_fwd", "pr_interp_fwd", out, a)
        ctx.save_for_backward(b_c, fa, p2f_c, fc)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        b_c, fa, p2f_c, fc = ctx.saved_tensors
        need_b, need_f = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if not (need_b or need_f):
            return None, None, None, None
        go = nat.dense(g, F32)
        gb = torch.empty_like(b_c) if need_b else None
        gf = torch.empty_like(fa) if need_f else None
        a = nat.PRInterpArgs()
        a.pix_to_face, a.bary, a.face_attr = nat.ptr(p2f_c), nat.ptr(b_c), nat.ptr(fa)
        a.PK, a.D = p2f_c.numel(), fa.shape[-1]
        a.F = fc.shape[0] if fc is not None else fa.shape[0]
        a.faces, a.V = nat.ptr(fc), (fa.shape[0] if fc is not None else 0)
        a.grad_out, a.grad_bary, a.grad_face_attr = nat.ptr(go), nat.ptr(gb), nat.ptr(gf)
        nat.call("pr_interp_bwd", "pr_interp_bwd", go, a)
        return gb, gf, None, None


def interpolate_face_attributes(pix_to_face, barycentric_coords, face_attributes):
    """(N,H,W,K) p2f, (N,H,W,K,3) bary, (F,3,D) attrs -> (N,H,W,K,D)."""
    if face_attributes.dim() != 3 or face_attributes.shape[1] != 3:
        raise ValueError("face_attributes must be (F,3,D)")
    return _InterpFn.apply(barycentric_coords, face_attributes, pix_to_face, None)


def interpolate_vertex_attributes(pix_to_face, barycentric_coords, vert_attributes, faces_packed):
    """Same result as interpolate_face_attributes(p2f, bary, vert_attributes[faces]), gathering
    the (V,D) per-vertex table through (F,3) faces inside the kernel."""
    if vert_attributes.dim() != 2 or faces_packed.dim() != 2 or faces_packed.shape[1] != 3:
        raise ValueError("vert_attributes must be (V,D) and faces (F,3)")
    return _InterpFn.apply(barycentric_coords, vert_attributes, pix_to_face, faces_packed)
