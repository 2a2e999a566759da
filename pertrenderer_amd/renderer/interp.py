"""Barycentric interpolation of per-face-vertex attributes on the native kernels
(pr_interp_fwd / pr_interp_bwd): PyTorch3D interpolate_face_attributes semantics,
0 on padded slots (pix_to_face < 0)."""
import torch

from .. import _native as nat

F32 = torch.float32


class _InterpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, bary, face_attr, p2f):
        nat.require_device(bary, face_attr, p2f)
        lib = nat.load()
        shape = tuple(p2f.shape)
        D = face_attr.shape[-1]
        p2f_c = p2f.detach().to(torch.int64).contiguous()
        b_c = bary.detach().to(F32).contiguous()
        fa = face_attr.detach().to(F32).contiguous()
        out = torch.empty(shape + (D,), dtype=F32, device=b_c.device)
        a = nat.PRInterpArgs()
        a.pix_to_face, a.bary, a.face_attr = nat.ptr(p2f_c), nat.ptr(b_c), nat.ptr(fa)
        a.PK, a.F, a.D, a.out = p2f_c.numel(), fa.shape[0], D, nat.ptr(out)
        nat.check(lib.pr_interp_fwd(a, nat.stream_of(out)), "pr_interp_fwd")
        ctx.save_for_backward(b_c, fa, p2f_c)
        return out

    @staticmethod
    def backward(ctx, g):
        b_c, fa, p2f_c = ctx.saved_tensors
        lib = nat.load()
        need_b, need_f = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        go = g.detach().to(F32).contiguous()
        gb = torch.empty_like(b_c) if need_b else None
        gf = torch.empty_like(fa) if need_f else None
        a = nat.PRInterpArgs()
        a.pix_to_face, a.bary, a.face_attr = nat.ptr(p2f_c), nat.ptr(b_c), nat.ptr(fa)
        a.PK, a.F, a.D = p2f_c.numel(), fa.shape[0], fa.shape[-1]
        a.grad_out, a.grad_bary, a.grad_face_attr = nat.ptr(go), nat.ptr(gb), nat.ptr(gf)
        if need_b or need_f:
            nat.check(lib.pr_interp_bwd(a, nat.stream_of(go)), "pr_interp_bwd")
        return gb, gf, None


def interpolate_face_attributes(pix_to_face, barycentric_coords, face_attributes):
    """(N,H,W,K) p2f, (N,H,W,K,3) bary, (F,3,D) attrs -> (N,H,W,K,D)."""
    if face_attributes.dim() != 3 or face_attributes.shape[1] != 3:
        raise ValueError("face_attributes must be (F,3,D)")
    return _InterpFn.apply(barycentric_coords, face_attributes, pix_to_face)
