"""SO(3) helpers and Rotate with PyTorch3D conventions (experiments/eval.py:49-55, 343-346,
428-430): row-vector rotation points @ R, so3_exponential_map = Rodrigues' formula.

On the GPU, so3_exponential_map and Rotate.transform_points run as single native
kernels (pr_so3_exp_*, pr_rotate_*: one launch per direction instead of the ~60
small kernels of the torch composition); CPU tensors use the torch formulas below.
"""
import math

import torch

from .. import _native as nat
from .. import host_layer

F32 = torch.float32


class _SO3ExpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, log_rot, eps):
        w = nat.dense(log_rot, F32)
        R = torch.empty((w.shape[0], 3, 3), dtype=F32, device=w.device)
        a = nat.PRSO3Args()
        a.N, a.eps, a.log_rot, a.R = w.shape[0], float(eps), nat.ptr(w), nat.ptr(R)
        nat.call("pr_so3_exp_fwd", "pr_so3_exp_fwd", R, a)
        ctx.save_for_backward(w)
        ctx.eps = eps
        return R

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gR):
        (w,) = ctx.saved_tensors
        g = nat.dense(gR, F32)
        gw = torch.empty_like(w)
        a = nat.PRSO3Args()
        a.N, a.eps, a.log_rot, a.grad_R, a.grad_log_rot = w.shape[0], float(ctx.eps), nat.ptr(w), nat.ptr(g), nat.ptr(gw)
        nat.call("pr_so3_exp_bwd", "pr_so3_exp_bwd", gw, a)
        return gw, None


class _RotateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, points, R):
        p = nat.dense(points, F32)
        r = nat.dense(R, F32)
        out = torch.empty_like(p)
        a = nat.PRRotateArgs()
        a.N, a.P, a.R_batched = p.shape[0], p.shape[1], int(r.shape[0] > 1)
        a.points, a.R, a.out = nat.ptr(p), nat.ptr(r), nat.ptr(out)
        nat.call("pr_rotate_fwd", "pr_rotate_fwd", out, a)
        ctx.save_for_backward(p, r)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gout):
        p, r = ctx.saved_tensors
        g = nat.dense(gout, F32)
        need_p, need_r = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        gp = torch.empty_like(p) if need_p else None
        gr = torch.empty_like(r) if need_r else None
        a = nat.PRRotateArgs()
        a.N, a.P, a.R_batched = p.shape[0], p.shape[1], int(r.shape[0] > 1)
        a.points, a.R, a.grad_out, a.grad_points, a.grad_R = nat.ptr(p), nat.ptr(r), nat.ptr(g), nat.ptr(gp), nat.ptr(gr)
        nat.call("pr_rotate_bwd", "pr_rotate_bwd", g, a)
        return gp, gr


def hat(v):
    N = v.shape[0]
    h = v.new_zeros(N, 3, 3)
    x, y, z = v.unbind(1)
    h[:, 0, 1], h[:, 0, 2] = -z, y
    h[:, 1, 0], h[:, 1, 2] = z, -x
    h[:, 2, 0], h[:, 2, 1] = -y, x
    return h


def so3_exponential_map(log_rot, eps=0.0001):
    if log_rot.is_cuda:
        ext = host_layer.get()
        return ext.so3_exp(log_rot, float(eps)) if ext is not None else _SO3ExpFn.apply(log_rot, eps)
    nrms = (log_rot * log_rot).sum(1)
    angles = torch.clamp(nrms, eps).sqrt()
    inv = 1.0 / angles
    fac1 = inv * angles.sin()
    fac2 = inv * inv * (1.0 - angles.cos())
    skews = hat(log_rot)
    skews2 = torch.bmm(skews, skews)
    eye = torch.eye(3, dtype=log_rot.dtype, device=log_rot.device)[None]
    return fac1[:, None, None] * skews + fac2[:, None, None] * skews2 + eye


so3_exp_map = so3_exponential_map


def so3_rotation_angle(R, eps=1e-4, cos_angle=False):
    tr = R[:, 0, 0] + R[:, 1, 1] + R[:, 2, 2]
    phi_cos = (tr - 1.0) * 0.5
    if cos_angle:
        return phi_cos
    return torch.acos(torch.clamp(phi_cos, -1.0 + eps, 1.0 - eps)) if eps > 0 else torch.acos(phi_cos)


def so3_relative_angle(R1, R2, cos_angle=False):
    return so3_rotation_angle(torch.bmm(R1, R2.permute(0, 2, 1)), cos_angle=cos_angle)


def so3_log_map(R, eps=0.0001):
    phi = so3_rotation_angle(R)
    phi_sin = phi.sin()
    phi_denom = torch.clamp(phi_sin.abs(), eps) * phi_sin.sign() + (phi_sin == 0).type_as(phi) * eps
    log_rot_hat = (phi / (2.0 * phi_denom))[:, None, None] * (R - R.permute(0, 2, 1))
    return torch.stack((log_rot_hat[:, 2, 1], log_rot_hat[:, 0, 2], log_rot_hat[:, 1, 0]), dim=1)


def random_quaternions(n, dtype=F32, device=None):
    o = torch.randn((n, 4), dtype=dtype, device=device)
    s = (o * o).sum(1)
    return o / torch.where(o[:, 0] < 0, -torch.sqrt(s), torch.sqrt(s))[:, None]


def quaternion_to_matrix(q):
    r, i, j, k = torch.unbind(q, -1)
    two_s = 2.0 / (q * q).sum(-1)
    o = torch.stack((1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
                     two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
                     two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)), -1)
    return o.reshape(q.shape[:-1] + (3, 3))


def random_rotations(n, dtype=F32, device=None):
    return quaternion_to_matrix(random_quaternions(n, dtype=dtype, device=device))


class Rotate:
    """points @ R (PyTorch3D Rotate)."""

    def __init__(self, R, device=None):
        self.R = R if R.dim() == 3 else R[None]

    def transform_points(self, points):
        pts = points if points.dim() == 3 else points[None]
        R = self.R.to(pts.device)
        if pts.is_cuda and R.shape[0] in (1, pts.shape[0]):
            ext = host_layer.get()
            out = ext.rotate(pts, R) if ext is not None else _RotateFn.apply(pts, R)
        else:
            out = torch.bmm(pts, R.expand(pts.shape[0], 3, 3))
        return out if points.dim() == 3 else out[0]

    def get_matrix(self):
        N = self.R.shape[0]
        M = torch.eye(4, dtype=self.R.dtype, device=self.R.device).repeat(N, 1, 1)
        M[:, :3, :3] = self.R
        return M
