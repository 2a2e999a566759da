"""Deterministic helpers of the aggregation operators (smoothagg.py:197-202,292-337):
log_corrected / prod_corrected with the reference's inf/nan-safe backward and the
logit assembly used by SoftAgg / HardAgg.  The Monte-Carlo operators (Gaussian,
Cauchy, with and without variance reduction) run on the native kernels (blend.py).
"""
import torch

F32 = torch.float32


class _LogC(torch.autograd.Function):
    """log with backward 1/x (inf -> 0), smoothagg.py:292-311."""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return x.log()

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        r = torch.ones_like(x) / x
        return torch.where(torch.isinf(r), torch.zeros_like(r), r) * g


class _ProdC(torch.autograd.Function):
    """x*y with inf-safe / nan-safe backward, smoothagg.py:314-337."""

    @staticmethod
    def forward(ctx, x, y):
        ctx.save_for_backward(x, y)
        return x * y

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        dx = dy = None
        if ctx.needs_input_grad[0]:
            dx = (torch.where(torch.isinf(y), torch.zeros_like(y), y) * g).nansum()
            dx = dx.to(x.device) if torch.is_tensor(x) else dx
        if ctx.needs_input_grad[1]:
            dy = x.to(g.device) * g if torch.is_tensor(x) else x * g
            dy = torch.where(torch.isnan(dy), torch.zeros_like(dy), dy)
        return dx, dy


class _ProdLast(torch.autograd.Function):
    """torch.prod(x, dim=-1) with torch's own backward values (grad * result / x when the
    tensor holds no zero, else the exclusive-cumprod form of prod_safe_zeros_backward) chosen
    on the device: torch's prod backward reads the zero count on the host (.item()), which a
    captured graph cannot do."""

    @staticmethod
    def forward(ctx, x):
        out = torch.prod(x, dim=-1)
        ctx.save_for_backward(x, out)
        return out

    @staticmethod
    def backward(ctx, g):
        x, out = ctx.saved_tensors
        g, out = g.unsqueeze(-1), out.unsqueeze(-1)
        plain = g * (out / x)
        ones = torch.ones_like(x[..., :1])
        excl_fwd = torch.cat([ones, x[..., :-1]], dim=-1).cumprod(-1)
        excl_rev = torch.cat([ones, x[..., 1:].flip(-1)], dim=-1).cumprod(-1).flip(-1)
        safe = g * (excl_fwd * excl_rev)
        return torch.where((x == 0).sum() == 0, plain, safe)


def prod_last(x):
    return _ProdLast.apply(x)


def log_corrected(x):
    return _LogC.apply(x)


def prod_corrected(x, y):
    return _ProdC.apply(x, y)


def logits(zbuf, zfar, znear, prob_map, mask, gamma, alpha, eps, scale_log=None):
    """Logit assembly of smoothagg.py:197-202 (K -> K+1 with the background logit)."""
    z_inv = (zfar - zbuf) / (zfar - znear) * mask
    zmax = torch.max(z_inv, dim=-1).values[..., None].clamp(min=eps)
    if scale_log is None:
        zk = prod_corrected(gamma / alpha, log_corrected(prob_map)) + z_inv - zmax
    else:
        zk = scale_log * log_corrected(prob_map) + z_inv - zmax
    bgz = torch.ones(zk.shape[:-1] + (1,), device=zk.device) * eps - zmax
    return torch.cat((zk, bgz), dim=-1)
