"""Non-Gaussian / non-variance-reduced perturbed operators.

ArctanRast (Cauchy Heaviside), GaussianRast_wovr, CauchyAgg, GaussianAgg_wovr.
These are the "next" rows beyond the Gaussian hot path: for now they are torch
tensor expressions of the reference's estimators (materialised noise, like the
reference) and run on whatever device the inputs live on.  The Gaussian
operators, which eval.py's benchmarked renderer uses, run on native kernels.

Noise draws follow the reference: Cauchy samples clamped to +-1e7
(smoothrast.py:22-24, smoothagg.py:25-27), Gaussian via torch.normal.
"""
import torch

F32 = torch.float32


def _noise(kind, shape, device):
    if kind == "gaussian":
        return torch.normal(mean=torch.zeros(shape, device=device), std=1.0)
    if kind == "cauchy":
        m = torch.distributions.cauchy.Cauchy(torch.tensor([0.0], device=device),
                                              torch.tensor([1.0], device=device))
        return torch.clamp(m.sample(shape).squeeze(-1), min=-1e7, max=1e7)
    raise NotImplementedError(f"noise type {kind!r} not implemented")


def _score(kind, e):
    """d/d eps of -log density: eps for Gaussian, 2 eps / (1 + eps^2) for Cauchy."""
    return e if kind == "gaussian" else (2 * e) / (1 + torch.square(e))


class _HeavisideVariant(torch.autograd.Function):
    """smoothrast.py:12-59 (vr=True) and :61-108 (vr=False)."""

    @staticmethod
    def forward(ctx, D, S, sigma, kind, vr):
        e = _noise(kind, (S,) + tuple(D.shape), D.device)
        one = torch.ones((), dtype=D.dtype, device=D.device)
        maps = torch.heaviside(D + sigma.to(D.device) * e, one)
        v = torch.heaviside(D, one)
        ctx.save_for_backward(maps, e, sigma, v)
        ctx.kind, ctx.vr = kind, vr
        return maps.mean(0)

    @staticmethod
    def backward(ctx, gP):
        maps, e, sigma, v = ctx.saved_tensors
        s = sigma.to(maps.device)
        base = (maps - v) if ctx.vr else maps
        gm = (base * _score(ctx.kind, e) / s).mean(0)
        gD = gm * gP
        return gD, None, gD.sum().reshape(()) if ctx.needs_input_grad[2] else None, None, None


def perturbed_heaviside_variant(dists, sigma, nb_samples, kind, variance_reduction=True):
    return _HeavisideVariant.apply(-dists, int(nb_samples), sigma, kind, variance_reduction)


class _ArgmaxVariant(torch.autograd.Function):
    """smoothagg.py:10-73 (vr=True) and :75-141 (vr=False)."""

    @staticmethod
    def forward(ctx, z, S, gamma, kind, vr, fixed_noise):
        if fixed_noise:
            torch.manual_seed(1)
        e = _noise(kind, (S,) + tuple(z.shape), z.device)
        zp = z + gamma.to(z.device) * e
        w = torch.zeros(zp.shape, device=z.device).scatter_(-1, torch.max(zp, -1, keepdim=True)[1], 1)
        v = torch.zeros(z.shape, device=z.device).scatter_(-1, torch.max(z, -1, keepdim=True)[1], 1)
        ctx.save_for_backward(w, e, gamma, v)
        ctx.kind, ctx.vr = kind, vr
        return w.mean(0)

    @staticmethod
    def backward(ctx, gW):
        w, e, gamma, v = ctx.saved_tensors
        g = gamma.to(w.device)
        diff = (w - v.unsqueeze(0)) if (ctx.vr or ctx.kind == "cauchy") else w
        a = (gW.unsqueeze(0) * diff).sum(-1, keepdim=True)
        sc = _score(ctx.kind, e)
        dz = (a * sc / g).mean(0)
        if ctx.kind == "gaussian":
            n = torch.square(torch.norm(e, dim=-1, keepdim=True))
        else:
            n = (sc * e).sum(-1, keepdim=True)
        gg = (gW.unsqueeze(0) * (diff * (n - 1.0) / g)).sum(dim=(1, 2, 3, 4)).mean(0)
        return dz, None, gg.reshape(()) if ctx.needs_input_grad[2] else None, None, None, None


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


def perturbed_aggregate_variant(zbuf, zfar, znear, prob_map, mask, gamma, alpha, nb_samples, eps,
                                kind, variance_reduction=True, fixed_noise=False):
    z = logits(zbuf, zfar, znear, prob_map, mask, gamma, alpha, eps)
    return _ArgmaxVariant.apply(z, int(nb_samples), gamma, kind, variance_reduction, fixed_noise)
