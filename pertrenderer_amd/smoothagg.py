"""Smooth aggregation operators — the reference's ``randomras.smoothagg`` surface.

Mirrors smoothagg.py:145-289: ``gamma`` / ``alpha`` are CPU 0-d leaves with
requires_grad, ``nb_samples`` an int, ``eps`` the background logit weight.
The Monte-Carlo operators (GaussianAgg, CauchyAgg, GaussianAgg_wovr) run on the
native kernels (pr_blend without RAST/COLOR, PR_BLEND_AGG_* variant flags); inside
``smooth_rgb_blend`` they fuse with a native rasterization operator into one launch.
``log_corrected`` / ``prod_corrected`` keep the reference's inf/nan-safe
backward conventions (smoothagg.py:292-337).
"""
import torch
from torch.nn import Module

from . import blend as _blend
from . import variants as _variants
from .variants import log_corrected as _log_c, prod_corrected as _prod_c


class _PerturbedAgg:
    """aggregate() of the Monte-Carlo operators: the native perturbed argmax."""

    noise_kind = "gaussian"
    variance_reduction = True

    def aggregate(self, zbuf, zfar, znear, prob_map, mask):
        return _blend.perturbed_aggregate(zbuf, zfar, znear, prob_map, mask, self.gamma, self.alpha,
                                          self.nb_samples, eps=self.eps, fixed_noise=self.fixed_noise,
                                          kind=self.noise_kind, variance_reduction=self.variance_reduction)


class SmoothAggBase(Module):
    """smoothagg.py:145-163."""

    def __init__(self, gamma, alpha, eps, nb_samples=1):
        super().__init__()
        self.gamma = torch.tensor(gamma, requires_grad=True)
        self.alpha = torch.tensor(alpha, requires_grad=True)
        self.nb_samples = nb_samples
        self.eps = eps

    def update_smoothing(self, gamma=4e-2, alpha=1.0):
        self.gamma = torch.tensor(gamma, requires_grad=True)
        self.alpha = torch.tensor(alpha, requires_grad=True)

    def update_nb_samples(self, nb_samples):
        self.nb_samples = nb_samples


class SoftAgg(SmoothAggBase):
    """Deterministic softmax aggregation (SoftRas-style, smoothagg.py:165-182)."""

    def __init__(self, gamma=4e-2, alpha=1.0, eps=1e-10):
        super().__init__(gamma, alpha, eps)

    def aggregate(self, zbuf, zfar, znear, prob_map, mask):
        z = _variants.logits(zbuf, zfar, znear, prob_map, mask, self.gamma, self.alpha, self.eps)
        return torch.softmax(_prod_c(1.0 / self.gamma, z), dim=-1)


class GaussianAgg(_PerturbedAgg, SmoothAggBase):
    """Monte-Carlo perturbed argmax with Gaussian noise (smoothagg.py:185-205)."""

    noise_kind = "gaussian"
    variance_reduction = True

    def __init__(self, nb_samples=16, gamma=4e-2, alpha=1.0, eps=1e-10, fixed_noise=False):
        super().__init__(gamma, alpha, eps, nb_samples)
        self.fixed_noise = fixed_noise


class GaussianAgg_wovr(_PerturbedAgg, SmoothAggBase):
    """Gaussian perturbed argmax without variance reduction (smoothagg.py:207-227)."""

    noise_kind = "gaussian"
    variance_reduction = False

    def __init__(self, nb_samples=16, gamma=4e-2, alpha=1.0, eps=1e-10, fixed_noise=False):
        super().__init__(gamma, alpha, eps, nb_samples)
        self.fixed_noise = fixed_noise


class CauchyAgg(_PerturbedAgg, SmoothAggBase):
    """Cauchy-perturbed argmax (smoothagg.py:230-250)."""

    noise_kind = "cauchy"
    variance_reduction = True

    def __init__(self, nb_samples=16, gamma=4e-2, alpha=1.0, eps=1e-10, fixed_noise=False):
        super().__init__(gamma, alpha, eps, nb_samples)
        self.fixed_noise = fixed_noise


class UniformAgg(_PerturbedAgg, SmoothAggBase):
    """Uniform-noise perturbed argmax (smoothagg.py:252-271): the native forward with
    U(-1/2, 1/2) noise; like the reference (smoothagg.py:64-70), the backward raises."""

    noise_kind = "uniform"
    variance_reduction = True

    def __init__(self, nb_samples=16, gamma=4e-2, alpha=1.0, eps=1e-10, fixed_noise=False):
        self.fixed_noise = fixed_noise
        super().__init__(gamma, alpha, eps, nb_samples)


class HardAgg:
    """Hard z-buffer argmax (smoothagg.py:274-289)."""

    def __init__(self, eps=1e-10):
        self.eps = eps

    def aggregate(self, zbuf, zfar, znear, prob_map, mask):
        z = _variants.logits(zbuf, zfar, znear, prob_map, mask, None, None, self.eps, scale_log=1.0 / 1e6)
        idx = torch.max(z, dim=-1, keepdim=True)[1]
        return torch.zeros(z.shape, device=z.device).scatter_(-1, idx, 1)


log_corrected = _log_c
prod_corrected = _prod_c
