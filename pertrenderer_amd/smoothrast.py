"""Smooth rasterization operators — the reference's ``randomras.smoothrast`` surface.

Class names, constructor signatures, attributes (``sigma`` a CPU 0-d leaf with
requires_grad, ``nb_samples`` an int) and the ``update_*`` mutators mirror
smoothrast.py:111-194.  The Monte-Carlo operators (GaussianRast, ArctanRast =
Cauchy noise, GaussianRast_wovr = no variance reduction) run on the native kernels
(pr_heaviside_* with PR_BLEND_RAST_* variant flags); inside ``smooth_rgb_blend`` any
of them paired with a native aggregation operator is fused into one pr_blend launch.
The deterministic variants (SoftRast, AffineRast, HardRast) are elementwise torch
expressions, as in the reference.
"""
import torch
from torch.nn import Module

from . import blend as _blend


class _PerturbedRast:
    """rasterize() of the Monte-Carlo operators: the native perturbed Heaviside."""

    noise_kind = "gaussian"
    variance_reduction = True

    def rasterize(self, dists):
        return _blend.perturbed_heaviside(dists, self.sigma, self.nb_samples, kind=self.noise_kind,
                                          variance_reduction=self.variance_reduction)


class SmoothRastBase(Module):
    """smoothrast.py:111-123."""

    def __init__(self, sigma=2e-4):
        super().__init__()
        self.sigma = torch.tensor(sigma, requires_grad=True)
        self.nb_samples = 1

    def update_smoothing(self, sigma):
        self.sigma = torch.tensor(sigma, requires_grad=True)

    def update_nb_samples(self, nb_samples):
        self.nb_samples = nb_samples


class SoftRast(SmoothRastBase):
    """sigmoid(-d / sigma) (smoothrast.py:126-134)."""

    def __init__(self, sigma=2e-4):
        super().__init__(sigma)

    def rasterize(self, dists):
        return torch.sigmoid(-dists / self.sigma)


class GaussianRast(_PerturbedRast, SmoothRastBase):
    """Monte-Carlo perturbed Heaviside with Gaussian noise (smoothrast.py:136-147)."""

    noise_kind = "gaussian"
    variance_reduction = True

    def __init__(self, nb_samples=16, sigma=2e-4):
        super().__init__(sigma)
        self.nb_samples = nb_samples


class GaussianRast_wovr(_PerturbedRast, SmoothRastBase):
    """Gaussian perturbed Heaviside without variance reduction (smoothrast.py:149-160)."""

    noise_kind = "gaussian"
    variance_reduction = False

    def __init__(self, nb_samples=16, sigma=2e-4):
        super().__init__(sigma)
        self.nb_samples = nb_samples


class ArctanRast(_PerturbedRast, SmoothRastBase):
    """Cauchy-perturbed Heaviside (smoothrast.py:162-173)."""

    noise_kind = "cauchy"
    variance_reduction = True

    def __init__(self, nb_samples=16, sigma=2e-4):
        super().__init__(sigma)
        self.nb_samples = nb_samples


class AffineRast(SmoothRastBase):
    """Clamped affine ramp (smoothrast.py:175-185)."""

    def __init__(self, nb_samples=16, sigma=2e-4):
        super().__init__(sigma)
        self.nb_samples = nb_samples

    def rasterize(self, dists):
        x = -dists / self.sigma
        ramp = torch.where(x > 0.5, torch.ones_like(dists), x + 0.5)
        return torch.where(ramp < 0.0, torch.zeros_like(ramp), ramp)


class HardRast:
    """Hard inside test H(-d) (smoothrast.py:187-194)."""

    def __init__(self):
        return

    def rasterize(self, dists):
        return torch.heaviside(-dists, torch.ones((), dtype=dists.dtype, device=dists.device))
