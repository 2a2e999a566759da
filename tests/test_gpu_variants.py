"""Native noise variants: ArctanRast (Cauchy), GaussianRast_wovr,
CauchyAgg, GaussianAgg_wovr — fused and standalone, against the reference's golden vectors
(injected noise) and the CPU oracle; Philox mode checked against closed forms."""
import math

import numpy as np
import pytest
import torch

from conftest import assert_close, load_golden
from oracle import blend_oracle as bo
import pertrenderer_amd as pa
from pertrenderer_amd import Noise, perturbed_aggregate, perturbed_blend, perturbed_heaviside

pytestmark = pytest.mark.gpu
VARIANT_CASES = ["var_arctan_cauchy", "var_wovr", "var_mixed"]


def _leaf(v):
    return torch.tensor(float(v), requires_grad=True)


@pytest.mark.parametrize("case", VARIANT_CASES)
def test_variant_fused_blend_matches_reference_golden(case, device):
    f = load_golden(case)
    d = torch.tensor(f["dists"], device=device, requires_grad=True)
    z = torch.tensor(f["zbuf"], device=device, requires_grad=True)
    c = torch.tensor(f["colors"], device=device, requires_grad=True)
    p2f = torch.tensor(f["pix_to_face"], device=device)
    s, g, a = _leaf(f["sigma"]), _leaf(f["gamma"]), _leaf(f["alpha"])
    N = p2f.shape[0]
    zn = torch.full((N, 1, 1, 1), float(f["znear"]), device=device)
    zf = torch.full((N, 1, 1, 1), float(f["zfar"]), device=device)
    noise = Noise.injected(torch.tensor(f["noise_r"], device=device), torch.tensor(f["noise_a"], device=device))
    img = perturbed_blend(c, p2f, d, z, s, g, a, int(f["Sr"]), int(f["Sa"]), eps=float(f["eps"]),
                          background=tuple(f["background"]), znear=zn, zfar=zf, noise=noise,
                          rast_kind=str(f["rast_kind"]), rast_vr=bool(f["rast_vr"]),
                          agg_kind=str(f["agg_kind"]), agg_vr=bool(f["agg_vr"]))
    (img * torch.tensor(f["grad_image"], device=device)).sum().backward()
    assert_close(img, f["image"], name="image")
    for k, t in (("dists", d), ("zbuf", z), ("colors", c)):
        assert_close(t.grad, f["grad_" + k], name=k)
    for k, t in (("sigma", s), ("gamma", g), ("alpha", a)):
        assert_close(t.grad, f["grad_" + k], rtol=2e-5, name=k)


@pytest.mark.parametrize("kind,vr", [("cauchy", True), ("gaussian", False), ("cauchy", False)])
def test_variant_heaviside_matches_oracle(kind, vr, device):
    gen = torch.Generator().manual_seed(2)
    D = (torch.rand((2, 5, 6, 9), generator=gen) - 0.5) * 6e-3
    S = 7
    e = torch.randn((S, 2, 5, 6, 9), generator=gen)
    if kind == "cauchy":
        e = torch.tan(math.pi * (torch.rand(e.shape, generator=gen) - 0.5))
    gP = torch.randn(D.shape, generator=gen)
    d = D.to(device).requires_grad_(True)
    sig = _leaf(1e-3)
    P = perturbed_heaviside(d, sig, S, noise=Noise.injected(e.to(device)), kind=kind, variance_reduction=vr)
    (P * gP.to(device)).sum().backward()
    oP, odd, ods = bo.rasterize_forward_backward(D, e, torch.tensor(1e-3), gP, kind, vr)
    np.testing.assert_array_equal(P.detach().cpu().numpy(), oP.numpy())
    assert_close(d.grad, odd, name="dists")
    # d sigma sums 7 x 540 signed terms (Cauchy: heavy cancellation) in another order than the
    # oracle's torch.sum: measured 2.2e-5 relative, bar 5e-5 as for every smoothing-scalar reduction
    assert_close(sig.grad, ods, rtol=5e-5, name="sigma")


@pytest.mark.parametrize("kind,vr", [("cauchy", True), ("gaussian", False)])
def test_variant_aggregate_matches_oracle(kind, vr, device):
    gen = torch.Generator().manual_seed(3)
    N, H, W, K, S = 2, 4, 5, 8, 6
    zbuf = 5.0 + torch.rand((N, H, W, K), generator=gen).sort(-1).values
    prob = torch.rand((N, H, W, K), generator=gen)
    mask = torch.rand((N, H, W, K), generator=gen) < 0.8
    prob = prob * mask
    e = torch.randn((S, N, H, W, K + 1), generator=gen)
    if kind == "cauchy":
        e = torch.tan(math.pi * (torch.rand(e.shape, generator=gen) - 0.5))
    gW = torch.randn((N, H, W, K + 1), generator=gen)
    zn, zf = torch.full((N, 1, 1, 1), 1.0), torch.full((N, 1, 1, 1), 100.0)
    z = zbuf.to(device).requires_grad_(True)
    pr = prob.to(device).requires_grad_(True)
    g, a = _leaf(1e-2), _leaf(1.0)
    Wt = perturbed_aggregate(z, zf.to(device), zn.to(device), pr, mask.to(device), g, a, S,
                             noise=Noise.injected(noise_a=e.to(device)), kind=kind, variance_reduction=vr)
    (Wt * gW.to(device)).sum().backward()
    oW, odz, odp, odg, oda = bo.aggregate_forward_backward(zbuf, zf, zn, prob, mask, e, torch.tensor(1e-2),
                                                           torch.tensor(1.0), 1e-10, gW, kind, vr)
    np.testing.assert_array_equal(Wt.detach().cpu().numpy(), oW.numpy())
    assert_close(z.grad, odz, name="zbuf")
    assert_close(pr.grad, odp, name="prob")
    assert_close(g.grad, odg, name="gamma")
    assert_close(a.grad, oda, name="alpha")


def test_philox_cauchy_heaviside_closed_form(device):
    """ArctanRast in Philox mode: E[P] = 1/2 + atan(D/sigma)/pi, and the (variance-reduced)
    score estimator is unbiased for dP/dD = 1 / (pi sigma (1 + (D/sigma)^2))."""
    sigma, S, reps = 1.0, 256, 256
    Dv = torch.linspace(-3.0, 3.0, 13)
    d = (-Dv).reshape(1, 1, 1, -1).repeat(1, reps, 1, 1).to(device).requires_grad_(True)
    P = perturbed_heaviside(d, torch.tensor(sigma), S, noise=Noise.philox(seed_r=11), kind="cauchy")
    P.sum().backward()
    est_p = P.detach().mean(dim=(0, 1, 2)).cpu().double()
    est_g = -d.grad.mean(dim=(0, 1, 2)).cpu().double()
    cdf = 0.5 + torch.atan(Dv.double() / sigma) / math.pi
    pdf = 1.0 / (math.pi * sigma * (1 + (Dv.double() / sigma) ** 2))
    n = S * reps
    assert torch.all((est_p - cdf).abs() <= 5 * torch.sqrt(cdf * (1 - cdf) / n) + 1e-3), (est_p, cdf)
    assert torch.all((est_g - pdf).abs() <= 0.02), (est_g, pdf)


def test_philox_wovr_heaviside_is_unbiased(device):
    """GaussianRast_wovr: same expectation as the variance-reduced estimator, phi(D/s)/s."""
    sigma, S, reps = 1.0, 256, 512
    Dv = torch.linspace(-2.0, 2.0, 9)
    d = (-Dv).reshape(1, 1, 1, -1).repeat(1, reps, 1, 1).to(device).requires_grad_(True)
    P = perturbed_heaviside(d, torch.tensor(sigma), S, noise=Noise.philox(seed_r=12), variance_reduction=False)
    P.sum().backward()
    est_g = -d.grad.mean(dim=(0, 1, 2)).cpu().double()
    phi = torch.exp(-0.5 * Dv.double() ** 2) / math.sqrt(2 * math.pi)
    assert torch.all((est_g - phi / sigma).abs() <= 0.03), (est_g, phi)


def test_philox_cauchy_argmax_frequencies(device):
    N, reps, K = 1, 4096, 2
    zbuf = torch.tensor([5.0, 5.02]).reshape(1, 1, 1, 2).repeat(1, reps, 1, 1).to(device)
    prob = torch.ones_like(zbuf) * 0.5
    mask = torch.ones_like(zbuf, dtype=torch.bool)
    W = perturbed_aggregate(zbuf, 100.0, 1.0, prob, mask, torch.tensor(1e-2), torch.tensor(1.0), 16,
                            noise=Noise.philox(seed_a=13), kind="cauchy")
    w = W.mean(dim=(0, 1, 2)).cpu().double()
    z_inv = (100.0 - np.array([5.0, 5.02])) / 99.0
    zk = 1e-2 * np.log(0.5) + z_inv - z_inv.max()
    z = np.concatenate([zk, [1e-10 - z_inv.max()]])
    e = np.random.default_rng(0).standard_cauchy((400000, 3))
    ref = np.bincount(np.argmax(z + 1e-2 * e, axis=1), minlength=3) / 400000.0
    assert np.all(np.abs(w.numpy() - ref) < 0.01), (w, ref)


def test_shader_fuses_variant_pairs(device):
    """RandomSimpleShader with ArctanRast + CauchyAgg takes the fused native path and
    matches the standalone composition rasterize -> aggregate -> colour mix (injected)."""
    from pertrenderer_amd.random_rasterizer import _is_fusable
    from pertrenderer_amd.renderer.rasterizer import Fragments
    p2f = torch.zeros((1, 2, 2, 3), dtype=torch.int64, device=device)
    fr = Fragments(p2f, p2f.float(), None, p2f.float())
    assert _is_fusable(pa.ArctanRast(), pa.CauchyAgg(), fr)
    assert _is_fusable(pa.GaussianRast_wovr(), pa.GaussianAgg_wovr(), fr)
    assert not _is_fusable(pa.SoftRast(), pa.CauchyAgg(), fr)
