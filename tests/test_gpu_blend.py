"""GPU parity of the native perturbed blend against the reference (golden vectors) and
the CPU oracle.  Injected-noise mode is compared element-wise at the 1e-5 relative
fp32 bar; Philox mode is compared with the numpy Philox restatement (counts are
integers: bit-exact) and checked statistically."""
import math

import numpy as np
import pytest
import torch

from conftest import assert_close, load_golden
from oracle import blend_oracle as bo
from oracle import philox_ref
from pertrenderer_amd import Noise, perturbed_aggregate, perturbed_blend, perturbed_heaviside
from pertrenderer_amd.renderer.rasterizer import attach_valid_counts

pytestmark = pytest.mark.gpu
BLEND_CASES = ["blend_small", "blend_eval", "blend_edge", "blend_fixed", "blend_k100"]
SCALAR_RTOL = 2e-5


def _leaf(v):
    return torch.tensor(float(v), requires_grad=True)


def _run_fused(f, dev, noise=None, counts=False):
    d = torch.tensor(f["dists"], device=dev, requires_grad=True)
    z = torch.tensor(f["zbuf"], device=dev, requires_grad=True)
    c = torch.tensor(f["colors"], device=dev, requires_grad=True)
    p2f = torch.tensor(f["pix_to_face"], device=dev)
    if counts:  # the rasterizer's valid-prefix counts (packed fragments only)
        attach_valid_counts(p2f, (p2f >= 0).sum(-1).to(torch.int32))
    s, g, a = _leaf(f["sigma"]), _leaf(f["gamma"]), _leaf(f["alpha"])
    N = p2f.shape[0]
    zn = torch.full((N, 1, 1, 1), float(f["znear"]), device=dev)
    zf = torch.full((N, 1, 1, 1), float(f["zfar"]), device=dev)
    if noise is None:
        noise = Noise.injected(torch.tensor(f["noise_r"], device=dev), torch.tensor(f["noise_a"], device=dev))
    img = perturbed_blend(c, p2f, d, z, s, g, a, int(f["Sr"]), int(f["Sa"]), eps=float(f["eps"]),
                          background=tuple(f["background"]), znear=zn, zfar=zf, noise=noise)
    (img * torch.tensor(f["grad_image"], device=dev)).sum().backward()
    return img, dict(dists=d.grad, zbuf=z.grad, colors=c.grad, sigma=s.grad, gamma=g.grad, alpha=a.grad)


@pytest.mark.parametrize("case", BLEND_CASES)
def test_fused_blend_matches_reference_golden(case, device):
    f = load_golden(case)
    img, g = _run_fused(f, device)
    assert_close(img, f["image"], name="image")
    for k in ("dists", "zbuf", "colors"):
        assert_close(g[k], f["grad_" + k], name=k)
    for k in ("sigma", "gamma", "alpha"):
        assert g[k].device.type == "cpu" and g[k].dim() == 0
        assert_close(g[k], f["grad_" + k], rtol=SCALAR_RTOL, name=k)


def test_standalone_rasterize_matches_reference_golden(device):
    f = load_golden("rast_only")
    d = torch.tensor(f["dists"], device=device, requires_grad=True)
    s = _leaf(f["sigma"])
    P = perturbed_heaviside(d, s, int(f["Sr"]), noise=Noise.injected(torch.tensor(f["noise_r"], device=device)))
    (P * torch.tensor(f["grad_P"], device=device)).sum().backward()
    np.testing.assert_array_equal(P.detach().cpu().numpy(), f["P"])
    assert_close(d.grad, f["grad_dists"], name="dists")
    assert_close(s.grad, f["grad_sigma"], rtol=SCALAR_RTOL, name="sigma")


def test_standalone_aggregate_matches_reference_golden(device):
    f = load_golden("agg_only")
    z = torch.tensor(f["zbuf"], device=device, requires_grad=True)
    pr = torch.tensor(f["prob"], device=device, requires_grad=True)
    mask = torch.tensor(f["pix_to_face"], device=device) >= 0
    g, a = _leaf(f["gamma"]), _leaf(f["alpha"])
    N = z.shape[0]
    W = perturbed_aggregate(z, torch.full((N, 1, 1, 1), float(f["zfar"]), device=device),
                            torch.full((N, 1, 1, 1), float(f["znear"]), device=device), pr, mask, g, a,
                            int(f["Sa"]), eps=float(f["eps"]),
                            noise=Noise.injected(noise_a=torch.tensor(f["noise_a"], device=device)))
    (W * torch.tensor(f["grad_W"], device=device)).sum().backward()
    np.testing.assert_array_equal(W.detach().cpu().numpy(), f["W"])
    assert_close(z.grad, f["grad_zbuf"], name="zbuf")
    assert_close(pr.grad, f["grad_prob"], name="prob")
    assert_close(g.grad, f["grad_gamma"], rtol=SCALAR_RTOL, name="gamma")
    assert_close(a.grad, f["grad_alpha"], rtol=SCALAR_RTOL, name="alpha")


def _synthetic(N, H, W, K, Sr, Sa, seed, sigma=1e-3, p_valid=0.6, packed=True):
    g = torch.Generator().manual_seed(seed)
    valid = torch.rand((N, H, W, K), generator=g) < p_valid
    if packed:
        cnt = valid.sum(-1, keepdim=True)
        valid = torch.arange(K).expand(N, H, W, K) < cnt
    p2f = torch.where(valid, torch.randint(0, 5000, (N, H, W, K), generator=g), torch.full((N, H, W, K), -1))
    dists = torch.where(valid, (torch.rand((N, H, W, K), generator=g) - 0.5) * 6 * sigma, torch.full((N, H, W, K), -1.0))
    zbuf = torch.where(valid, 5.0 + torch.rand((N, H, W, K), generator=g), torch.full((N, H, W, K), -1.0))
    colors = torch.rand((N, H, W, K, 3), generator=g)
    f = dict(pix_to_face=p2f.numpy(), dists=dists.numpy(), zbuf=zbuf.numpy(), colors=colors.numpy(),
             sigma=np.float32(sigma), gamma=np.float32(1e-2), alpha=np.float32(1.0), eps=1e-10,
             background=np.array([0.1, 0.2, 0.3], np.float32), znear=1.0, zfar=100.0, Sr=Sr, Sa=Sa)
    f["noise_r"] = torch.randn((Sr, N, H, W, K), generator=g).numpy()
    f["noise_a"] = torch.randn((Sa, N, H, W, K + 1), generator=g).numpy()
    f["grad_image"] = torch.randn((N, H, W, 4), generator=g).numpy()
    return f


def _oracle(f):
    T = lambda a: torch.from_numpy(np.asarray(a))
    N = f["pix_to_face"].shape[0]
    zn, zf = torch.full((N, 1, 1, 1), float(f["znear"])), torch.full((N, 1, 1, 1), float(f["zfar"]))
    img, s = bo.blend_forward(T(f["pix_to_face"]), T(f["dists"]), T(f["zbuf"]), T(f["colors"]), T(f["noise_r"]),
                              T(f["noise_a"]), T(f["sigma"]), T(f["gamma"]), T(f["alpha"]), float(f["eps"]),
                              T(f["background"]), zn, zf)
    return img, bo.blend_backward(T(f["grad_image"]), s), s


@pytest.mark.parametrize("counts", [False, True])
@pytest.mark.parametrize("shape", [(2, 16, 20, 50, 8, 8), (1, 8, 8, 150, 16, 4), (1, 12, 9, 7, 3, 5),
                                   (1, 4, 4, 255, 4, 4)])
def test_fused_blend_matches_oracle_random(shape, counts, device):
    """counts=True: the rasterizer's valid-prefix counts are attached, so the kernels walk
    valid slots only and fill masked slots' gradients without reading them."""
    N, H, W, K, Sr, Sa = shape
    if counts and K == 7:
        pytest.skip("scattered valid slots: no valid prefix")
    f = _synthetic(N, H, W, K, Sr, Sa, seed=sum(shape), packed=K != 7)
    img, g = _run_fused(f, device, counts=counts)
    oimg, og, saved = _oracle(f)
    # the Monte-Carlo weights are counts / Sa: exact, so the image matches to fp32 summation order
    assert_close(img, oimg, name="image")
    for k in ("dists", "zbuf", "colors"):
        assert_close(g[k], og[k], name=k)
    for k in ("sigma", "gamma", "alpha"):
        assert_close(g[k], og[k], rtol=1e-4, atol_rel=0, name=k)


def test_empty_and_fully_masked_pixels(device):
    f = _synthetic(1, 4, 4, 6, 4, 4, seed=3, p_valid=0.0)
    img, g = _run_fused(f, device)
    bg = f["background"]
    np.testing.assert_allclose(img[..., :3].detach().cpu().numpy(), np.broadcast_to(bg, (1, 4, 4, 3)), rtol=0)
    np.testing.assert_array_equal(img[..., 3].detach().cpu().numpy(), 0.0)
    assert torch.all(g["dists"] == 0) and torch.all(g["zbuf"] == 0) and torch.all(g["colors"] == 0)


# ------------------------------------------------------------------ Philox mode
def test_philox_heaviside_counts_match_numpy_stream(device):
    N, H, W, K, S = 1, 6, 7, 9, 12
    g = torch.Generator().manual_seed(0)
    sigma = 1e-3
    d = ((torch.rand((N, H, W, K), generator=g) - 0.5) * 4 * sigma)
    seed = 0x1234_5678_9ABC
    P = perturbed_heaviside(d.to(device), torch.tensor(sigma), S, noise=Noise.philox(seed_r=seed)).cpu().numpy()
    e = philox_ref.rast_normals(seed, N * H * W, K, S).reshape((S, N, H, W, K))
    cnt = ((-d.numpy().astype(np.float64))[None] + sigma * e >= 0).sum(0)
    ref = (cnt.astype(np.float32) / np.float32(S))
    mismatch = (P != ref).mean()
    assert mismatch < 2e-3, mismatch  # only samples within a few ulp of the threshold may differ


def test_philox_score_matches_numpy_stream(device):
    """d dists of the standalone Heaviside vs the numpy Box-Muller stream (score form)."""
    N, H, W, K, S = 1, 5, 6, 7, 8
    g = torch.Generator().manual_seed(1)
    sigma = 1e-3
    d = ((torch.rand((N, H, W, K), generator=g) - 0.5) * 6 * sigma).to(device).requires_grad_(True)
    gP = torch.randn((N, H, W, K), generator=g)
    seed = 99
    P = perturbed_heaviside(d, torch.tensor(sigma), S, noise=Noise.philox(seed_r=seed))
    (P * gP.to(device)).sum().backward()
    e = philox_ref.rast_normals(seed, N * H * W, K, S).reshape((S, N, H, W, K))
    D = -d.detach().cpu().numpy().astype(np.float64)
    m = (D[None] + sigma * e >= 0).astype(np.float64)
    vr = (D >= 0).astype(np.float64)
    gm = ((m - vr[None]) * e).mean(0) / sigma
    ref = -gm * gP.numpy()
    got = d.grad.cpu().numpy()
    close = np.isclose(got, ref, rtol=1e-4, atol=1e-2)
    assert close.mean() > 0.995, close.mean()


def test_philox_sharding_is_additive(device):
    """Disjoint sample ranges partition the estimator: (P[0:4] + P[4:8]) / 2 == P[0:8]."""
    d = ((torch.rand((1, 8, 8, 20), generator=torch.Generator().manual_seed(1)) - 0.5) * 4e-3).to(device)
    s = torch.tensor(1e-3)
    full = perturbed_heaviside(d, s, 8, noise=Noise.philox(seed_r=77))
    a = perturbed_heaviside(d, s, 4, noise=Noise.philox(seed_r=77, offset_r=0))
    b = perturbed_heaviside(d, s, 4, noise=Noise.philox(seed_r=77, offset_r=4))
    torch.testing.assert_close((a + b) / 2, full, rtol=0, atol=0)


def test_philox_heaviside_is_unbiased(device):
    """E[P] = Phi(D/sigma) and E[dP/dD estimate] = phi(D/sigma)/sigma (smoothrast.py:46,53)."""
    sigma = 1.0
    Dv = torch.linspace(-2.0, 2.0, 9)
    S = 256
    reps = 256
    d = (-Dv).reshape(1, 1, 1, -1).repeat(1, reps, 1, 1).to(device).requires_grad_(True)
    P = perturbed_heaviside(d, torch.tensor(sigma), S, noise=Noise.philox(seed_r=2024))
    P.sum().backward()
    est_p = P.detach().mean(dim=(0, 1, 2)).cpu().double()
    est_g = -d.grad.mean(dim=(0, 1, 2)).cpu().double()
    phi = torch.exp(-0.5 * Dv.double() ** 2) / math.sqrt(2 * math.pi)
    Phi = 0.5 * torch.erfc(-Dv.double() / math.sqrt(2))
    n = S * reps
    assert torch.all((est_p - Phi).abs() <= 5 * torch.sqrt(Phi * (1 - Phi) / n) + 1e-3)
    assert torch.all((est_g - phi / sigma).abs() <= 0.02), (est_g, phi)


def test_philox_argmax_frequencies(device):
    """Perturbed-argmax weights converge to P(argmax_j z_j + gamma*eps_j) (Gaussian, 3 logits)."""
    N, reps, K = 1, 4096, 2
    zbuf = torch.tensor([5.0, 5.02]).reshape(1, 1, 1, 2).repeat(1, reps, 1, 1).to(device)
    prob = torch.ones_like(zbuf) * 0.5
    mask = torch.ones_like(zbuf, dtype=torch.bool)
    gamma = torch.tensor(1e-2)
    W = perturbed_aggregate(zbuf, 100.0, 1.0, prob, mask, gamma, torch.tensor(1.0), 16, noise=Noise.philox(seed_a=9))
    w = W.mean(dim=(0, 1, 2)).cpu().double()
    # Monte-Carlo reference probabilities with numpy normals
    z_inv = (100.0 - np.array([5.0, 5.02])) / 99.0
    zk = 1e-2 * np.log(0.5) + z_inv - z_inv.max()
    z = np.concatenate([zk, [1e-10 - z_inv.max()]])
    rng = np.random.default_rng(0)
    e = rng.standard_normal((400000, 3))
    ref = np.bincount(np.argmax(z + 1e-2 * e, axis=1), minlength=3) / 400000.0
    assert np.all(np.abs(w.numpy() - ref) < 0.01), (w, ref)


def test_philox_is_deterministic_per_seed(device):
    f = _synthetic(1, 8, 8, 20, 8, 8, seed=5)
    n = Noise.philox(seed_r=11, seed_a=12)
    i1, g1 = _run_fused(f, device, noise=n)
    i2, g2 = _run_fused(f, device, noise=n)
    assert torch.equal(i1, i2)
    for k in ("dists", "zbuf", "colors"):
        assert torch.equal(g1[k], g2[k])


def test_philox_masked_tail_draw_matches_per_slot_draws(device):
    """With valid-prefix counts the backward draws a pixel's masked agg slots jointly
    (pr_blend.hip tail_pair: Sum eps = sqrt(m) Z, Sum eps^2 = Z^2 + chi2(m-1)) instead of
    one normal per (slot, sample).  Every gradient that sees per-slot noise matches the
    per-slot path (to fp32 summation order); d zbuf at each pixel's nearest slot (it carries d z_max) and
    d gamma (Sum eps^2) are equal in distribution: means and variances agree across
    pixels and seeds."""
    f = _synthetic(1, 64, 64, 60, 8, 64, seed=21, p_valid=0.1)
    valid = f["pix_to_face"] >= 0
    km = np.where(valid, -f["zbuf"], -np.inf).argmax(-1)[..., None]  # first max of z_inv
    xs, ys, gx, gy = [], [], [], []
    for seed in range(12):
        n = Noise.philox(seed_r=1000 + seed, seed_a=2000 + seed)
        ix, x = _run_fused(f, device, noise=n, counts=True)
        iy, y = _run_fused(f, device, noise=n)
        assert torch.equal(ix, iy)
        assert torch.equal(x["colors"], y["colors"])
        # per-slot d z sums may be split over a different number of lanes (fewer B6 rows):
        # fp32 summation order
        assert_close(x["dists"], y["dists"], rtol=1e-5, name="dists")
        zx, zy = x["zbuf"].cpu().numpy(), y["zbuf"].cpu().numpy()
        other = np.ones_like(valid)
        np.put_along_axis(other, km, False, -1)
        np.testing.assert_allclose(zx[other], zy[other], rtol=1e-5, atol=1e-6 * np.abs(zy).max())
        px, py = np.take_along_axis(zx, km, -1), np.take_along_axis(zy, km, -1)
        sel = valid.any(-1, keepdims=True) & (px != 0)  # pixels whose d z_max is live
        xs.append(px[sel]), ys.append(py[sel])
        gx.append(float(x["gamma"])), gy.append(float(y["gamma"]))
    xs, ys = np.concatenate(xs).astype(np.float64), np.concatenate(ys).astype(np.float64)
    assert xs.size > 5000, xs.size
    se = np.sqrt(xs.var() / xs.size + ys.var() / ys.size)
    assert abs(xs.mean() - ys.mean()) < 5 * se, (xs.mean(), ys.mean(), se)
    assert 0.85 < xs.var() / ys.var() < 1.15, (xs.var(), ys.var())
    gx, gy = np.array(gx), np.array(gy)
    se = np.sqrt(gx.var(ddof=1) / gx.size + gy.var(ddof=1) / gy.size)
    assert abs(gx.mean() - gy.mean()) < 5 * se, (gx, gy)
    assert 0.15 < gx.var() / gy.var() < 7.0, (gx, gy)


@pytest.mark.parametrize("mode", ["philox", "injected"])
def test_rast_cache_is_bit_identical(mode, device):
    """The forward's (prob, score) cache and the backward's regeneration agree bitwise."""
    import pertrenderer_amd.blend as pb
    f = _synthetic(2, 9, 11, 30, 8, 8, seed=17)
    noise = Noise.philox(seed_r=5, seed_a=6) if mode == "philox" else None
    old = pb.RAST_CACHE
    try:
        pb.RAST_CACHE = True
        i1, g1 = _run_fused(f, device, noise=noise)
        pb.RAST_CACHE = False
        i2, g2 = _run_fused(f, device, noise=noise)
    finally:
        pb.RAST_CACHE = old
    assert torch.equal(i1, i2)
    for k in ("dists", "zbuf", "colors", "sigma", "gamma", "alpha"):
        assert torch.equal(g1[k], g2[k]), k
