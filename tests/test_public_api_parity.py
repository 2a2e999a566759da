"""Seeded parity through the PUBLIC plugin surface (what eval.py and the README call), not the
internal ops: the reference's golden vectors (tests/golden/gen_golden.py) were produced by
  torch.manual_seed(seed); randomras.smooth_rgb_blend(colors, fragments, GaussianRast(...),
  GaussianAgg(...), BlendParams(...), znear, zfar)      (random_rasterizer.py:34-56)
with the reference drawing eps_r (smoothrast.py:21) then eps_a (smoothagg.py:21) from the
global CPU generator.  Here the same call goes through pertrenderer_amd's classes with
``set_noise_source("torch")`` and the same seed: the native kernels consume exactly the
reference's draws, so outputs and every gradient (including the CPU 0-d sigma / gamma / alpha
leaves) must match at the 1e-5 relative fp32 bar.

The deterministic SoftRast + SoftAgg pair (eval.py's default "softras" renderer) is pure torch in
both code bases and is checked on the CPU as well as on the GPU.
"""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import pertrenderer_amd as pa
from conftest import assert_close, load_golden
from pertrenderer_amd.random_rasterizer import BlendParams, smooth_rgb_blend
from pertrenderer_amd.renderer.rasterizer import Fragments

BLEND_CASES = ["blend_small", "blend_eval", "blend_edge", "blend_fixed", "blend_k100"]
VARIANT_CASES = ["var_arctan_cauchy", "var_wovr", "var_mixed"]
SCALAR_RTOL = 2e-5


@pytest.fixture
def torch_noise():
    old = pa.noise.get_noise_source()
    pa.set_noise_source("torch")
    yield
    pa.set_noise_source(old)


def _fragments(f, dev, grad=True):
    d = torch.tensor(f["dists"], device=dev, requires_grad=grad)
    z = torch.tensor(f["zbuf"], device=dev, requires_grad=grad)
    p2f = torch.tensor(f["pix_to_face"], device=dev)
    bary = torch.zeros(tuple(p2f.shape) + (3,), device=dev)  # not read by the blend
    return Fragments(p2f, z, bary, d), d, z


def _planes(f, N, dev):
    return (torch.full((N, 1, 1, 1), float(f["znear"]), device=dev),
            torch.full((N, 1, 1, 1), float(f["zfar"]), device=dev))


def _check(f, img, d, z, c, rast, agg, cauchy_gamma=False):
    assert_close(img, f["image"], name="image")
    assert_close(d.grad, f["grad_dists"], name="dists")
    assert_close(z.grad, f["grad_zbuf"], name="zbuf")
    assert_close(c.grad, f["grad_colors"], name="colors")
    for name, leaf in (("sigma", rast.sigma), ("gamma", agg.gamma), ("alpha", agg.alpha)):
        assert leaf.grad is not None and leaf.grad.device.type == "cpu" and leaf.grad.dim() == 0, name
        assert_close(leaf.grad, f["grad_" + name], rtol=SCALAR_RTOL, name=name)


def _blend_through_api(f, dev, rast, agg, use_shader=False):
    fr, d, z = _fragments(f, dev)
    c = torch.tensor(f["colors"], device=dev, requires_grad=True)
    N = fr.pix_to_face.shape[0]
    zn, zf = _planes(f, N, dev)
    bp = BlendParams(float(f["sigma"]), float(f["gamma"]), tuple(float(v) for v in f["background"]))
    torch.manual_seed(int(f["seed"]))
    if use_shader:
        # a RandomSimpleShader over a mesh whose sample_textures() returns the fixture's texels
        # (random_rasterizer.py:164-177); the camera supplies znear / zfar as (N,) tensors
        cams = SimpleNamespace(znear=zn.reshape(N), zfar=zf.reshape(N))
        mesh = SimpleNamespace(sample_textures=lambda fragments: c)
        shader = pa.RandomSimpleShader(device=dev, cameras=cams, smoothrast=rast, smoothagg=agg, blend_params=bp)
        img = shader(fr, mesh)
    else:
        img = smooth_rgb_blend(c, fr, rast, agg, bp, znear=zn, zfar=zf)
    (img * torch.tensor(f["grad_image"], device=dev)).sum().backward()
    return img, d, z, c


@pytest.mark.gpu
@pytest.mark.parametrize("case", BLEND_CASES)
@pytest.mark.parametrize("entry", ["smooth_rgb_blend", "RandomSimpleShader"])
def test_seeded_gaussian_pair_matches_reference(case, entry, device, torch_noise):
    f = load_golden(case)
    rast = pa.GaussianRast(nb_samples=int(f["Sr"]), sigma=float(f["sigma"]))
    agg = pa.GaussianAgg(nb_samples=int(f["Sa"]), gamma=float(f["gamma"]), alpha=float(f["alpha"]),
                         eps=float(f["eps"]), fixed_noise=bool(f["fixed_noise"]))
    img, d, z, c = _blend_through_api(f, device, rast, agg, use_shader=entry == "RandomSimpleShader")
    _check(f, img, d, z, c, rast, agg)


@pytest.mark.gpu
@pytest.mark.parametrize("case", VARIANT_CASES)
def test_seeded_variant_pairs_match_reference(case, device, torch_noise):
    f = load_golden(case)
    rast = getattr(pa, str(f["rast_cls"]))(nb_samples=int(f["Sr"]), sigma=float(f["sigma"]))
    agg = getattr(pa, str(f["agg_cls"]))(nb_samples=int(f["Sa"]), gamma=float(f["gamma"]),
                                         alpha=float(f["alpha"]), eps=float(f["eps"]))
    img, d, z, c = _blend_through_api(f, device, rast, agg)
    _check(f, img, d, z, c, rast, agg)


@pytest.mark.gpu
def test_seeded_standalone_rasterize_matches_reference(device, torch_noise):
    f = load_golden("rast_only")
    rast = pa.GaussianRast(nb_samples=int(f["Sr"]), sigma=float(f["sigma"]))
    d = torch.tensor(f["dists"], device=device, requires_grad=True)
    torch.manual_seed(int(f["seed"]))
    P = rast.rasterize(d)
    (P * torch.tensor(f["grad_P"], device=device)).sum().backward()
    np.testing.assert_array_equal(P.detach().cpu().numpy(), f["P"])
    assert_close(d.grad, f["grad_dists"], name="dists")
    assert_close(rast.sigma.grad, f["grad_sigma"], rtol=SCALAR_RTOL, name="sigma")


@pytest.mark.gpu
def test_seeded_standalone_aggregate_matches_reference(device, torch_noise):
    f = load_golden("agg_only")
    agg = pa.GaussianAgg(nb_samples=int(f["Sa"]), gamma=float(f["gamma"]), alpha=float(f["alpha"]),
                         eps=float(f["eps"]))
    z = torch.tensor(f["zbuf"], device=device, requires_grad=True)
    pr = torch.tensor(f["prob"], device=device, requires_grad=True)
    mask = torch.tensor(f["pix_to_face"], device=device) >= 0
    N = z.shape[0]
    zn, zf = _planes(f, N, device)
    torch.manual_seed(int(f["seed"]))
    W = agg.aggregate(z, zf, zn, pr, mask)
    (W * torch.tensor(f["grad_W"], device=device)).sum().backward()
    np.testing.assert_array_equal(W.detach().cpu().numpy(), f["W"])
    assert_close(z.grad, f["grad_zbuf"], name="zbuf")
    assert_close(pr.grad, f["grad_prob"], name="prob")
    assert_close(agg.gamma.grad, f["grad_gamma"], rtol=SCALAR_RTOL, name="gamma")
    assert_close(agg.alpha.grad, f["grad_alpha"], rtol=SCALAR_RTOL, name="alpha")


@pytest.mark.gpu
def test_seeded_uniform_aggregate_matches_reference(device, torch_noise):
    """UniformAgg.aggregate (smoothagg.py:252-271) through the public class, seeded like the
    reference: weights equal; the backward raises as the reference's does (:64-70)."""
    f = load_golden("agg_uniform")
    agg = pa.UniformAgg(nb_samples=int(f["Sa"]), gamma=float(f["gamma"]), alpha=float(f["alpha"]),
                        eps=float(f["eps"]))
    z = torch.tensor(f["zbuf"], device=device, requires_grad=True)
    pr = torch.tensor(f["prob"], device=device)
    mask = torch.tensor(f["pix_to_face"], device=device) >= 0
    zn, zf = _planes(f, z.shape[0], device)
    torch.manual_seed(int(f["seed"]))
    W = agg.aggregate(z, zf, zn, pr, mask)
    np.testing.assert_array_equal(W.detach().cpu().numpy(), f["W"])
    with pytest.raises(NotImplementedError):
        W.sum().backward()


@pytest.mark.gpu
def test_philox_uniform_argmax_frequencies(device):
    """Native Philox U(-1/2, 1/2) agg noise: weights converge to P(argmax z + gamma u) (numpy MC)."""
    reps = 4096
    zbuf = torch.tensor([5.0, 5.004]).reshape(1, 1, 1, 2).repeat(1, reps, 1, 1).to(device)
    prob = torch.ones_like(zbuf) * 0.5
    mask = torch.ones_like(zbuf, dtype=torch.bool)
    agg = pa.UniformAgg(nb_samples=16, gamma=1e-2)
    W = agg.aggregate(zbuf, 100.0, 1.0, prob, mask)
    w = W.detach().mean(dim=(0, 1, 2)).cpu().double().numpy()
    z_inv = (100.0 - np.array([5.0, 5.004])) / 99.0
    z = np.concatenate([1e-2 * np.log(0.5) + z_inv - z_inv.max(), [1e-10 - z_inv.max()]])
    u = np.random.default_rng(0).uniform(-0.5, 0.5, (400000, 3))
    ref = np.bincount(np.argmax(z + 1e-2 * u, axis=1), minlength=3) / 400000.0
    assert np.all(np.abs(w - ref) < 0.01), (w, ref)


def _soft(dev):
    f = load_golden("soft_blend")
    fr, d, z = _fragments(f, dev)
    c = torch.tensor(f["colors"], device=dev, requires_grad=True)
    zn, zf = _planes(f, 1, dev)
    rast = pa.SoftRast(sigma=float(f["sigma"]))
    agg = pa.SoftAgg(gamma=float(f["gamma"]), alpha=float(f["alpha"]), eps=float(f["eps"]))
    bp = BlendParams(float(f["sigma"]), float(f["gamma"]), tuple(float(v) for v in f["background"]))
    img = smooth_rgb_blend(c, fr, rast, agg, bp, znear=zn, zfar=zf)
    (img * torch.tensor(f["grad_image"], device=dev)).sum().backward()
    return f, img, d, z, c, rast, agg


def test_product_softrast_softagg_matches_reference_cpu():
    """The product SoftRast / SoftAgg classes (not the oracle) against soft_blend.npz: bitwise on
    the CPU, where both run the same torch ops."""
    f, img, d, z, c, rast, agg = _soft(torch.device("cpu"))
    np.testing.assert_array_equal(img.detach().numpy(), f["image"])
    for k, t in (("dists", d.grad), ("zbuf", z.grad), ("colors", c.grad), ("sigma", rast.sigma.grad),
                 ("gamma", agg.gamma.grad), ("alpha", agg.alpha.grad)):
        np.testing.assert_array_equal(t.numpy(), f["grad_" + k], err_msg=k)


@pytest.mark.gpu
def test_product_softrast_softagg_matches_reference_gpu(device):
    f, img, d, z, c, rast, agg = _soft(device)
    _check(f, img, d, z, c, rast, agg)
