"""The CPU oracle (oracle/blend_oracle.py) reproduces the reference's own outputs.

Golden vectors were produced by importing the reference randomras package
(tests/golden/gen_golden.py).  The bar for the oracle is bit-exactness."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import blend_oracle as bo

T = lambda a: torch.from_numpy(np.asarray(a))
BLEND_CASES = ["blend_small", "blend_eval", "blend_edge", "blend_fixed", "blend_k100"]


def _planes(f, N):
    return torch.full((N, 1, 1, 1), float(f["znear"])), torch.full((N, 1, 1, 1), float(f["zfar"]))


@pytest.mark.parametrize("case", BLEND_CASES)
def test_blend_oracle_matches_reference_bitwise(case):
    f = load_golden(case)
    zn, zf = _planes(f, f["pix_to_face"].shape[0])
    img, saved = bo.blend_forward(T(f["pix_to_face"]), T(f["dists"]), T(f["zbuf"]), T(f["colors"]),
                                  T(f["noise_r"]), T(f["noise_a"]), T(f["sigma"]), T(f["gamma"]),
                                  T(f["alpha"]), float(f["eps"]), T(f["background"]), zn, zf)
    g = bo.blend_backward(T(f["grad_image"]), saved)
    np.testing.assert_array_equal(img.numpy(), f["image"])
    for k in ("dists", "zbuf", "colors", "sigma", "gamma", "alpha"):
        np.testing.assert_array_equal(g[k].numpy(), f["grad_" + k], err_msg=k)


def test_rasterize_oracle_matches_reference_bitwise():
    f = load_golden("rast_only")
    P, dd, ds = bo.rasterize_forward_backward(T(f["dists"]), T(f["noise_r"]), T(f["sigma"]), T(f["grad_P"]))
    np.testing.assert_array_equal(P.numpy(), f["P"])
    np.testing.assert_array_equal(dd.numpy(), f["grad_dists"])
    np.testing.assert_array_equal(ds.numpy(), f["grad_sigma"])


def test_aggregate_oracle_matches_reference_bitwise():
    f = load_golden("agg_only")
    zn, zf = _planes(f, f["zbuf"].shape[0])
    W, dzb, dpr, dg, da = bo.aggregate_forward_backward(
        T(f["zbuf"]), zf, zn, T(f["prob"]), T(f["pix_to_face"]) >= 0, T(f["noise_a"]), T(f["gamma"]),
        T(f["alpha"]), float(f["eps"]), T(f["grad_W"]))
    np.testing.assert_array_equal(W.numpy(), f["W"])
    np.testing.assert_array_equal(dzb.numpy(), f["grad_zbuf"])
    np.testing.assert_array_equal(dpr.numpy(), f["grad_prob"])
    np.testing.assert_array_equal(dg.numpy(), f["grad_gamma"])
    np.testing.assert_array_equal(da.numpy(), f["grad_alpha"])


def test_uniform_aggregate_oracle_matches_reference_bitwise():
    """UniformAgg forward (smoothagg.py:252-271): the oracle's logits + argmax with the
    reference's U(-1/2, 1/2) draw reproduce its weights."""
    f = load_golden("agg_uniform")
    zn, zf = _planes(f, f["zbuf"].shape[0])
    z, _ = bo.logits(T(f["zbuf"]), zf, zn, T(f["prob"]), T(f["pix_to_face"]) >= 0, T(f["gamma"]), T(f["alpha"]),
                     float(f["eps"]))
    W, _, _ = bo.argmax_fwd(z, T(f["noise_a"]), T(f["gamma"]))
    np.testing.assert_array_equal(W.numpy(), f["W"])


def test_soft_blend_oracle_matches_reference_bitwise():
    f = load_golden("soft_blend")
    zn, zf = _planes(f, 1)
    img, g = bo.soft_blend_forward_backward(
        T(f["pix_to_face"]), T(f["dists"]), T(f["zbuf"]), T(f["colors"]), float(f["sigma"]), float(f["gamma"]),
        float(f["alpha"]), float(f["eps"]), T(f["background"]), zn, zf, T(f["grad_image"]))
    np.testing.assert_array_equal(img.numpy(), f["image"])
    for k in ("dists", "zbuf", "colors", "sigma", "gamma", "alpha"):
        np.testing.assert_array_equal(g[k].numpy(), f["grad_" + k], err_msg=k)


def test_golden_noise_is_the_reference_draw_order():
    """randn(Sr,N,H,W,K) then randn(Sa,N,H,W,K+1) from the seeded CPU generator."""
    f = load_golden("blend_small")
    torch.manual_seed(int(f["seed"]))
    er = torch.randn(f["noise_r"].shape)
    ea = torch.randn(f["noise_a"].shape)
    np.testing.assert_array_equal(er.numpy(), f["noise_r"])
    np.testing.assert_array_equal(ea.numpy(), f["noise_a"])


VARIANT_CASES = ["var_arctan_cauchy", "var_wovr", "var_mixed"]


def variant_kinds(f):
    return str(f["rast_kind"]), bool(f["rast_vr"]), str(f["agg_kind"]), bool(f["agg_vr"])


@pytest.mark.parametrize("case", VARIANT_CASES)
def test_variant_blend_oracle_matches_reference(case):
    """ArctanRast / GaussianRast_wovr x CauchyAgg / GaussianAgg_wovr (smoothrast.py:61-173,
    smoothagg.py:75-250): bitwise, except d gamma with Cauchy agg noise (the reference
    contracts score.eps with a matmul: fp32 summation order)."""
    f = load_golden(case)
    zn, zf = _planes(f, f["pix_to_face"].shape[0])
    rk, rvr, ak, avr = variant_kinds(f)
    img, saved = bo.blend_forward(T(f["pix_to_face"]), T(f["dists"]), T(f["zbuf"]), T(f["colors"]),
                                  T(f["noise_r"]), T(f["noise_a"]), T(f["sigma"]), T(f["gamma"]),
                                  T(f["alpha"]), float(f["eps"]), T(f["background"]), zn, zf, rk, rvr, ak, avr)
    g = bo.blend_backward(T(f["grad_image"]), saved)
    np.testing.assert_array_equal(img.numpy(), f["image"])
    for k in ("dists", "zbuf", "colors", "sigma", "gamma", "alpha"):
        if k == "gamma" and ak == "cauchy":
            np.testing.assert_allclose(g[k].numpy(), f["grad_" + k], rtol=2e-6, err_msg=k)
        else:
            np.testing.assert_array_equal(g[k].numpy(), f["grad_" + k], err_msg=k)
