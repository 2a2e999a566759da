"""Pins the rasterizer oracle (oracle/rast_oracle.c, PyTorch3D 0.4.0 rasterize_meshes semantics).

PyTorch3D is not vendored and not installable here, so the reference cannot pin the rasterizer
("parity unpinned").  Instead the oracle is pinned by
  * hand-computed known-answer cases (tests/rast_kat.py): inside / outside signed squared
    distance, the squared blur threshold with a sqrt(blur) bounding box, zmax < 0 and pz < 0
    culls, degenerate-area and back-face culls, K truncation with (z, face index) tie order,
    clipped and perspective-correct barycentrics, the non-square NDC mapping, packed batches;
  * an fp64 central-difference check of its backward (d zbuf, d bary, d dists -> d face verts)
    with and without perspective correction / clipping.
The HIP kernels are compared with the same cases in tests/test_gpu_rast_kat.py.
"""
import numpy as np
import pytest

import rast_kat
from oracle import rast_ref


def _run(case, dtype=np.float32):
    return rast_ref.rast_fwd(case["fv"], case["first"], case["nfaces"], case["H"], case["W"], case["K"],
                             case["blur"], case["persp"], case["clip"], case["cull"], dtype=dtype)


@pytest.mark.parametrize("case", rast_kat.CASES, ids=[c["name"] for c in rast_kat.CASES])
def test_oracle_known_answers(case):
    rast_kat.check(case, *_run(case))


@pytest.mark.parametrize("name", ["blur_kept", "clip", "perspective_clip", "cull_pz", "nonsquare_wide",
                                  "k_truncation", "two_meshes"])
def test_oracle_known_answers_fp64(name):
    """The same answers in double precision (no fp32 rounding luck)."""
    case = next(c for c in rast_kat.CASES if c["name"] == name)
    rast_kat.check(case, *_run(case, np.float64), tol=1e-7)


def _loss_terms(F, H, W, K, seed):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((1, H, W, K)), rng.standard_normal((1, H, W, K, 3)),
            rng.standard_normal((1, H, W, K)))


@pytest.mark.parametrize("persp,clip", [(False, False), (False, True), (True, False), (True, True)])
def test_oracle_backward_matches_central_differences_fp64(persp, clip):
    F, H, W, K, blur = 10, 14, 14, 5, 0.02
    fv = rast_kat.soup(F, seed=3)
    first, nf = np.array([0]), np.array([F])
    p2f, zb, ba, di = rast_ref.rast_fwd(fv, first, nf, H, W, K, blur, persp, clip, False, dtype=np.float64)
    valid = p2f >= 0
    assert valid.sum() > 100
    if persp:
        # PyTorch3D clamps the perspective denominator sum_i w_i prod_{j!=i} z_j at 1e-8; outside
        # pixels where it is <= 0 get ~1e8 weights (a kink, not a gradient): leave those out
        valid &= rast_kat.persp_denominator(fv, p2f, H, W) > 0.1
    gz, gb, gd = _loss_terms(F, H, W, K, 1)
    gz, gb, gd = gz * valid, gb * valid[..., None], gd * valid

    def loss(x):
        p, z, b, d = rast_ref.rast_fwd(x, first, nf, H, W, K, blur, persp, clip, False, dtype=np.float64)
        return p, float((gz * z).sum() + (gb * b).sum() + (gd * d).sum())

    analytic = rast_ref.rast_bwd(fv, p2f, gz, gb, gd, persp, clip, dtype=np.float64)
    h = 1e-6
    used = 0
    for idx in np.ndindex(fv.shape):
        xp, xm = fv.copy(), fv.copy()
        xp[idx] += h
        xm[idx] -= h
        pp, lp = loss(xp)
        pm, lm = loss(xm)
        if not (np.array_equal(pp, p2f) and np.array_equal(pm, p2f)):
            continue  # the perturbation changed which faces a pixel keeps: not differentiable there
        used += 1
        fd = (lp - lm) / (2 * h)
        assert abs(analytic[idx] - fd) <= 1e-5 * max(1.0, abs(fd)), (idx, analytic[idx], fd)
    assert used >= 0.9 * fv.size, used


def test_oracle_fp32_and_fp64_agree_on_random_soup():
    """Away from ties the fp32 oracle (the parity target) selects the same faces as fp64."""
    fv = rast_kat.soup(40, seed=5)
    a = rast_ref.rast_fwd(fv, [0], [40], 24, 20, 6, 5e-3, False, True, False, dtype=np.float32)
    b = rast_ref.rast_fwd(fv, [0], [40], 24, 20, 6, 5e-3, False, True, False, dtype=np.float64)
    np.testing.assert_array_equal(a[0], b[0])
    for x, y in zip(a[1:], b[1:]):
        np.testing.assert_allclose(x, y, rtol=1e-4, atol=1e-5)
