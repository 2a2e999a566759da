"""GPU twin of tests/test_rast_oracle.py: the HIP rasterizer (pr_rast_fwd / pr_rast_bwd through
the C ABI) on the hand-computed known-answer cases, and its backward against the fp64 oracle
backward that the finite-difference test pins."""
import numpy as np
import pytest
import torch

import rast_kat
from conftest import assert_close
from oracle import rast_ref
from pertrenderer_amd.renderer.rasterizer import _rasterize, valid_counts

pytestmark = pytest.mark.gpu


def _native(case, dev, requires_grad=False, bins=(0, 0)):
    fv = torch.tensor(case["fv"], dtype=torch.float32, device=dev, requires_grad=requires_grad)
    out = _rasterize(fv, torch.tensor(case["first"], device=dev), torch.tensor(case["nfaces"], device=dev),
                     case["H"], case["W"], case["K"], case["blur"], case["persp"], case["clip"], case["cull"], bins)
    return fv, out


@pytest.mark.parametrize("bins", [(0, 0), (8, 10000)], ids=["naive", "bins8"])
@pytest.mark.parametrize("case", rast_kat.CASES, ids=[c["name"] for c in rast_kat.CASES])
def test_hip_rasterizer_known_answers(case, bins, device):
    _, (p2f, zbuf, bary, dists) = _native(case, device, bins=bins)
    rast_kat.check(case, p2f.cpu().numpy(), zbuf.cpu().numpy(), bary.cpu().numpy(), dists.cpu().numpy())
    np.testing.assert_array_equal(valid_counts(p2f).cpu().numpy(), (case["p2f"] >= 0).sum(-1))


@pytest.mark.parametrize("persp,clip", [(False, False), (False, True), (True, True)])
def test_hip_rasterizer_backward_matches_fd_pinned_oracle(persp, clip, device):
    F, H, W, K, blur = 10, 14, 14, 5, 0.02
    fv64 = rast_kat.soup(F, seed=3)
    case = dict(fv=fv64.astype(np.float32), first=np.array([0]), nfaces=np.array([F]), H=H, W=W, K=K, blur=blur,
                persp=persp, clip=clip, cull=False)
    fv, (p2f, zbuf, bary, dists) = _native(case, device, requires_grad=True)
    p = p2f.cpu().numpy()
    valid = p >= 0
    if persp:
        valid &= rast_kat.persp_denominator(fv64, p, H, W) > 0.1
    rng = np.random.default_rng(1)
    gz = rng.standard_normal((1, H, W, K)) * valid
    gb = rng.standard_normal((1, H, W, K, 3)) * valid[..., None]
    gd = rng.standard_normal((1, H, W, K)) * valid
    T = lambda a: torch.tensor(a, dtype=torch.float32, device=device)
    ((zbuf * T(gz)).sum() + (bary * T(gb)).sum() + (dists * T(gd)).sum()).backward()
    got = fv.grad.cpu().numpy()
    # the fp32 oracle, at the 1e-5 bar (the default backward sums faces with float atomics) and bit
    # for bit in deterministic mode (slot-order face sums)
    gz32, gb32, gd32 = (x.astype(np.float32) for x in (gz, gb, gd))
    ref32 = rast_ref.rast_bwd(case["fv"], p, gz32, gb32, gd32, persp, clip)
    assert_close(got, ref32, name="d face_verts vs fp32 oracle")
    old = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True)
    try:
        fvd, (_, zd, bd, dd) = _native(case, device, requires_grad=True)
        (gdet,) = torch.autograd.grad((zd * T(gz)).sum() + (bd * T(gb)).sum() + (dd * T(gd)).sum(), fvd)
    finally:
        torch.use_deterministic_algorithms(old)
    np.testing.assert_array_equal(gdet.cpu().numpy(), ref32)
    # and the fp64 oracle (pinned by central differences, test_rast_oracle.py): the fp32 rounding of
    # the same formulas (edge functions of nearby points cancel: the absolute bound is the scale)
    ref = rast_ref.rast_bwd(fv64, p, gz, gb, gd, persp, clip, dtype=np.float64)
    np.testing.assert_allclose(got.astype(np.float64), ref, rtol=1e-3, atol=1e-4 * np.abs(ref).max())
