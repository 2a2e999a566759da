"""Native deterministic SoftRast + SoftAgg blend (PR_BLEND_SOFT, csrc/pr_softblend.hip) against the
CPU oracle (oracle/blend_oracle.py: the reference composition, bitwise-pinned by soft_blend.npz)
on random fragments: K up to 150, z ties, saturated sigmoids (P = 1 and P = 0 slots), packed and
scattered valid slots, with and without the rasterizer's valid-prefix counts.  The golden-vector
check through the public classes is tests/test_public_api_parity.py."""
import numpy as np
import pytest
import torch

from conftest import assert_close
from oracle import blend_oracle as bo
from pertrenderer_amd import soft_blend
from pertrenderer_amd.renderer.rasterizer import attach_valid_counts

pytestmark = pytest.mark.gpu


def _frags(N, H, W, K, seed, packed, sigma):
    g = torch.Generator().manual_seed(seed)
    valid = torch.rand((N, H, W, K), generator=g) < 0.6
    if packed:
        cnt = valid.sum(-1, keepdim=True)
        valid = torch.arange(K).expand(N, H, W, K) < cnt
    p2f = torch.where(valid, torch.randint(0, 900, (N, H, W, K), generator=g), torch.full((N, H, W, K), -1))
    d = (torch.rand((N, H, W, K), generator=g) - 0.5) * 8 * sigma
    d[..., 0] = torch.where(torch.rand((N, H, W), generator=g) < 0.1, torch.full((N, H, W), -1.0), d[..., 0])  # P=1
    z = 5.0 + torch.rand((N, H, W, K), generator=g)
    if packed:
        z = z.sort(-1).values
    z[..., 1] = torch.where(torch.rand((N, H, W), generator=g) < 0.2, z[..., 0], z[..., 1])  # ties
    d = torch.where(valid, d, torch.full_like(d, -1.0))
    z = torch.where(valid, z, torch.full_like(z, -1.0))
    cols = torch.rand((N, H, W, K, 3), generator=g)
    gimg = torch.randn((N, H, W, 4), generator=g)
    return p2f, d, z, cols, gimg, valid


@pytest.mark.parametrize("shape,packed,counts", [((1, 16, 20, 50), True, True), ((2, 9, 7, 12), False, False),
                                                 ((1, 6, 5, 150), True, False), ((1, 8, 8, 3), True, True)])
def test_soft_blend_matches_oracle(shape, packed, counts, device):
    N, H, W, K = shape
    sigma, gamma, alpha, eps, bg = 1e-3, 1e-2, 1.3, 1e-10, (0.1, 0.2, 0.3)
    p2f, d, z, cols, gimg, valid = _frags(N, H, W, K, sum(shape), packed, sigma)
    zn, zf = torch.ones((N, 1, 1, 1)), torch.full((N, 1, 1, 1), 100.0)
    oimg, og = bo.soft_blend_forward_backward(p2f, d, z, cols, sigma, gamma, alpha, eps, bg, zn, zf, gimg)
    P = p2f.to(device)
    if counts:
        attach_valid_counts(P, valid.sum(-1).to(torch.int32).to(device))
    dd, zz, cc = (t.to(device).requires_grad_(True) for t in (d, z, cols))
    s, gm, al = (torch.tensor(v, requires_grad=True) for v in (sigma, gamma, alpha))
    img = soft_blend(cc, P, dd, zz, s, gm, al, eps=eps, background=bg, znear=zn.to(device), zfar=zf.to(device))
    (img * gimg.to(device)).sum().backward()
    assert_close(img, oimg, name="image")
    for k, t in (("dists", dd), ("colors", cc)):
        assert_close(t.grad, og[k], name=k)
    # d zbuf of a pixel's nearest slot carries d zmax = -(sum of all K+1 logit gradients), which
    # is exactly 0 in real arithmetic (a softmax is shift-invariant): both sides hold only its
    # fp32 rounding residue (~K ulp of the largest term), so that slot's bar is 1e-4 of the max
    assert_close(zz.grad, og["zbuf"], atol_rel=1e-4, name="zbuf")
    # the smoothing scalars are sums over all N*H*W*K slots of signed terms, reduced by the kernel's
    # workgroup tree and by the oracle's torch.sum: fp32 summation order alone moves them by ~1e-5
    # relative on the larger frames (measured 1.4e-5), so their bar is 5e-5
    for k, t in (("sigma", s), ("gamma", gm), ("alpha", al)):
        assert t.grad.device.type == "cpu"
        assert_close(t.grad, og[k], rtol=5e-5, name=k)


def test_soft_blend_device_scalars_and_capture(device):
    """Device smoothing leaves are read by pointer: the step captures into a HIP graph and
    replays to the eager result."""
    p2f, d, z, cols, gimg, _ = _frags(1, 12, 12, 20, 3, True, 1e-3)
    P, cc, gi, zz = p2f.to(device), cols.to(device), gimg.to(device), z.to(device)
    s, gm, al = (torch.tensor(v, device=device, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
    de = d.to(device).requires_grad_(True)
    eager = soft_blend(cc, P, de, zz, s, gm, al, background=(0, 0, 0))
    (eager * gi).sum().backward()
    ref_img, ref_g = eager.detach().clone(), de.grad.clone()
    del eager
    # a fresh leaf: its gradient accumulator must be created on the capture's side of the stream
    dd = d.to(device).requires_grad_(True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        (soft_blend(cc, P, dd, zz, s, gm, al, background=(0, 0, 0)) * gi).sum().backward()
    torch.cuda.current_stream().wait_stream(side)
    dd.grad.zero_()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        img = soft_blend(cc, P, dd, zz, s, gm, al, background=(0, 0, 0))
        (img * gi).sum().backward()
    dd.grad.zero_()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(img, ref_img)
    torch.testing.assert_close(dd.grad, ref_g, rtol=0, atol=0)
