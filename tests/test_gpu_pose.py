"""Native pose ops (pr_so3_exp_*, pr_rotate_*) against the torch formulas of
PyTorch3D 0.4.0's so3_exponential_map / Rotate.transform_points (evaluated on CPU)."""
import pytest
import torch

from pertrenderer_amd.renderer.transforms import Rotate, so3_exponential_map

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scale", [1e-4, 0.3, 2.5])
def test_so3_exponential_map_fwd_bwd(scale, device):
    g = torch.Generator().manual_seed(3)
    w = (scale * torch.randn((7, 3), generator=g))
    w[0] = 0.0  # below the clamp: zero gradient through the norm
    gR = torch.randn((7, 3, 3), generator=g)
    wc = w.clone().requires_grad_(True)
    Rc = so3_exponential_map(wc)
    (Rc * gR).sum().backward()
    wg = w.to(device).requires_grad_(True)
    Rg = so3_exponential_map(wg)
    (Rg * gR.to(device)).sum().backward()
    torch.testing.assert_close(Rg.detach().cpu(), Rc.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(wg.grad.cpu(), wc.grad, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("N,P,shared", [(1, 642, True), (3, 1000, False), (4, 17, True)])
def test_rotate_transform_points_fwd_bwd(N, P, shared, device):
    g = torch.Generator().manual_seed(N * P)
    pts = torch.randn((N, P, 3), generator=g)
    R = torch.randn((1 if shared else N, 3, 3), generator=g)
    gout = torch.randn((N, P, 3), generator=g)
    pc, Rc = pts.clone().requires_grad_(True), R.clone().requires_grad_(True)
    oc = Rotate(Rc).transform_points(pc)
    (oc * gout).sum().backward()
    pg, Rg = pts.to(device).requires_grad_(True), R.to(device).requires_grad_(True)
    og = Rotate(Rg).transform_points(pg)
    (og * gout.to(device)).sum().backward()
    torch.testing.assert_close(og.detach().cpu(), oc.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(pg.grad.cpu(), pc.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(Rg.grad.cpu(), Rc.grad, rtol=1e-4, atol=1e-4)
