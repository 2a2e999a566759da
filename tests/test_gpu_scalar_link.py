"""The smoothing-scalar gradient link (blend._ScalarLink, MeshRenderer's prelink).

The reference keeps sigma / gamma / alpha as CPU 0-d leaves (smoothrast.py:111-123,
smoothagg.py:145-163), so their gradients reach the host once per backward.  The link moves that
copy out of the blend's backward to a node that autograd runs after the rasterizer's backward,
waiting only for the blend kernels' event.  It must not change a single value: the same seeded
frame (torch noise, manual_seed) with and without the link gives bitwise-equal gradients of the
scalars and of the pose, through MeshRenderer (prelinked), through the shader alone (linked in the
blend call), with eval.py's in-place reset of the scalar gradients between backwards
(eval.py:386), and through torch.autograd.grad.
"""
import pytest
import torch

import pertrenderer_amd as pa
from pertrenderer_amd import blend

pytestmark = pytest.mark.gpu


def _frame(device, use_renderer, seed=11):
    import bench
    wl = bench.Workload(device, image_size=64, K=12, samples=4)
    torch.manual_seed(seed)
    if use_renderer:
        loss = wl.forward()
    else:
        from pertrenderer_amd.renderer import Rotate, so3_exponential_map
        R = so3_exponential_map(wl.log_rot)
        mesh = wl.base.update_padded(Rotate(R).transform_points(wl.base.verts_padded()))
        frag = wl.renderer.rasterizer(mesh, cameras=wl.cameras)
        torch.manual_seed(seed)
        img = wl.renderer.shader(frag, mesh, cameras=wl.cameras)
        loss = ((img[..., :3] - wl.target) ** 2).mean()
    return wl, loss


def _grads(device, use_renderer, link, reset=False):
    old = blend._LINK
    blend._LINK = link
    try:
        wl, loss = _frame(device, use_renderer)
        if reset:  # eval.py:386: the scalars' gradients replaced by zeros before this backward
            for p in (wl.rast.sigma, wl.agg.gamma, wl.agg.alpha):
                p.grad = torch.zeros_like(p)
        loss.backward()
        torch.cuda.synchronize()
        out = [p.grad.detach().clone() for p in wl.params()]
        assert all(p.grad.device.type == "cpu" and p.grad.dim() == 0 for p in wl.params()[1:])
        return out
    finally:
        blend._LINK = old


@pytest.mark.parametrize("use_renderer", [True, False])
@pytest.mark.parametrize("reset", [False, True])
def test_link_gradients_bitwise(device, use_renderer, reset):
    # deterministic-order backward: the pose gradient is then bitwise reproducible
    old, old_det = pa.noise.get_noise_source(), torch.are_deterministic_algorithms_enabled()
    pa.set_noise_source("torch")
    torch.use_deterministic_algorithms(True)
    try:
        a = _grads(device, use_renderer, True, reset)
        b = _grads(device, use_renderer, False, reset)
    finally:
        pa.set_noise_source(old)
        torch.use_deterministic_algorithms(old_det)
    for x, y, name in zip(a, b, ("log_rot", "sigma", "gamma", "alpha")):
        assert torch.equal(x.cpu(), y.cpu()), name
    assert float(a[1].abs()) > 0 and float(a[2].abs()) > 0


def test_link_autograd_grad_and_prelink_consumed(device):
    old, old_det = pa.noise.get_noise_source(), torch.are_deterministic_algorithms_enabled()
    pa.set_noise_source("torch")
    torch.use_deterministic_algorithms(True)
    try:
        wl, loss = _frame(device, True)
        assert blend._state().get("pre") is None  # MeshRenderer's prelink was consumed or dropped
        gs = torch.autograd.grad(loss, [wl.rast.sigma, wl.agg.gamma, wl.agg.alpha, wl.log_rot])
        ref = _grads(device, True, False)
    finally:
        pa.set_noise_source(old)
        torch.use_deterministic_algorithms(old_det)
    for x, y in zip(gs, [ref[1], ref[2], ref[3], ref[0]]):
        assert torch.equal(x.cpu(), y.cpu())
