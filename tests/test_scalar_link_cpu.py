"""CPU checks of the smoothing-scalar gradient link's plumbing (blend._ScalarLink, prelink): the
link node hands each CPU 0-d leaf its component of the (3,) gradient, with the leaf's dtype and
shape; leaves without requires_grad get none; nothing links on the CPU or without grad mode; a
shader without perturbed operators has nothing to prelink.  The GPU behaviour (bitwise equal
gradients with and without the link) is tests/test_gpu_scalar_link.py."""
import torch

from pertrenderer_amd import blend


def test_link_backward_routes_components_to_leaves():
    s = torch.tensor(1e-3, requires_grad=True)
    g = torch.tensor(1e-2, dtype=torch.float64, requires_grad=True)
    a = torch.tensor(1.0)  # no grad
    link = blend._ScalarLink.apply(torch.device("cpu"), s, g, a)
    assert link.shape == (3,)
    (link * torch.tensor([2.0, -3.0, 5.0])).sum().backward()
    assert s.grad.shape == () and float(s.grad) == 2.0
    assert g.grad.dtype == torch.float64 and float(g.grad) == -3.0
    assert a.grad is None


def test_nothing_links_on_cpu_or_without_grad():
    s = torch.tensor(1e-3, requires_grad=True)
    vals = (s, torch.tensor(1e-2), torch.tensor(1.0))
    assert not blend._linkable(vals, torch.device("cpu"))
    with torch.no_grad():
        assert not blend._linkable(vals, torch.device("cuda"))
    assert blend._link_scalars(vals, torch.device("cpu")) == (vals, None)
    assert blend.prelink(vals, torch.device("cpu")) is None
    assert blend._state().get("pre") is None


def test_prelink_shader_without_perturbed_operators():
    class Plain(torch.nn.Module):
        pass
    assert blend.prelink_shader(Plain(), None) is None
    blend.drop_prelink(None)  # a no-op
