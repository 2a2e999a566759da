"""The C++ autograd nodes (csrc/pr_torch.cpp) keep their tensors through save_for_backward, so
they are released once the backward has run (saved_data kept the rast cache, winners
and input copies alive until the graph itself died, doubling an eager loop's peak memory), a
second backward without retain_graph raises as for any torch node, and with retain_graph it
gives the same gradients again."""
import pytest
import torch

import pertrenderer_amd as pa
from pertrenderer_amd import Noise, host_layer

pytestmark = pytest.mark.gpu


def _frags(device, N=1, H=256, W=256, K=50):
    g = torch.Generator(device).manual_seed(7)
    cnt = torch.randint(0, K + 1, (N, H, W), generator=g, device=device)
    valid = torch.arange(K, device=device) < cnt[..., None]
    p2f = torch.where(valid, torch.randint(0, 900, (N, H, W, K), generator=g, device=device), -1)
    dists = (torch.rand((N, H, W, K), generator=g, device=device) - 0.5) * 6e-3
    zbuf = torch.where(valid, (5.0 + torch.rand((N, H, W, K), generator=g, device=device)).sort(-1).values, -1.)
    colors = torch.rand((N, H, W, K, 3), generator=g, device=device)
    return p2f, dists, zbuf, colors


def _blend(p2f, d, z, c):
    sig, gam, alp = (torch.tensor(v, device=d.device, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
    return pa.perturbed_blend(c, p2f, d, z, sig, gam, alp, 8, 8, background=(0.0, 0.0, 0.0),
                              noise=Noise.philox(seed_r=1, seed_a=2))


def test_blend_buffers_released_after_backward(device):
    if host_layer.layer() != "c++":
        pytest.skip(f"C++ autograd layer not loaded: {host_layer.error()}")
    p2f, d0, z0, c0 = _frags(device)
    gimg = torch.randn((1, 256, 256, 4), device=device)
    # one call first: per-process caches made on first use (znear / zfar planes, background, valid
    # counts of these fragments) are not per-call buffers (their size depends on the tests run before)
    w = [t.clone().requires_grad_(True) for t in (d0, z0, c0)]
    _blend(p2f, *w).backward(gimg)
    del w
    d, z, c = (t.clone().requires_grad_(True) for t in (d0, z0, c0))
    torch.cuda.synchronize()
    m0 = torch.cuda.memory_allocated(device)
    img = _blend(p2f, d, z, c)
    torch.cuda.synchronize()
    held = torch.cuda.memory_allocated(device) - m0  # image + the node's saved buffers (rast cache 26 MB)
    cache = p2f.numel() * 8
    assert held > cache, (held, cache)
    img.backward(gimg)
    torch.cuda.synchronize()
    grads = sum(t.grad.numel() * t.grad.element_size() for t in (d, z, c))
    after = torch.cuda.memory_allocated(device) - m0 - grads
    # img is still referenced (its grad_fn too): only the image itself may remain
    assert after < img.numel() * img.element_size() + (1 << 20), (after, held)
    with pytest.raises(RuntimeError):
        img.backward(gimg)


def test_blend_retain_graph_second_backward_matches(device):
    if host_layer.layer() != "c++":
        pytest.skip(f"C++ autograd layer not loaded: {host_layer.error()}")
    p2f, d0, z0, c0 = _frags(device, H=64, W=64, K=20)
    d, z, c = (t.clone().requires_grad_(True) for t in (d0, z0, c0))
    img = _blend(p2f, d, z, c)
    g = torch.randn(img.shape, device=device)
    img.backward(g, retain_graph=True)
    first = [t.grad.clone() for t in (d, z, c)]
    for t in (d, z, c):
        t.grad = None
    img.backward(g)
    for a, b in zip(first, (d.grad, z.grad, c.grad)):
        assert torch.equal(a, b)


def test_inplace_change_of_a_saved_input_raises(device):
    """save_for_backward's version check: modifying dists in place after the forward is refused."""
    if host_layer.layer() != "c++":
        pytest.skip(f"C++ autograd layer not loaded: {host_layer.error()}")
    p2f, d0, z0, c0 = _frags(device, H=32, W=32, K=10)
    d = d0.clone().requires_grad_(True)
    dd = d * 1.0  # a non-leaf the node saves
    img = _blend(p2f, dd, z0, c0)
    with torch.no_grad():
        dd.add_(1.0)
    with pytest.raises(RuntimeError):
        img.sum().backward()
