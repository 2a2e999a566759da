"""The in-process collectives of pertrenderer_amd.multidevice as autograd functions (CPU, logical
devices): broadcast's adjoint is the sum-reduce and the weighted reduce's adjoint is the weighted
broadcast -- checked with torch.autograd.gradcheck in float64 -- plus the shard split that
set_sample_devices uses."""
import torch

from pertrenderer_amd import multidevice as md
from pertrenderer_amd.parallel import sample_shard


def test_broadcast_and_weighted_reduce_are_adjoint():
    cpu = torch.device("cpu")
    x = torch.randn(3, 4, dtype=torch.float64, requires_grad=True)
    ys = torch.randn(3, 3, 4, dtype=torch.float64, requires_grad=True)

    def f(x, ys):
        b = md._Broadcast.apply([cpu, cpu, cpu], x)
        parts = [b[i] * ys[i] for i in range(3)]
        return md._WeightedReduce.apply(cpu, [0.25, 0.25, 0.5], *parts)

    assert torch.autograd.gradcheck(f, (x, ys))
    out = f(x, ys)
    torch.testing.assert_close(out, x * (0.25 * ys[0] + 0.25 * ys[1] + 0.5 * ys[2]))


def test_broadcast_outputs_are_distinct_tensors():
    x = torch.randn(5, requires_grad=True)
    outs = md._Broadcast.apply([torch.device("cpu")] * 2, x)
    assert len(outs) == 2 and outs[0] is not outs[1]
    (outs[0].sum() + 2 * outs[1].sum()).backward()
    torch.testing.assert_close(x.grad, torch.full((5,), 3.0))


def test_device_shards_cover_the_samples():
    for S in (4, 8, 16, 64):
        for n in (1, 2, 3, 4, 8):
            if S < n:
                continue
            sh = [sample_shard(S, i, n) for i in range(n)]
            assert sum(c for _, c in sh) == S and all(c >= 1 for _, c in sh)
            assert [o for o, _ in sh] == sorted(o for o, _ in sh) and sh[0][0] == 0


def test_set_sample_devices_needs_rocm_devices():
    import pytest
    with pytest.raises(ValueError):
        md.set_sample_devices(["cpu", "cpu"])
    md.set_sample_devices(None)
    assert md.sample_devices() is None


def test_count_reduce_is_exact_and_its_adjoint_is_the_weighted_broadcast():
    """P = (sum_i round(n_i P_i)) / Sr: the one-device count / Sr bit for bit even when n_i does not
    divide Sr (6 / 5 / 5 of 16), and the gradient that of sum_i (n_i / Sr) P_i."""
    cpu = torch.device("cpu")
    g = torch.Generator().manual_seed(0)
    ns, Sr = [6, 5, 5], 16
    cnt = [torch.randint(0, n + 1, (7, 9), generator=g) for n in ns]
    ps = [(c.float() / n).requires_grad_(True) for c, n in zip(cnt, ns)]
    P = md._CountReduce.apply(cpu, ns, Sr, *ps)
    assert torch.equal(P, sum(c for c in cnt).float() / Sr)
    w = torch.randn(7, 9, generator=g)
    (P * w).sum().backward()
    for p, n in zip(ps, ns):
        torch.testing.assert_close(p.grad, w * (n / Sr))


def test_shard_images_route_rgb_by_weight_and_alpha_to_the_primary():
    cpu = torch.device("cpu")
    image = torch.rand(1, 2, 3, 4)
    shards = [torch.rand(1, 2, 3, 4, requires_grad=True) for _ in range(3)]
    out = md._ShardImages.apply(image, [0.5, 0.25, 0.25], *shards)
    assert torch.equal(out, image)
    g = torch.randn(1, 2, 3, 4)
    out.backward(g)
    for i, (s, w) in enumerate(zip(shards, [0.5, 0.25, 0.25])):
        torch.testing.assert_close(s.grad[..., :3], g[..., :3] * w)
        torch.testing.assert_close(s.grad[..., 3], g[..., 3] if i == 0 else torch.zeros_like(g[..., 3]))
