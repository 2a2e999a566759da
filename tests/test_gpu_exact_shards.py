"""Exact sample-sharded mode (pertrenderer_amd.parallel.exact_sharded_blend):
2 and 4 ranks (gloo, all on cuda:0) reproduce the single-process full-S result -- image
bitwise (P and W are exact counts), gradients up to the summation order of the rank
partials -- and the single-process composition of the standalone native ops equals the
fused perturbed_blend with the same Philox keys."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
SEEDS = (1234, 5678)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(dev, S):
    g = torch.Generator().manual_seed(11)
    N, H, W, K = 1, 24, 20, 12
    cnt = torch.randint(0, K + 1, (N, H, W, 1), generator=g)
    valid = torch.arange(K).expand(N, H, W, K) < cnt
    p2f = torch.where(valid, torch.randint(0, 500, (N, H, W, K), generator=g), torch.full((N, H, W, K), -1))
    dists = torch.where(valid, (torch.rand((N, H, W, K), generator=g) - 0.5) * 6e-3, torch.full((N, H, W, K), -1.0))
    zbuf = torch.where(valid, (5.0 + torch.rand((N, H, W, K), generator=g)).sort(-1).values,
                       torch.full((N, H, W, K), -1.0))
    colors = torch.rand((N, H, W, K, 3), generator=g)
    gimg = torch.randn((N, H, W, 4), generator=g)
    to = lambda t, grad=False: t.to(dev).requires_grad_(grad)
    leaves = [torch.tensor(v, requires_grad=True) for v in (1e-3, 1e-2, 1.0)]
    return to(p2f), to(dists, True), to(zbuf, True), to(colors, True), to(gimg), leaves, S


def _worker(rank, world, port, S, out_path, backend="gloo"):
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    if backend == "nccl":  # RCCL: one rank per GPU, so world 1 on the one-GPU box
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from pertrenderer_amd import Noise, perturbed_blend
        from pertrenderer_amd.parallel import exact_sharded_blend, reduce_scalar_grads
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        p2f, d, z, c, gimg, (s, gm, al), S = _inputs(dev, S)
        img = exact_sharded_blend(c, p2f, d, z, s, gm, al, S, S, SEEDS[0], SEEDS[1], background=(0.1, 0.2, 0.3))
        (img * gimg).sum().backward()
        reduce_scalar_grads([s, gm, al])
        out = dict(image=img.detach().cpu(), dists=d.grad.cpu(), zbuf=z.grad.cpu(), colors=c.grad.cpu(),
                   scalars=torch.stack([s.grad, gm.grad, al.grad]))
        # a second backward without zeroing (eval.py's first 100 iterations accumulate the
        # smoothing leaves, eval.py:382-385): exactly twice the one-backward gradient
        img = exact_sharded_blend(c, p2f, d, z, s, gm, al, S, S, SEEDS[0], SEEDS[1], background=(0.1, 0.2, 0.3))
        (img * gimg).sum().backward()
        reduce_scalar_grads([s, gm, al])
        out["scalars2"] = torch.stack([s.grad, gm.grad, al.grad])
        # then eval.py:386's reset (grads replaced by zeros) before a third backward: one gradient
        for t in (s, gm, al):
            t.grad = torch.zeros_like(t)
        img = exact_sharded_blend(c, p2f, d, z, s, gm, al, S, S, SEEDS[0], SEEDS[1], background=(0.1, 0.2, 0.3))
        (img * gimg).sum().backward()
        reduce_scalar_grads([s, gm, al])
        out["scalars3"] = torch.stack([s.grad, gm.grad, al.grad])
        if world == 1:  # the fused kernel pair with the same keys
            p2f, d, z, c, gimg, (s, gm, al), S = _inputs(dev, S)
            img = perturbed_blend(c, p2f, d, z, s, gm, al, S, S, background=(0.1, 0.2, 0.3),
                                  noise=Noise.philox(seed_r=SEEDS[0], seed_a=SEEDS[1]))
            (img * gimg).sum().backward()
            out.update(f_image=img.detach().cpu(), f_dists=d.grad.cpu(), f_zbuf=z.grad.cpu(),
                       f_colors=c.grad.cpu(), f_scalars=torch.stack([s.grad, gm.grad, al.grad]))
        torch.cuda.synchronize()
        if rank == 0:
            torch.save(out, out_path)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(world, S, backend="gloo"):
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "out.pt")
        mp.spawn(_worker, args=(world, _free_port(), S, path, backend), nprocs=world, join=True)
        return torch.load(path, weights_only=True)


def _close(a, b, rtol=1e-5, name=""):
    scale = float(b.abs().max())
    err = float((a - b).abs().max())
    assert err <= rtol * max(scale, 1e-30), (name, err, scale)


@pytest.mark.parametrize("world,S", [(2, 8), (4, 16)])
def test_exact_shards_match_single_process(world, S):
    one = _run(1, S)
    many = _run(world, S)
    assert torch.equal(one["image"], many["image"])
    for k in ("dists", "zbuf", "colors"):
        _close(many[k], one[k], name=k)
    _close(many["scalars"], one["scalars"], rtol=2e-5, name="scalars")
    _close(many["scalars2"], 2 * one["scalars"], rtol=2e-5, name="accumulated scalars")
    _close(many["scalars3"], one["scalars"], rtol=2e-5, name="scalars after the eval.py:386 reset")


def test_exact_mode_composition_matches_fused_blend():
    one = _run(1, 8)
    torch.testing.assert_close(one["image"], one["f_image"], rtol=1e-5, atol=1e-6)
    for k in ("dists", "zbuf", "colors"):
        _close(one[k], one["f_" + k], name=k)
    _close(one["scalars"], one["f_scalars"], rtol=2e-5, name="scalars")


def test_exact_mode_on_one_rccl_rank():
    """The same exact-mode step over an RCCL (torch.distributed "nccl") process group of one rank:
    its collectives (device all-reduces in both autograd directions, the smoothing-scalar completion)
    run through RCCL and return the gloo run's values bit for bit."""
    one = _run(1, 8)
    rccl = _run(1, 8, backend="nccl")
    for k in ("image", "dists", "zbuf", "colors", "scalars", "scalars2", "scalars3"):
        assert torch.equal(rccl[k], one[k]), k
