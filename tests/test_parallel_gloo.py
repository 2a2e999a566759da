"""Multi-process (gloo, world size 2, CPU) tests of the data-parallel logic:
shard arithmetic, the single flattened gradient all-reduce, that Monte-Carlo
sample shards recombine exactly (counts are additive) using the CPU oracle, and the
exact mode's collective autograd pair."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pertrenderer_amd.parallel import average_gradients, sample_shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sample_shard_covers_range():
    for S in (1, 3, 4, 8, 13, 64, 128):
        for world in (1, 2, 3, 8):
            got = [sample_shard(S, r, world) for r in range(world)]
            off = 0
            for o, n in got:
                assert o == off and n >= 0
                off += n
            assert off == S
            if S % (4 * world) == 0:
                assert all(o % 4 == 0 for o, _ in got)
            if S >= world:  # every rank gets work (S=8 on 4 or 8 ranks splits per sample)
                assert all(n >= 1 for _, n in got), (S, world, got)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import blend_oracle as bo
        # 1) gradient averaging: one buffer holding a tensor grad and a 0-d CPU leaf grad
        a = torch.zeros(3, requires_grad=True)
        s = torch.tensor(1e-3, requires_grad=True)
        a.grad = torch.full((3,), float(rank + 1))
        s.grad = torch.tensor(float(10 * (rank + 1)))
        average_gradients([a, s])
        ok1 = torch.allclose(a.grad, torch.full((3,), 1.5)) and abs(float(s.grad) - 15.0) < 1e-6
        # 2) sample shards of the perturbed Heaviside recombine exactly
        g = torch.Generator().manual_seed(0)
        S = 8
        D = (torch.rand((1, 4, 5, 6), generator=g) - 0.5) * 4e-3
        noise = torch.randn((S, 1, 4, 5, 6), generator=g)
        off, n = sample_shard(S, rank, world)
        P_local, _, _ = bo.heaviside_fwd(D, noise[off:off + n], torch.tensor(1e-3))
        counts = P_local * n
        dist.all_reduce(counts)
        P_full, _, _ = bo.heaviside_fwd(D, noise, torch.tensor(1e-3))
        ok2 = torch.equal(counts / S, P_full)
        # 3) bench's sample-parallel mode: same keys, rank r draws global samples [r*S, (r+1)*S)
        from pertrenderer_amd import noise as nz
        nz.set_sample_shard(rank)
        torch.manual_seed(5)
        nr = nz.draw_rast((1, 2, 2, 3), 8, "cpu")
        na = nz.draw_agg((1, 2, 2, 4), 8, "cpu")
        keys = torch.tensor([nr.seed_r, na.seed_a], dtype=torch.int64)
        allk = [torch.zeros_like(keys) for _ in range(world)]
        dist.all_gather(allk, keys)
        ok3 = (nr.offset_r == 8 * rank and na.offset_a == 8 * rank and all(torch.equal(k, allk[0]) for k in allk))
        nz.set_sample_shard(0)
        # 4) exact mode's collective autograd pair (parallel.exact_sharded_blend): a
        #    rank-specific shard function between _SumBackward and _SumForward gives the
        #    full function's value and gradient on every rank
        from pertrenderer_amd.parallel import _SumBackward, _SumForward
        x = torch.tensor([0.3, -0.7, 1.1], requires_grad=True)
        c = torch.tensor([1.0, 2.0, 3.0])
        P = _SumForward.apply(_SumBackward.apply(x, None) ** (rank + 2), 0.5, None)
        (torch.sin(P) * c).sum().backward()
        xr = x.detach()
        P_ref = 0.5 * (xr ** 2 + xr ** 3)
        g_ref = torch.cos(P_ref) * c * 0.5 * (2 * xr + 3 * xr ** 2)
        ok4 = torch.allclose(P.detach(), P_ref, atol=1e-6) and torch.allclose(x.grad, g_ref, atol=1e-6)
        # 5) reduce_scalar_grads on a CPU 0-d leaf (the reference's sigma): each call completes
        #    only what the backwards since the last call delivered, so the leaf ends as in one
        #    process whether it accumulates (eval.py:382-385), is replaced with zeros
        #    (eval.py:386) or reset to None (optimizer.zero_grad) between iterations
        from pertrenderer_amd.parallel import reduce_scalar_grads, track_scalar_grads
        sg = torch.tensor(2.0, requires_grad=True)
        track_scalar_grads([sg])
        vals = []
        for _ in range(3):
            (sg * float(rank + 1)).backward()
            reduce_scalar_grads([sg])
            vals.append(float(sg.grad))
        sg.grad = torch.zeros_like(sg)  # eval.py:386
        (sg * float(rank + 1)).backward()
        reduce_scalar_grads([sg])
        vals.append(float(sg.grad))
        sg.grad.zero_()
        (sg * float(rank + 1)).backward()
        (sg * float(rank + 1)).backward()  # two backwards, one reduction
        reduce_scalar_grads([sg])
        vals.append(float(sg.grad))
        sg.grad = None
        (sg * float(rank + 1)).backward()
        reduce_scalar_grads([sg])
        vals.append(float(sg.grad))
        ok5 = sg.grad.device.type == "cpu" and np.allclose(vals, [3.0, 6.0, 9.0, 3.0, 6.0, 3.0]), vals
        ok4 = ok4 and ok5[0]
        q.put((rank, bool(ok1), bool(ok2 and ok3 and ok4)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gradient_average_and_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(r[0] for r in res) == [0, 1]
    assert all(r[1] for r in res), res
    assert all(r[2] for r in res), res
