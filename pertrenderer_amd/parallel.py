"""Data-parallel helpers: Monte-Carlo sample sharding and the single gradient reduction.

The north-star parallel axis is the Monte-Carlo sample dimension:
every rank renders the same frame with a disjoint range of global sample indices
(Philox counters are keyed by the global index, ``Noise.philox(offset_r=..,
offset_a=..)``), then ONE flattened all-reduce (RCCL over xGMI with the "nccl"
backend, gloo on CPU) averages the gradients.  Frame-parallel (weak-scaling)
training uses the same reduction with one frame per rank (bench.py).
"""
import torch
import torch.distributed as dist

from .noise import Noise


def sample_shard(S, rank, world, align=4):
    """(offset, count) of `rank`'s share of S samples.  Shards are contiguous, cover
    [0, S) exactly, and start on Philox-group boundaries (multiples of `align`) when
    S allows, so no 4-sample Philox block is split between ranks."""
    if S <= 0 or world <= 0 or not 0 <= rank < world:
        raise ValueError("bad shard request")
    groups = (S + align - 1) // align
    g0 = (groups * rank) // world
    g1 = (groups * (rank + 1)) // world
    lo, hi = min(S, g0 * align), min(S, g1 * align)
    return lo, hi - lo


def shard_noise(seed_r, seed_a, Sr, Sa, rank, world):
    """Noise for this rank's shard plus its local sample counts: (noise, Sr_local, Sa_local)."""
    off_r, n_r = sample_shard(Sr, rank, world)
    off_a, n_a = sample_shard(Sa, rank, world)
    return Noise.philox(seed_r=seed_r, seed_a=seed_a, offset_r=off_r, offset_a=off_a), n_r, n_a


def average_gradients(params, group=None, weight=None):
    """One flattened all-reduce of every gradient (the step's only collective).

    weight: this rank's share of the estimator (e.g. local samples / total samples);
    None averages uniformly.  CPU-resident grads (the reference's 0-d smoothing
    leaves) ride along in the same buffer."""
    world = dist.get_world_size(group)
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    dev = next((g.device for g in grads if g.device.type != "cpu"), torch.device("cpu"))
    flat = torch.cat([g.detach().reshape(-1).to(dev, torch.float32) for g in grads])
    if weight is not None:
        flat.mul_(float(weight))
    dist.all_reduce(flat, group=group)
    if weight is None:
        flat.div_(world)
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].reshape(g.shape).to(g.device, g.dtype))
        off += n
