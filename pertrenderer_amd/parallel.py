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
    """(offset, count) of `rank`'s share of S samples.  Shards are contiguous and cover
    [0, S) exactly.  They start on Philox-group boundaries (multiples of `align`) when there
    are at least `world` groups, so no 4-sample Philox block is split between ranks;
    otherwise the split is per sample, so every rank gets >= 1 sample whenever S >= world."""
    if S <= 0 or world <= 0 or not 0 <= rank < world:
        raise ValueError("bad shard request")
    if (S + align - 1) // align < world:
        align = 1
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


def _collective_device(group, tensors=()):
    """Where a collective's buffer must live: a CUDA device for RCCL ("nccl" cannot reduce
    CPU tensors, and the reference's smoothing leaves are CPU 0-d tensors), else the CPU."""
    if dist.get_backend(group) == "gloo":
        return torch.device("cpu")
    return next((t.device for t in tensors if t.is_cuda), torch.device("cuda", torch.cuda.current_device()))


def average_gradients(params, group=None, weight=None):
    """One flattened all-reduce of every gradient (the step's only collective).

    weight: this rank's share of the estimator (e.g. local samples / total samples);
    None averages uniformly.  CPU-resident grads (the reference's 0-d smoothing
    leaves) ride along in the same buffer."""
    world = dist.get_world_size(group)
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    dev = _collective_device(group, grads)
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


# ------------------------------------------------------ exact sample-sharded mode
# SURVEY.md §8(e) "exact mode": every rank renders the same frame with its shard of the
# Monte-Carlo samples, and the collectives make the result the full-S estimator (the same
# values as one GPU up to fp summation order), not an average of per-rank estimators:
#   forward : all-reduce of the rast probabilities P (counts) and of the agg weights W;
#   backward: all-reduce of dL/dP (the agg shards' contributions) and of dL/d dists and
#             dL/d zbuf; the smoothing scalars' per-rank partials are completed after the
#             backward by reduce_scalar_grads (only the part accumulated since its last call).
# Built from the standalone native ops (perturbed_heaviside / perturbed_aggregate), the
# colour blend in torch: it serves the large-S configurations, where the messages
# (N,H,W,K) are small against the per-rank RNG work.

def _all_reduce_sum(t, group):
    """In-place SUM all-reduce of `t`, staged through the collective's device when it lives
    elsewhere (gloo reduces host copies of CUDA tensors; RCCL device copies of CPU tensors)."""
    dev = _collective_device(group, (t,))
    if t.device != dev:
        c = t.detach().to(dev)
        dist.all_reduce(c, group=group)
        t.copy_(c)
    else:
        dist.all_reduce(t, group=group)
    return t


class _SumForward(torch.autograd.Function):
    """y = sum over ranks of weight_r * x_r.  The gradient arriving at y is the same on
    every rank, so x_r's gradient is weight_r * dy (no collective)."""

    @staticmethod
    def forward(ctx, x, weight, group):
        ctx.weight = weight
        return _all_reduce_sum(x.detach() * weight, group)

    @staticmethod
    def backward(ctx, g):
        return g * ctx.weight, None, None


class _SumBackward(torch.autograd.Function):
    """Identity forward; the backward sums the rank-local gradients (each rank's shard
    contributes its own part of dL/dx)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return _all_reduce_sum(g.detach().clone(memory_format=torch.contiguous_format), ctx.group), None


def exact_sharded_blend(colors, pix_to_face, dists, zbuf, sigma, gamma, alpha, nb_samples_rast, nb_samples_agg,
                        seed_r, seed_a, eps=1e-10, background=(1.0, 1.0, 1.0), znear=1.0, zfar=100.0,
                        group=None):
    """smooth_rgb_blend (random_rasterizer.py:34-56) with GaussianRast / GaussianAgg over
    `nb_samples_*` GLOBAL samples split across the ranks of `group` (sample_shard): the
    image and the gradients of colors, dists and zbuf equal the single-process full-S
    result up to fp summation order (P and W are exact: counts).  Call reduce_scalar_grads
    after each backward for sigma / gamma / alpha (tracked here; their leaves are CPU tensors: a collective
    inside their backward nodes would run on autograd's CPU thread, unordered against the
    device-thread collectives, so the ranks could disagree on the collective order)."""
    from .blend import perturbed_aggregate, perturbed_heaviside
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    off_r, n_r = sample_shard(nb_samples_rast, rank, world)
    off_a, n_a = sample_shard(nb_samples_agg, rank, world)
    if n_r == 0 or n_a == 0:
        raise ValueError(f"exact sharding needs >= 1 sample per rank (Sr={nb_samples_rast}, "
                         f"Sa={nb_samples_agg}, world={world})")
    K = dists.shape[-1]
    track_scalar_grads([t for t in (sigma, gamma, alpha) if torch.is_tensor(t)])
    mask = pix_to_face >= 0
    d_in = _SumBackward.apply(dists, group)
    z_in = _SumBackward.apply(zbuf, group)
    P_r = perturbed_heaviside(d_in, sigma, n_r, noise=Noise.philox(seed_r=seed_r, offset_r=off_r))
    P = _SumForward.apply(P_r * mask, n_r / nb_samples_rast, group)  # smooth_rgb_blend :47
    P_in = _SumBackward.apply(P, group)
    W_r = perturbed_aggregate(z_in, zfar, znear, P_in, mask, gamma, alpha, n_a, eps=eps,
                              noise=Noise.philox(seed_a=seed_a, offset_a=off_a))
    W = _SumForward.apply(W_r, n_a / nb_samples_agg, group)
    bg = torch.as_tensor(background, dtype=colors.dtype, device=colors.device)
    rgb = (W[..., :K, None] * colors).sum(dim=-2) + W[..., K:K + 1] * bg  # :50-53
    a = 1.0 - torch.prod(1.0 - P, dim=-1, keepdim=True)  # :48, :54
    return torch.cat([rgb, a], dim=-1)


def track_scalar_grads(params):
    """Record, per smoothing leaf, the gradient each backward delivers to it (a tensor hook), so
    reduce_scalar_grads completes exactly what arrived since its last call -- whatever the caller
    did to ``.grad`` in between.  eval.py replaces sigma / gamma / alpha.grad with zeros after
    every iteration past 100 (eval.py:386) and optimizer.zero_grad() resets grads too; a
    subtraction of the last reduced total would then be wrong.  Idempotent;
    exact_sharded_blend calls it for its leaves."""
    for p in params:
        if p is None or not p.requires_grad or not p.is_leaf or getattr(p, "_pr_tracked", False):
            continue

        def hook(g, p=p):
            g = g.detach().reshape(()).to(torch.float32)
            p._pr_pending = g.clone() if p._pr_pending is None else p._pr_pending + g.to(p._pr_pending.device)

        p._pr_pending = None
        p.register_hook(hook)
        p._pr_tracked = True


def reduce_scalar_grads(params, group=None):
    """Exact mode: complete the smoothing scalars' gradients after a backward.  Each rank holds
    its shard's partial; the partials that backward delivered to a leaf since the last call
    (track_scalar_grads) are all-reduced (SUM) and the other ranks' share is added to ``.grad``,
    so the leaf ends as in one process whether it accumulates across iterations or is zeroed /
    replaced in between (eval.py:382-388).  An untracked leaf's whole ``.grad`` counts as this
    backward's partial.  One collective for all leaves, staged on the device for RCCL (the
    leaves are CPU 0-d tensors)."""
    leaves = [p for p in params if p is not None and p.grad is not None]
    if not leaves:
        return
    local = []
    for p in leaves:
        if getattr(p, "_pr_tracked", False):
            pend = p._pr_pending
            local.append(pend if pend is not None else torch.zeros((), dtype=torch.float32))
        else:
            local.append(p.grad.detach().reshape(()).to(torch.float32))
    dev = local[0].device
    flat = torch.stack([t.to(dev) for t in local])
    mine = flat.clone()
    _all_reduce_sum(flat, group)
    for p, total, own in zip(leaves, flat, mine):
        with torch.no_grad():
            p.grad.add_((total - own).to(p.grad.device, p.grad.dtype).reshape(p.grad.shape))
        if getattr(p, "_pr_tracked", False):
            p._pr_pending = None
