"""In-process multi-device Monte-Carlo sample sharding (SURVEY.md §5 "Distributed comm
backend", §8(e) exact mode) for callers that stay one process, as eval.py does (it pins
``cuda:0``, experiments/eval.py:112-114).

    import pertrenderer_amd as pa
    pa.set_sample_devices(["cuda:0", "cuda:1", ...])
    # or, with eval.py's source unchanged:  PR_SAMPLE_DEVICES=all python experiments/eval.py

Every ``smooth_rgb_blend`` of a native Monte-Carlo pair (GaussianRast / ArctanRast /
*_wovr x GaussianAgg / CauchyAgg / *_wovr), and RandomSimpleShader's fused TexturesVertex blend,
then splits its Sr rast and Sa agg samples over the devices (``parallel.sample_shard``: global
sample indices, one Philox key per operator as on one device, host keys or a graph-mode
``DeviceSeed``) and assembles the full-S estimator with in-process collectives:

  forward : fragments broadcast to the devices; each device's perturbed Heaviside counts over
            its rast shard are summed on the primary as integers (P = sum_i C_i / Sr, the
            one-device P bit for bit) and P is broadcast back; each device runs the fused blend
            kernel on P (prob input, PR_BLEND_RAST off) over its agg shard -- texel or vertex
            colours -- and its per-sample winners are gathered on the primary, whose
            PR_BLEND_WINNERS_IN launch forms the image from all Sa winners: the one-device
            fused image bit for bit (same win counts, same colour mix);
  backward: the image is sum_i (n_i / Sa) rgb_i (+ alpha, which every shard computes alike), so
            shard i's fused backward takes (n_i / Sa) g_rgb (and g_alpha on the primary only);
            the adjoints of the broadcasts / count sum carry d P to the Heaviside shards:
            d dists, d zbuf, d colours / d bary / d vertex colours and the smoothing scalars'
            gradients are the full-S ones up to the summation order of the shards' partials.

The collectives are ``torch.cuda.comm`` broadcast / reduce_add, i.e. RCCL (ncclCommInitAll)
over xGMI when the devices are distinct GPUs; logical shards on one device (tests, one-GPU
boxes) copy instead.  This is the north star's sample partition without torchrun; the torchrun
paths (``parallel.py``, bench.py) remain the measured multi-GPU configuration.
"""
import os
import warnings

import torch
import torch.cuda.comm as _comm

from . import _native as nat
from . import noise as noise_mod
from .noise import Noise
from .parallel import sample_shard

_DEVICES = None


def set_sample_devices(devices):
    """Shard every native Monte-Carlo blend's samples over `devices` (None or one device: off).
    The first device is the primary: fragments, colours and the image live there."""
    global _DEVICES
    if devices is None:
        _DEVICES = None
        return
    devs = [torch.device(d) for d in devices]
    if any(d.type != "cuda" for d in devs):
        raise ValueError("sample devices must be ROCm devices")
    devs = [torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device()) for d in devs]
    _DEVICES = devs if len(devs) > 1 else None


def sample_devices():
    return _DEVICES


def devices_from_env(value=None):
    """The device list of PR_SAMPLE_DEVICES ("all", a count "8", or a list "0,1,2,3" /
    "cuda:0,cuda:1"), or None when unset / empty.  Counting devices does not initialise HIP."""
    value = os.environ.get("PR_SAMPLE_DEVICES", "") if value is None else value
    value = value.strip()
    if not value:
        return None
    if value.lower() == "all":
        n = torch.cuda.device_count()
        return [f"cuda:{i}" for i in range(n)] if n > 1 else None
    if value.isdigit():
        n = min(int(value), torch.cuda.device_count())
        return [f"cuda:{i}" for i in range(n)] if n > 1 else None
    items = [v.strip() for v in value.split(",") if v.strip()]
    devs = [v if v.startswith("cuda") else f"cuda:{int(v)}" for v in items]
    n = torch.cuda.device_count()  # 0 on a host without GPUs: nothing to check against there
    bad = [d for d in devs if n > 0 and torch.device(d).index is not None and torch.device(d).index >= n]
    if bad:
        raise ValueError(f"PR_SAMPLE_DEVICES names {bad}, but this process sees {n} GPU(s)")
    return devs


def activate_from_env():
    """set_sample_devices(PR_SAMPLE_DEVICES), run at import: eval.py (which pins cuda:0 and stays
    one process, eval.py:112-116) shards its Monte-Carlo samples over the node's GPUs with no
    change to its source -- `PR_SAMPLE_DEVICES=all python experiments/eval.py ...`."""
    devs = devices_from_env()
    if devs is not None and int(os.environ.get("WORLD_SIZE", "1") or 1) > 1:
        # a torchrun rank owns its LOCAL_RANK device: sharding its samples over every GPU from cuda:0
        # would collide with the other ranks (bench.py / parallel.py shard across processes instead)
        warnings.warn("PR_SAMPLE_DEVICES is ignored in a multi-process job (WORLD_SIZE > 1)", RuntimeWarning)
        return None
    if devs is not None:
        set_sample_devices(devs)
    return devs


def _distinct(devs):
    return len(set(devs)) == len(devs)


def _broadcast(x, devices):
    if len(devices) > 1 and _distinct(devices) and x.device in devices:
        src = devices.index(x.device)
        order = [devices[src]] + [d for i, d in enumerate(devices) if i != src]
        outs = _comm.broadcast(x.contiguous(), devices=order)  # RCCL broadcast
        back = dict(zip(order, outs))
        return [back[d] for d in devices]
    return [x.view_as(x) if d == x.device else x.to(d) for d in devices]  # distinct outputs


def _reduce_add(xs, dst):
    devs = [x.device for x in xs]
    if len(devs) > 1 and _distinct(devs) and dst in devs:
        return _comm.reduce_add([x.contiguous() for x in xs], destination=dst)  # RCCL reduce
    out = xs[0].to(dst, copy=True)
    for x in xs[1:]:
        out.add_(x.to(dst))
    return out


class _Broadcast(torch.autograd.Function):
    """x -> one copy per device; backward: the sum of the copies' gradients on x's device."""

    @staticmethod
    def forward(ctx, devices, x):
        ctx.src = x.device
        return tuple(_broadcast(x.detach(), devices))

    @staticmethod
    def backward(ctx, *gs):
        gs = [g for g in gs if g is not None]
        return None, (_reduce_add(gs, ctx.src) if gs else None)


class _WeightedReduce(torch.autograd.Function):
    """(x_i on device i) -> sum_i w_i x_i on dst; backward: w_i * g broadcast to device i."""

    @staticmethod
    def forward(ctx, dst, weights, *xs):
        ctx.devs, ctx.weights = [x.device for x in xs], weights
        return _reduce_add([x.detach() * w for x, w in zip(xs, weights)], dst)

    @staticmethod
    def backward(ctx, g):
        gs = _broadcast(g.detach(), ctx.devs)
        return (None, None) + tuple(gi * w for gi, w in zip(gs, ctx.weights))


class _CountReduce(torch.autograd.Function):
    """(P_i on device i, P_i = C_i / n_i) -> (sum_i C_i) / Sr on dst with the integer counts
    C_i = round(n_i P_i) summed exactly (the one-device P bit for bit); backward: the adjoint of
    sum_i (n_i / Sr) P_i, i.e. (n_i / Sr) g broadcast to device i."""

    @staticmethod
    def forward(ctx, dst, ns, Sr, *ps):
        ctx.devs, ctx.weights = [x.device for x in ps], [n / Sr for n in ns]
        counts = [torch.round(x.detach() * float(n)) for x, n in zip(ps, ns)]
        return _reduce_add(counts, dst) / float(Sr)

    @staticmethod
    def backward(ctx, g):
        gs = _broadcast(g.detach(), ctx.devs)
        return (None, None, None) + tuple(gi * w for gi, w in zip(gs, ctx.weights))


class _ShardImages(torch.autograd.Function):
    """image (the primary's PR_BLEND_WINNERS_IN image) standing for sum_i w_i rgb_i (+ alpha): the
    forward returns `image`; the backward hands shard i the gradient of w_i rgb_i, and the alpha
    gradient to shard 0 only (every shard's alpha is the same function of P)."""

    @staticmethod
    def forward(ctx, image, weights, *shard_images):
        ctx.devs, ctx.weights = [x.device for x in shard_images], weights
        return image

    @staticmethod
    def backward(ctx, g):
        out = []
        for i, (d, w) in enumerate(zip(ctx.devs, ctx.weights)):
            gi = g.detach().to(d, copy=True)
            gi[..., :3] *= w
            if i:
                gi[..., 3] = 0.0
            out.append(gi)
        return (None, None) + tuple(out)


def _seeds_on(noise, devices):
    """The DeviceSeed base of `noise` on every device (the tensor itself on its own device)."""
    s = noise.seeds
    if s is None:
        return [None] * len(devices)
    return [s if d == s.device else s.to(d) for d in devices]


def sharded_blend(colors, pix_to_face, dists, zbuf, sigma, gamma, alpha, nb_samples_rast, nb_samples_agg,
                  devices=None, eps=1e-10, background=(1.0, 1.0, 1.0), znear=1.0, zfar=100.0, fixed_noise=False,
                  rast_kind="gaussian", rast_vr=True, agg_kind="gaussian", agg_vr=True, vert_colors=None, faces=None):
    """smooth_rgb_blend (random_rasterizer.py:34-56) of a native Monte-Carlo pair with its samples
    split over `devices` (default: set_sample_devices) -- see the module docstring.  With
    vert_colors / faces, `colors` are the fragments' barycentrics and the slot colours are the
    fused TexturesVertex sampling's (RandomSimpleShader, random_rasterizer.py:164-177)."""
    from .blend import (_FusedBlendFn, _FusedVertexBlendFn, _background, _counts_for, image_from_winners,
                        perturbed_heaviside, variant_flags)
    from .renderer.rasterizer import attach_valid_counts
    devices = [torch.device(d) for d in (devices or _DEVICES or [pix_to_face.device])]
    primary = pix_to_face.device
    if devices[0] != primary:
        raise ValueError(f"the first sample device ({devices[0]}) must hold the fragments ({primary})")
    vertex = vert_colors is not None
    shape = tuple(pix_to_face.shape)
    N, H, W, K = shape
    # one key per operator, drawn as the one-device path draws them (rast, then agg)
    nr = noise_mod.draw_rast(shape, nb_samples_rast, primary, rast_kind)
    na = noise_mod.draw_agg((N, H, W, K + 1), nb_samples_agg, primary, fixed_noise, agg_kind)
    if nr.mode != nat.PR_NOISE_PHILOX or na.mode != nat.PR_NOISE_PHILOX:
        raise NotImplementedError("sample sharding over devices needs Philox noise (not the 'torch' noise source)")
    n = len(devices)
    sh_r = [sample_shard(nb_samples_rast, i, n) for i in range(n)]
    sh_a = [sample_shard(nb_samples_agg, i, n) for i in range(n)]
    if any(c == 0 for _, c in sh_r + sh_a):
        raise ValueError(f"{n} sample devices need >= {n} rast and agg samples "
                         f"(Sr={nb_samples_rast}, Sa={nb_samples_agg})")
    counts = _counts_for(pix_to_face)
    p2f_b = _broadcast(pix_to_face, devices)
    if counts is not None:  # the valid-prefix counts travel with the fragments
        for p2f_i, c_i in zip(p2f_b, _broadcast(counts, devices)):
            attach_valid_counts(p2f_i, c_i)
    mask_b = [p >= 0 for p in p2f_b]
    d_b = _Broadcast.apply(devices, dists)
    z_b = _Broadcast.apply(devices, zbuf)
    c_b = _Broadcast.apply(devices, colors)
    v_b = _Broadcast.apply(devices, vert_colors) if vertex else [None] * n
    f_b = _broadcast(faces, devices) if vertex else [None] * n
    sr_b, sa_b = _seeds_on(nr, devices), _seeds_on(na, devices)
    # ---- rast shards -> P: exact integer counts summed on the primary
    # device smoothing scalars are read by pointer: each shard's from its own device (a
    # differentiable copy); CPU leaves and floats go by value
    on = lambda x, d: x.to(d) if torch.is_tensor(x) and x.is_cuda and x.device != d else x
    P_i = [perturbed_heaviside(d_b[i], on(sigma, devices[i]), sh_r[i][1],
                               noise=Noise.philox(seed_r=nr.seed_r, offset_r=nr.offset_r + sh_r[i][0], seeds=sr_b[i]),
                               kind=rast_kind, variance_reduction=rast_vr) * mask_b[i] for i in range(n)]
    P = _CountReduce.apply(primary, [c for _, c in sh_r], nb_samples_rast, *P_i)
    P_b = _Broadcast.apply(devices, P)
    # ---- agg shards: the fused blend on P (prob input) over each shard's samples
    vflags = variant_flags(rast_kind, rast_vr, agg_kind, agg_vr)
    bg = _background(background)
    sink = []
    images = []
    for i, d in enumerate(devices):
        cfg = dict(Sr=nb_samples_rast, Sa=sh_a[i][1], eps=float(eps), bg=bg, vflags=vflags,
                   counts=_counts_for(p2f_b[i]), prob_in=True, winners_sink=sink,
                   noise=Noise.philox(seed_a=na.seed_a, offset_a=na.offset_a + sh_a[i][0], seeds=sa_b[i]))
        zn = znear.to(d) if torch.is_tensor(znear) else znear
        zf = zfar.to(d) if torch.is_tensor(zfar) else zfar
        sc = [on(x, d) for x in (sigma, gamma, alpha)]
        if vertex:
            images.append(_FusedVertexBlendFn.apply(P_b[i], z_b[i], c_b[i], v_b[i], *sc, None, p2f_b[i], f_b[i], zn,
                                                    zf, cfg))
        else:
            images.append(_FusedBlendFn.apply(P_b[i], z_b[i], c_b[i], *sc, None, p2f_b[i], zn, zf, cfg))
    # ---- the image from every sample's winner on the primary (the one-device image bit for bit)
    winners = torch.cat([w.to(primary) for w in sink], dim=1)
    with torch.no_grad():
        image = image_from_winners(P.detach(), zbuf.detach(), colors.detach(), pix_to_face, winners,
                                   gamma.detach() if torch.is_tensor(gamma) else gamma,
                                   alpha.detach() if torch.is_tensor(alpha) else alpha, eps=eps,
                                   background=bg, znear=znear, zfar=zfar,
                                   vert_colors=vert_colors.detach() if vertex else None, faces=faces)
    return _ShardImages.apply(image, [c / nb_samples_agg for _, c in sh_a], *images)
