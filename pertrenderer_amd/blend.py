"""Autograd operators over the native perturbed-blend kernels.

* :func:`perturbed_blend`      — fused smooth_rgb_blend with GaussianRast + GaussianAgg
  (random_rasterizer.py:34-56 + smoothrast.py:12-59 + smoothagg.py:10-73,185-205):
  one pr_blend_fwd / pr_blend_bwd launch pair per render.
* :func:`perturbed_heaviside`  — GaussianRast.rasterize standalone (smoothrast.py:144-147).
* :func:`perturbed_aggregate`  — GaussianAgg.aggregate standalone (smoothagg.py:196-205).

Gradients follow the reference's custom backward passes, including
its quirks: d sigma = sum(gmaps * dP) (smoothrast.py:57-58) and |eps|^2 over all K+1
logits in d gamma (smoothagg.py:54).  sigma / gamma / alpha may be CPU 0-d leaves
(smoothrast.py:116, smoothagg.py:153-154: values passed by value, gradients returned
as 0-d tensors that autograd moves to the CPU) or device tensors (passed by pointer:
no host synchronisation, so the step can be captured in a HIP graph).
"""
import collections
import os
import threading

import torch

from . import _native as nat
from . import host_layer
from . import noise as noise_mod
from . import timing as _timing
from .noise import Noise

F32 = torch.float32
_ABS = 1 << 63  # absolute-key marker (see PRBlendParams.seeds)


_PLANE_CACHE = collections.OrderedDict()
_PLANE_CACHE_MAX = 16  # LRU: a caller scheduling float planes per step does not grow it without bound


def _planes(z, N, device):
    """znear / zfar as an (N,) float32 device tensor (accepts float, (N,), (N,1,1,1)).  Plain
    floats (the cameras' defaults) are made once per (value, N, device): no fill kernel per render."""
    if not torch.is_tensor(z):
        key = (float(z), N, str(device))
        t = _PLANE_CACHE.get(key)
        if t is None:
            t = _PLANE_CACHE[key] = torch.full((N,), float(z), dtype=F32, device=device)
            while len(_PLANE_CACHE) > _PLANE_CACHE_MAX:
                _PLANE_CACHE.popitem(last=False)
        else:
            _PLANE_CACHE.move_to_end(key)
        return t
    if torch.is_tensor(z):
        if z.dtype is F32 and z.device == device and z.numel() == N:  # the cameras' (N,) planes: a view
            r = z.detach().reshape(N)
            if r.is_contiguous():
                return r
        z = z.detach().to(device=device, dtype=F32).reshape(-1)
        if z.numel() == 1:
            z = z.expand(N)
        if z.numel() != N:
            raise ValueError(f"znear/zfar must have N={N} entries, got {z.numel()}")
        return z.contiguous()
    return torch.full((N,), float(z), dtype=F32, device=device)


def _background(bg):
    if torch.is_tensor(bg):
        bg = bg.detach().cpu().reshape(-1).tolist()
    bg = [float(v) for v in bg]
    if len(bg) != 3:
        raise ValueError("background_color must have 3 entries")
    return bg


def _contig(t, dtype=F32):
    return nat.dense(t, dtype)


def _scalars(vals, device):
    """(host floats, device 0-d tensors or None) for the smoothing scalars.  When every tensor
    input lives on the device they are passed by pointer to their own storage (capture-safe,
    no stacking kernel); plain floats stay by-value.  Otherwise values are read on the host."""
    tens = [v for v in vals if torch.is_tensor(v)]
    if tens and all(v.is_cuda for v in tens):
        dev = [v.detach().reshape(()).to(F32) if torch.is_tensor(v) else None for v in vals]
        return tuple(0.0 if torch.is_tensor(v) else float(v) for v in vals), dev
    return tuple(float(v.detach().cpu()) if torch.is_tensor(v) else float(v) for v in vals), None


KINDS = ("gaussian", "cauchy", "uniform")  # uniform: UniformAgg's forward only


def variant_flags(rast_kind="gaussian", rast_vr=True, agg_kind="gaussian", agg_vr=True):
    """PR_BLEND_* noise-variant bits: ArctanRast (Cauchy rast), GaussianRast_wovr, CauchyAgg,
    GaussianAgg_wovr."""
    for k in (rast_kind, agg_kind):
        if k not in KINDS:
            raise NotImplementedError(f"noise type {k!r} not implemented (gaussian, cauchy, uniform)")
    if rast_kind == "uniform":
        raise NotImplementedError("uniform noise exists for the aggregation only (smoothagg.py:28-30)")
    f = 0
    f |= nat.PR_BLEND_RAST_CAUCHY if rast_kind == "cauchy" else 0
    f |= nat.PR_BLEND_AGG_CAUCHY if agg_kind == "cauchy" else 0
    f |= nat.PR_BLEND_AGG_UNIFORM if agg_kind == "uniform" else 0
    f |= 0 if rast_vr else nat.PR_BLEND_RAST_WOVR
    f |= 0 if agg_vr else nat.PR_BLEND_AGG_WOVR
    return f


def _params(shape, Sr, Sa, sc, sc_dev, eps, bg, noise, znear, zfar, flags):
    N, H, W, K = shape
    p = nat.PRBlendParams()
    p.N, p.H, p.W, p.K = N, H, W, K
    p.Sr, p.Sa = int(Sr), int(Sa)
    p.sample_offset_r, p.sample_offset_a = noise.offset_r, noise.offset_a
    p.sigma, p.gamma, p.alpha, p.eps = sc[0], sc[1], sc[2], eps
    for i in range(3):
        p.background[i] = bg[i]
    p.noise_mode = noise.mode
    p.seed_r, p.seed_a = noise.seed_r & (2 ** 64 - 1), noise.seed_a & (2 ** 64 - 1)
    p.noise_r, p.noise_a = nat.ptr(noise.noise_r), nat.ptr(noise.noise_a)
    p.znear, p.zfar = nat.ptr(znear), nat.ptr(zfar)
    p.flags = flags
    for i in range(3):
        p.scalars[i] = nat.ptr(sc_dev[i]) if sc_dev is not None and i < len(sc_dev) else None
    p.seeds = nat.ptr(noise.seeds)
    return p


def _check_injected(noise, Sr, Sa, shape, need_r, need_a):
    if noise.mode != nat.PR_NOISE_INJECTED:
        return
    N, H, W, K = shape
    if need_r and (noise.noise_r is None or tuple(noise.noise_r.shape) != (Sr, N, H, W, K)):
        raise ValueError(f"injected noise_r must have shape {(Sr, N, H, W, K)}")
    if need_a and (noise.noise_a is None or tuple(noise.noise_a.shape) != (Sa, N, H, W, K + 1)):
        raise ValueError(f"injected noise_a must have shape {(Sa, N, H, W, K + 1)}")


def _merge(nr, na):
    """One Noise for the fused call from the rast draw and the agg draw."""
    if nr.mode != na.mode:
        raise ValueError("rast and agg noise must use the same source")
    seeds = nr.seeds if nr.seeds is not None else na.seeds
    seed_r, seed_a = nr.seed_r, na.seed_a
    if seeds is not None:  # a host-keyed draw next to a device-seeded one keeps its key verbatim
        seed_r = seed_r if nr.seeds is not None else seed_r | _ABS
        seed_a = seed_a if na.seeds is not None else seed_a | _ABS
    return Noise(nr.mode, seed_r, seed_a, nr.noise_r, na.noise_a, nr.offset_r, na.offset_a, seeds)


def _scalar_grads(gs, needs, refs):
    """The smoothing scalars' gradients from the kernel's (3,) device buffer.  For the
    reference's CPU 0-d leaves the three values come to the host in ONE copy (autograd would
    otherwise copy each 0-d device grad separately: three host synchronisations per backward)."""
    want = [need and torch.is_tensor(ref) for need, ref in zip(needs, refs)]
    if any(w and ref.device.type == "cpu" for w, ref in zip(want, refs)) and gs.is_cuda:
        host = gs.detach().to("cpu")
        return [(host[i] if ref.device.type == "cpu" else gs[i]).to(dtype=ref.dtype) if w else None
                for i, (w, ref) in enumerate(zip(want, refs))]
    return [gs[i].to(dtype=ref.dtype) if w else None for i, (w, ref) in enumerate(zip(want, refs))]


# ------------------------------------------------ smoothing-scalar gradient link
# The reference's smoothing scalars are CPU 0-d leaves (smoothrast.py:111-123, smoothagg.py:145-163),
# so every backward must bring their gradients to the host: one synchronisation.  Taken inside the
# blend's backward it stalls the host until the GPU has drained, before the rasterizer's backward
# is even launched.  A _ScalarLink node carries them instead: the blend's backward hands it the
# (3,) device buffer plus an event recorded after the kernels that write it, and the link's
# backward waits for that event only (a side-stream copy into pinned memory).  MeshRenderer
# creates the link before the rasterizer (prelink), so autograd, which runs the highest sequence
# number first, reaches it after the rasterizer's backward is launched; the host then waits only
# for the blend's kernels, not for the whole queue.
_LINK = os.environ.get("PR_SCALAR_LINK", "1") != "0"  # 0: the blend's backward copies them itself
_TLS = threading.local()  # per thread: the pending prelink, and per device a side stream + pinned buffer


def _state():
    st = getattr(_TLS, "state", None)
    if st is None:
        st = _TLS.state = {}
    return st


class _ScalarLink(torch.autograd.Function):
    @staticmethod
    def forward(ctx, device, sigma, gamma, alpha):
        ctx.meta = [(t.dtype, t.shape) if torch.is_tensor(t) and t.requires_grad else None
                    for t in (sigma, gamma, alpha)]
        return torch.empty(3, dtype=F32, device=device)  # a conduit: the kernels read host floats

    @staticmethod
    def backward(ctx, g):
        host = _host_copy(g, getattr(g, "_pr_ready", None))
        return (None,) + tuple(host[i].to(m[0]).reshape(m[1]) if m is not None else None
                               for i, m in enumerate(ctx.meta))


def _new_link(device, vals):
    """The link node: the C++ layer's when it is in use (its backward waits for the event the C++
    blend backward records), else _ScalarLink."""
    ext = host_layer.get()
    if ext is not None:
        idx = device.index if device.index is not None else torch.cuda.current_device()
        t = lambda v: v if torch.is_tensor(v) else None
        return ext.scalar_link(t(vals[0]), t(vals[1]), t(vals[2]), idx)
    return _ScalarLink.apply(device, *vals)


def _host_copy(g, ready):
    """g (3,) on the device -> a CPU tensor, waiting only for the event `ready` (when given)."""
    if ready is None or not g.is_cuda:
        return g.detach().to("cpu")
    dev = g.device
    st = _state()
    side = st.get(("side", dev))
    if side is None:
        side = st[("side", dev)] = torch.cuda.Stream(dev)
        st[("pinned", dev)] = torch.empty(3, dtype=F32, pin_memory=True)
    buf = st[("pinned", dev)]
    side.wait_event(ready)
    with torch.cuda.stream(side):
        buf.copy_(g.detach(), non_blocking=True)
    g.record_stream(side)
    side.synchronize()
    return buf.clone()


def _linkable(vals, device):
    if not (_LINK and torch.is_grad_enabled() and device.type == "cuda"):
        return False
    tens = [v for v in vals if torch.is_tensor(v)]
    if not any(t.requires_grad for t in tens) or any(t.device.type != "cpu" or t.numel() != 1 for t in tens):
        return False
    return not torch.cuda.is_current_stream_capturing()


def _key(vals, device):
    return (str(device),) + tuple((id(v), v._version) if torch.is_tensor(v) else v for v in vals)


def prelink(vals, device):
    """Create the link of the smoothing scalars `vals` now (MeshRenderer: before the rasterizer);
    the next native blend of the same scalars on `device` uses it.  Returns a token for drop."""
    if not _linkable(vals, device):
        return None
    key = _key(vals, device)
    _state()["pre"] = (key, _new_link(device, vals), _floats(vals))
    return key


def drop_prelink(token):
    st = _state()
    pre = st.get("pre")
    if token is not None and pre is not None and pre[0] == token:
        del st["pre"]


def prelink_shader(shader, meshes):
    """prelink for a shader holding perturbed smoothing operators (RandomSimpleShader /
    RandomPhongShader); None when it holds none."""
    sr, sa = getattr(shader, "smoothrast", None), getattr(shader, "smoothagg", None)
    if sr is None or sa is None or not hasattr(sr, "sigma") or not hasattr(sa, "gamma"):
        return None
    device = getattr(meshes, "device", None)
    return prelink((sr.sigma, sa.gamma, sa.alpha), torch.device(device)) if device is not None else None


def _floats(vals):
    return tuple(float(v.detach()) if torch.is_tensor(v) else float(v) for v in vals)


def _link_scalars(vals, device):
    """(values, link): with a link, the scalars go to the kernel as host floats and their gradients
    through the link; otherwise the tensors themselves (the blend copies their gradients).  The
    renderer's prelink of the same scalars (same ids and versions: checked linkable when it was
    made, in this forward) is taken with the host values it read."""
    st = _state()
    pre = st.get("pre")
    if pre is not None and pre[0] == _key(vals, device):
        del st["pre"]
        return pre[2], pre[1]
    if not _linkable(vals, device):
        return vals, None
    return _floats(vals), _new_link(device, vals)


def _link_grad(gsc, need):
    """The device gradient buffer for the link, marked with the event after its kernels."""
    if not need:
        return None
    ev = torch.cuda.Event()
    ev.record()
    gsc._pr_ready = ev
    return gsc


_valid_counts = None


class _ZPlaneGrad(torch.autograd.Function):
    """Identity on zbuf whose backward also gives znear / zfar their gradients.  zbuf enters the
    blend only through z_inv = (zfar - zbuf) / (zfar - znear) * mask (smoothagg.py:198), so the
    kernels' d zbuf = -dL/dz_inv / (zfar - znear) at valid slots fixes dL/dz_inv, and then
    d znear = sum -d zbuf (zfar - zbuf) / (zfar - znear), d zfar = sum -d zbuf (zbuf - znear) /
    (zfar - znear) over each image's valid slots.  Used only when a plane requires grad."""

    @staticmethod
    def forward(ctx, zbuf, znear, zfar, valid):
        ctx.save_for_backward(zbuf, valid)
        ctx.planes = (znear, zfar)
        return zbuf.clone()

    @staticmethod
    def backward(ctx, gz):
        if gz is None:
            return None, None, None, None
        zb, valid = ctx.saved_tensors
        N = zb.shape[0]
        zn_in, zf_in = ctx.planes
        zn = _planes(zn_in, N, zb.device).reshape(N, 1, 1, 1)
        zf = _planes(zf_in, N, zb.device).reshape(N, 1, 1, 1)
        d = zf - zn
        g = torch.where(valid, gz, torch.zeros((), dtype=gz.dtype, device=gz.device))
        z = torch.where(valid, zb, zn)  # (masked slots contribute 0 either way; no inf / nan)
        out = []
        for plane, term in ((zn_in, zf - z), (zf_in, z - zn)):
            if torch.is_tensor(plane) and plane.requires_grad:
                per = (-(g * term) / d).sum(dim=(1, 2, 3))  # (N,)
                gp = per.sum() if plane.numel() == 1 else per
                out.append(gp.reshape(plane.shape).to(device=plane.device, dtype=plane.dtype))
            else:
                out.append(None)
        return gz, out[0], out[1], None


def _planes_need_grad(znear, zfar):
    return torch.is_grad_enabled() and any(torch.is_tensor(z) and z.requires_grad for z in (znear, zfar))


def plane_link(zbuf, znear, zfar, pix_to_face=None, mask=None):
    """zbuf, linked to znear / zfar when either requires grad (the native kernels take the planes
    as constants): returns (zbuf, linked).  Valid slots from the rasterizer's counts when attached,
    else pix_to_face >= 0, else `mask`."""
    if not _planes_need_grad(znear, zfar):
        return zbuf, False
    if mask is None:
        counts = _counts_for(pix_to_face)
        K = pix_to_face.shape[-1]
        mask = (torch.arange(K, device=pix_to_face.device) < counts[..., None].long()) if counts is not None \
            else pix_to_face >= 0
    valid = mask.expand(zbuf.shape).to(torch.bool)
    return _ZPlaneGrad.apply(zbuf, znear, zfar, valid), True


def _counts_for(pix_to_face):
    """The native rasterizer's valid-prefix counts of these fragments (int32 (N,H,W) on the same
    device), or None: the kernels then read pix_to_face at every slot."""
    global _valid_counts
    if _valid_counts is None:
        from .renderer.rasterizer import valid_counts as _vc
        _valid_counts = _vc
    c = _valid_counts(pix_to_face)
    if c is None or c.device != pix_to_face.device or tuple(c.shape) != tuple(pix_to_face.shape[:3]):
        return None
    return c.contiguous()


def _plan(lib, p, counts, dev):
    """The entry-balanced segment plan buffer of a fused blend call (None when the library does not
    plan this call: no valid-prefix counts, or a frame above its plan size)."""
    if counts is None:
        return None
    n = lib.pr_blend_plan_size(nat.C.byref(p))
    return torch.empty((n + 3) // 4, dtype=torch.int32, device=dev) if n else None


# The backward's fused scalar reduction (PRBlendFwdArgs.sync: its last workgroup forms d sigma /
# d gamma / d alpha instead of a finalize kernel; PR_BLEND_SYNC=0 restores the kernel).  With a
# release fence per workgroup (an L2 writeback of its XCD) it took cfg 2's blend_bwd from 75 to
# 182 us; fence-free (partials by atomic exchange) the kernel grows ~3 us and the finalize node it
# saves costs ~2 us of graph time: equal in graph mode, one launch fewer per eager backward
# (profiles/r4_experiments.txt).  Bitwise equal either way (tests/test_gpu_fused_finalize.py).
_FUSED_FINALIZE = os.environ.get("PR_BLEND_SYNC", "1") == "1"


def _sync(dev):
    return torch.empty(nat.PR_BLEND_SYNC_BYTES // 4, dtype=torch.int32, device=dev) if _FUSED_FINALIZE else None


def _timed(name, fn):
    hook = _timing.active()
    if hook is not None:
        hook.start(name)
    fn()
    if hook is not None:
        hook.stop(name)


# ============================================================== fused blend
# Keep the per-slot (prob, rast score) of the forward for the backward (8 B/slot of
# HBM) instead of regenerating the rast noise there.  Either way the results are
# bit-identical (tests/test_gpu_blend.py::test_rast_cache_is_bit_identical).  PR_RAST_CACHE=0
# regenerates (measurement knob).
RAST_CACHE = os.environ.get("PR_RAST_CACHE", "1") != "0"


def _no_uniform_grad(vflags):
    """The reference's randomArgmax.backward has no uniform branch and fails on it
    (smoothagg.py:64-70: grad_z stays None): so does every backward here."""
    if vflags & nat.PR_BLEND_AGG_UNIFORM:
        raise NotImplementedError("UniformAgg: the reference implements no gradient for uniform noise "
                                  "(smoothagg.py:64-70)")


class _FusedBlendFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dists, zbuf, colors, sigma, gamma, alpha, link, p2f, znear, zfar, cfg):
        nat.require_device(dists, zbuf, colors, p2f)
        N, H, W, K = p2f.shape
        dev = p2f.device
        p2f_c = nat.dense(p2f, torch.int64)
        d_c, z_c, c_c = _contig(dists), _contig(zbuf), _contig(colors)
        zn, zf = _planes(znear, N, dev), _planes(zfar, N, dev)
        noise = cfg["noise"].to(dev)
        sc, sc_dev = _scalars((sigma, gamma, alpha), dev)
        prob_in = bool(cfg.get("prob_in"))  # `dists` holds the probabilities (multidevice sample shards)
        p = _params((N, H, W, K), cfg["Sr"], cfg["Sa"], sc, sc_dev, cfg["eps"], cfg["bg"], noise, zn, zf,
                    (0 if prob_in else nat.PR_BLEND_RAST) | nat.PR_BLEND_COLOR | cfg["vflags"])
        image = torch.empty((N, H, W, 4), dtype=F32, device=dev)
        winners = torch.empty((N * H * W, cfg["Sa"]), dtype=torch.uint8, device=dev)
        # per-slot (prob, rast score) kept for the backward instead of regenerating rast noise
        soft = bool(cfg["vflags"] & nat.PR_BLEND_SOFT)
        cache = (torch.empty((N, H, W, K, 2), dtype=F32, device=dev)
                 if RAST_CACHE and not soft and not prob_in and any(ctx.needs_input_grad[:7]) else None)
        plan = None if soft else _plan(nat.load(), p, cfg["counts"], dev)
        sync = None if soft else _sync(dev)
        a = nat.PRBlendFwdArgs()
        a.p = p
        a.pix_to_face, a.zbuf, a.colors = nat.ptr(p2f_c), nat.ptr(z_c), nat.ptr(c_c)
        if prob_in:
            a.prob = nat.ptr(d_c)
        else:
            a.dists = nat.ptr(d_c)
        a.image, a.winners, a.rast_cache = nat.ptr(image), nat.ptr(winners), nat.ptr(cache)
        a.pix_count, a.plan, a.sync = nat.ptr(cfg["counts"]), nat.ptr(plan), nat.ptr(sync)
        _timed("blend_fwd", lambda: nat.call("pr_blend_fwd", "pr_blend_fwd", image, a))
        if cfg.get("winners_sink") is not None:
            cfg["winners_sink"].append(winners)
        ctx.save_for_backward(p2f_c, d_c, z_c, c_c, zn, zf, winners, cache, plan, sync)
        ctx.p = p  # the backward's parameter block is the forward's
        ctx.sc_dev = sc_dev
        ctx.cfg, ctx.noise, ctx.sc = cfg, noise, sc
        ctx.refs = (sigma, gamma, alpha)
        return image

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gimg):
        _no_uniform_grad(ctx.cfg.get("vflags", 0))
        p2f_c, d_c, z_c, c_c, zn, zf, winners, cache, plan, sync = ctx.saved_tensors
        sc_dev = ctx.sc_dev
        cfg, noise, sc = ctx.cfg, ctx.noise, ctx.sc
        lib = nat.load()
        N, H, W, K = p2f_c.shape
        dev = p2f_c.device
        p = ctx.p
        g = nat.dense(gimg, F32)
        gd, gz, gc = torch.empty_like(d_c), torch.empty_like(z_c), torch.empty_like(c_c)
        gsc = torch.empty(3, dtype=F32, device=dev)
        a = nat.PRBlendBwdArgs()
        a.p = p
        a.pix_to_face, a.zbuf, a.colors = nat.ptr(p2f_c), nat.ptr(z_c), nat.ptr(c_c)
        a.winners, a.grad_image, a.rast_cache = nat.ptr(winners), nat.ptr(g), nat.ptr(cache)
        a.grad_zbuf, a.grad_colors, a.grad_scalars = nat.ptr(gz), nat.ptr(gc), nat.ptr(gsc)
        if cfg.get("prob_in"):
            a.prob, a.grad_prob = nat.ptr(d_c), nat.ptr(gd)
        else:
            a.dists, a.grad_dists = nat.ptr(d_c), nat.ptr(gd)
        a.pix_count, a.plan, a.sync = nat.ptr(cfg["counts"]), nat.ptr(plan), nat.ptr(sync)
        ws = torch.empty(max(1, lib.pr_blend_bwd_workspace_size(a)), dtype=torch.uint8, device=dev)
        a.workspace, a.workspace_bytes = nat.ptr(ws), ws.numel()
        _timed("blend_bwd", lambda: nat.call("pr_blend_bwd", "pr_blend_bwd", g, a))
        need = ctx.needs_input_grad
        s_g, g_g, a_g = _scalar_grads(gsc, need[3:6], ctx.refs)
        return (gd if need[0] else None, gz if need[1] else None, gc if need[2] else None,
                s_g, g_g, a_g, _link_grad(gsc, need[6]), None, None, None, None)


class _FusedVertexBlendFn(torch.autograd.Function):
    """perturbed_blend with TexturesVertex sampling fused in: slot colours are
    interpolated from per-vertex colours on demand (PR_BLEND_VERTEX); gradients go
    to bary (-> rasterizer backward) and the vertex colours instead of a texel tensor."""

    @staticmethod
    def forward(ctx, dists, zbuf, bary, vert_colors, sigma, gamma, alpha, link, p2f, faces, znear, zfar, cfg):
        nat.require_device(dists, zbuf, bary, vert_colors, p2f, faces)
        N, H, W, K = p2f.shape
        dev = p2f.device
        p2f_c = nat.dense(p2f, torch.int64)
        f_c = nat.dense(faces, torch.int64)
        d_c, z_c, b_c, v_c = _contig(dists), _contig(zbuf), _contig(bary), _contig(vert_colors)
        zn, zf = _planes(znear, N, dev), _planes(zfar, N, dev)
        noise = cfg["noise"].to(dev)
        sc, sc_dev = _scalars((sigma, gamma, alpha), dev)
        prob_in = bool(cfg.get("prob_in"))  # `dists` holds the probabilities (multidevice sample shards)
        flags = (0 if prob_in else nat.PR_BLEND_RAST) | nat.PR_BLEND_COLOR | nat.PR_BLEND_VERTEX | cfg["vflags"]
        p = _params((N, H, W, K), cfg["Sr"], cfg["Sa"], sc, sc_dev, cfg["eps"], cfg["bg"], noise, zn, zf, flags)
        image = torch.empty((N, H, W, 4), dtype=F32, device=dev)
        winners = torch.empty((N * H * W, cfg["Sa"]), dtype=torch.uint8, device=dev)
        need = ctx.needs_input_grad
        cache = (torch.empty((N, H, W, K, 2), dtype=F32, device=dev)
                 if RAST_CACHE and not prob_in and any(need[:8]) else None)
        a = nat.PRBlendFwdArgs()
        a.p = p
        a.pix_to_face, a.zbuf = nat.ptr(p2f_c), nat.ptr(z_c)
        if prob_in:
            a.prob = nat.ptr(d_c)
        else:
            a.dists = nat.ptr(d_c)
        a.bary, a.faces, a.vert_colors = nat.ptr(b_c), nat.ptr(f_c), nat.ptr(v_c)
        a.image, a.winners, a.rast_cache = nat.ptr(image), nat.ptr(winners), nat.ptr(cache)
        plan, sync = _plan(nat.load(), p, cfg["counts"], dev), _sync(dev)
        a.pix_count, a.plan, a.sync = nat.ptr(cfg["counts"]), nat.ptr(plan), nat.ptr(sync)
        _timed("blend_fwd", lambda: nat.call("pr_blend_fwd", "pr_blend_fwd", image, a))
        if cfg.get("winners_sink") is not None:
            cfg["winners_sink"].append(winners)
        ctx.save_for_backward(p2f_c, d_c, z_c, b_c, v_c, f_c, zn, zf, winners, cache, plan, sync)
        ctx.p = p  # the backward's parameter block is the forward's
        ctx.sc_dev = sc_dev
        ctx.cfg, ctx.noise, ctx.sc, ctx.flags = cfg, noise, sc, flags
        ctx.refs = (sigma, gamma, alpha)
        return image

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gimg):
        _no_uniform_grad(ctx.cfg.get("vflags", 0))
        p2f_c, d_c, z_c, b_c, v_c, f_c, zn, zf, winners, cache, plan, sync = ctx.saved_tensors
        sc_dev = ctx.sc_dev
        cfg, noise, sc = ctx.cfg, ctx.noise, ctx.sc
        lib = nat.load()
        N, H, W, K = p2f_c.shape
        dev = p2f_c.device
        p = ctx.p
        need = ctx.needs_input_grad
        g = nat.dense(gimg, F32)
        gd, gz, gb = torch.empty_like(d_c), torch.empty_like(z_c), torch.empty_like(b_c)
        gv = torch.zeros_like(v_c) if need[3] else None
        gsc = torch.empty(3, dtype=F32, device=dev)
        a = nat.PRBlendBwdArgs()
        a.p = p
        a.pix_to_face, a.zbuf = nat.ptr(p2f_c), nat.ptr(z_c)
        a.bary, a.faces, a.vert_colors = nat.ptr(b_c), nat.ptr(f_c), nat.ptr(v_c)
        a.winners, a.grad_image, a.rast_cache = nat.ptr(winners), nat.ptr(g), nat.ptr(cache)
        a.grad_zbuf, a.grad_scalars = nat.ptr(gz), nat.ptr(gsc)
        if cfg.get("prob_in"):
            a.prob, a.grad_prob = nat.ptr(d_c), nat.ptr(gd)
        else:
            a.dists, a.grad_dists = nat.ptr(d_c), nat.ptr(gd)
        a.grad_bary, a.grad_vert_colors = nat.ptr(gb), nat.ptr(gv)
        a.pix_count, a.plan, a.sync = nat.ptr(cfg["counts"]), nat.ptr(plan), nat.ptr(sync)
        ws = torch.empty(max(1, lib.pr_blend_bwd_workspace_size(a)), dtype=torch.uint8, device=dev)
        a.workspace, a.workspace_bytes = nat.ptr(ws), ws.numel()
        _timed("blend_bwd", lambda: nat.call("pr_blend_bwd", "pr_blend_bwd", g, a))
        s_g, g_g, a_g = _scalar_grads(gsc, need[4:7], ctx.refs)
        return (gd if need[0] else None, gz if need[1] else None, gb if need[2] else None, gv,
                s_g, g_g, a_g, _link_grad(gsc, need[7]), None, None, None, None, None)


_SHADE_ROWS = ("ambient", "diffuse_color", "specular_color", "mat_diffuse", "mat_specular", "shininess")


def _phong_args(sh, p2f_c, t):
    """PRShadeArgs of the fused Phong blend (renderer.shading._args over the blend's fragments)."""
    from .renderer.shading import _args
    cfg = dict(p2f=p2f_c, counts=sh["counts"], faces=sh["faces"], mode=sh["mode"], face_uvs=sh["face_uvs"],
               directional=sh["directional"], **sh["rows"])
    return _args(cfg, t)


class _FusedPhongBlendFn(torch.autograd.Function):
    """perturbed_blend with RandomPhongShader's shading fused into the forward (PR_BLEND_PHONG):
    a slot's colour is Phong-shaded only where it wins a sample (TexturesUV / TexturesVertex texel,
    point or directional light), and only the colours the backward reads (winners, each pixel's
    unperturbed argmax) are kept.  Backward: pr_blend_bwd on those (PR_BLEND_COLOR_SPARSE) -> d colours
    -> pr_shade_bwd (its chain rule for the slots with a non-zero d colour only); gradients go to
    dists, zbuf, bary, the vertex positions and normals, the texture, the light and the camera."""

    @staticmethod
    def forward(ctx, dists, zbuf, bary, verts, normals, tex, light, camera, sigma, gamma, alpha, link, p2f, znear,
                zfar, cfg, sh):
        nat.require_device(dists, zbuf, bary, verts, normals, tex, light, camera, p2f)
        N, H, W, K = p2f.shape
        dev = p2f.device
        p2f_c = nat.dense(p2f, torch.int64)
        d_c, z_c = _contig(dists), _contig(zbuf)
        t = dict(bary=_contig(bary), verts=_contig(verts), normals=_contig(normals), tex=_contig(tex),
                 light=_contig(light), camera=_contig(camera))
        zn, zf = _planes(znear, N, dev), _planes(zfar, N, dev)
        noise = cfg["noise"].to(dev)
        sc, sc_dev = _scalars((sigma, gamma, alpha), dev)
        flags = nat.PR_BLEND_RAST | nat.PR_BLEND_COLOR | nat.PR_BLEND_PHONG | cfg["vflags"]
        p = _params((N, H, W, K), cfg["Sr"], cfg["Sa"], sc, sc_dev, cfg["eps"], cfg["bg"], noise, zn, zf, flags)
        need = ctx.needs_input_grad
        any_grad = any(need[:12])
        image = torch.empty((N, H, W, 4), dtype=F32, device=dev)
        winners = torch.empty((N * H * W, cfg["Sa"]), dtype=torch.uint8, device=dev)
        cache = torch.empty((N, H, W, K, 2), dtype=F32, device=dev) if RAST_CACHE and any_grad else None
        # the colours the backward reads, written at those slots only
        colors = torch.empty((N, H, W, K, 3), dtype=F32, device=dev) if any_grad else None
        sync = _sync(dev)
        shade = _phong_args(sh, p2f_c, t)
        a = nat.PRBlendFwdArgs()
        a.p = p
        a.pix_to_face, a.zbuf, a.dists, a.bary = nat.ptr(p2f_c), nat.ptr(z_c), nat.ptr(d_c), nat.ptr(t["bary"])
        a.colors, a.image, a.winners, a.rast_cache = nat.ptr(colors), nat.ptr(image), nat.ptr(winners), nat.ptr(cache)
        a.pix_count, a.sync, a.shade = nat.ptr(cfg["counts"]), nat.ptr(sync), nat.C.addressof(shade)
        _timed("blend_fwd", lambda: nat.call("pr_blend_fwd", "pr_blend_fwd", image, a))
        ctx.save_for_backward(p2f_c, d_c, z_c, zn, zf, winners, cache, sync, colors, *t.values())
        ctx.p, ctx.sc_dev, ctx.cfg, ctx.sh, ctx.noise = p, sc_dev, cfg, sh, noise
        ctx.refs = (sigma, gamma, alpha)
        return image

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gimg):
        _no_uniform_grad(ctx.cfg.get("vflags", 0))
        p2f_c, d_c, z_c, zn, zf, winners, cache, sync, colors, *tv = ctx.saved_tensors
        t = dict(zip(("bary", "verts", "normals", "tex", "light", "camera"), tv))
        cfg, sh = ctx.cfg, ctx.sh
        lib = nat.load()
        dev = p2f_c.device
        need = ctx.needs_input_grad
        g = nat.dense(gimg, F32)
        # 1. blend backward on the sparse colours
        p = nat.PRBlendParams.from_buffer_copy(ctx.p)
        p.flags = (p.flags & ~nat.PR_BLEND_PHONG) | nat.PR_BLEND_COLOR_SPARSE
        gd, gz, gc = torch.empty_like(d_c), torch.empty_like(z_c), torch.empty_like(colors)
        gsc = torch.empty(3, dtype=F32, device=dev)
        a = nat.PRBlendBwdArgs()
        a.p = p
        a.pix_to_face, a.zbuf, a.dists, a.colors = nat.ptr(p2f_c), nat.ptr(z_c), nat.ptr(d_c), nat.ptr(colors)
        a.winners, a.grad_image, a.rast_cache = nat.ptr(winners), nat.ptr(g), nat.ptr(cache)
        a.grad_dists, a.grad_zbuf, a.grad_colors, a.grad_scalars = nat.ptr(gd), nat.ptr(gz), nat.ptr(gc), nat.ptr(gsc)
        a.pix_count, a.sync = nat.ptr(cfg["counts"]), nat.ptr(sync)
        ws = torch.empty(max(1, lib.pr_blend_bwd_workspace_size(a)), dtype=torch.uint8, device=dev)
        a.workspace, a.workspace_bytes = nat.ptr(ws), ws.numel()
        _timed("blend_bwd", lambda: nat.call("pr_blend_bwd", "pr_blend_bwd", g, a))
        # 2. shading backward (the zero-d-colour slots skipped by the kernel)
        keys = ("bary", "verts", "normals", "tex", "light", "camera")
        out = [torch.empty_like(t[k]) if need[2 + i] else None for i, k in enumerate(keys)]
        if any(o is not None for o in out):
            from .renderer.shading import _shade_bwd_args
            sa = _shade_bwd_args(_phong_args(sh, p2f_c, t), sh["mode"], gc, out)
            if p.flags & nat.PR_BLEND_LIVE_ONLY and cfg["counts"] is not None:
                sa.flags |= nat.PR_SHADE_LIVE_ONLY
            wss = None
            if nat.deterministic():
                sa.flags |= nat.PR_DETERMINISTIC
                wss = nat.workspace(lib.pr_shade_bwd_workspace_size(sa), dev)
                sa.workspace, sa.workspace_bytes = nat.ptr(wss), wss.numel()
            nat.call("pr_shade_bwd", "pr_shade_bwd", g, sa)
            del wss
        s_g, g_g, a_g = _scalar_grads(gsc, need[8:11], ctx.refs)
        return (gd if need[0] else None, gz if need[1] else None, *out,
                s_g, g_g, a_g, _link_grad(gsc, need[11]), None, None, None, None, None)


def perturbed_blend_phong(sh, pix_to_face, bary, dists, zbuf, sigma, gamma, alpha, nb_samples_rast,
                          nb_samples_agg, eps=1e-10, background=(1.0, 1.0, 1.0), znear=1.0, zfar=100.0, noise=None,
                          fixed_noise=False, rast_kind="gaussian", rast_vr=True, agg_kind="gaussian", agg_vr=True,
                          live_only=False):
    """smooth_rgb_blend(phong_shading(..., meshes.sample_textures(fragments)), fragments, <Rast>, <Agg>)
    (random_rasterizer.py:99-116) as one native op: `sh` is renderer.shading.phong_inputs(...) (mesh,
    vertex normals, TexturesUV maps or vertex colours, light / material rows, camera centres).  The
    colour of a slot is shaded only where it wins a Monte-Carlo sample.  Differentiable w.r.t.
    dists, zbuf, bary, the vertex positions and normals, the texture, light, camera and the 0-d
    smoothing tensors."""
    shape = tuple(pix_to_face.shape)
    N, H, W, K = shape
    if tuple(bary.shape) != shape + (3,) or tuple(dists.shape) != shape or tuple(zbuf.shape) != shape:
        raise ValueError("bary must be (N,H,W,K,3), dists / zbuf (N,H,W,K)")
    vflags = variant_flags(rast_kind, rast_vr, agg_kind, agg_vr)
    if noise is None:
        pair = noise_mod.draw_pair(shape, nb_samples_rast, nb_samples_agg, pix_to_face.device, fixed_noise, rast_kind,
                                   agg_kind)
        if pair is None:
            pair = (noise_mod.draw_rast(shape, nb_samples_rast, pix_to_face.device, rast_kind),
                    noise_mod.draw_agg((N, H, W, K + 1), nb_samples_agg, pix_to_face.device, fixed_noise, agg_kind))
        noise = _merge(*pair)
    _check_injected(noise, nb_samples_rast, nb_samples_agg, shape, True, True)
    zbuf, linked = plane_link(zbuf, znear, zfar, pix_to_face)
    live_only = live_only and not linked  # the plane link reads d zbuf at every slot
    counts = _counts_for(pix_to_face)
    cfg = dict(Sr=int(nb_samples_rast), Sa=int(nb_samples_agg), eps=float(eps),
               bg=_background(background), noise=noise, vflags=vflags, counts=counts)
    if live_only and counts is not None:  # every consumer reads the valid prefix only (backward: no zero rows)
        cfg["vflags"] |= nat.PR_BLEND_LIVE_ONLY
    sh = dict(sh, counts=counts)
    (sigma, gamma, alpha), link = _link_scalars((sigma, gamma, alpha), pix_to_face.device)
    dev = pix_to_face.device
    ext = host_layer.get()
    if ext is not None:
        sc, sc_dev = _scalars((sigma, gamma, alpha), dev)
        vals = (sigma, gamma, alpha)
        if sc_dev is None or all(d is None or d.data_ptr() == v.data_ptr() for d, v in zip(sc_dev, vals)):
            zn, zf = _planes(znear, N, dev), _planes(zfar, N, dev)
            noise = noise.to(dev)
            flags = nat.PR_BLEND_RAST | nat.PR_BLEND_COLOR | nat.PR_BLEND_PHONG | cfg["vflags"]
            p = _params(shape, cfg["Sr"], cfg["Sa"], sc, sc_dev, cfg["eps"], cfg["bg"], noise, zn, zf, flags)
            tt = lambda v: v if torch.is_tensor(v) else None
            return ext.blend_phong(dists, zbuf, bary, sh["verts"], sh["normals"], sh["tex"], sh["light"], sh["camera"],
                                   tt(sigma), tt(gamma), tt(alpha), link, pix_to_face, sh["faces"], counts,
                                   sh["face_uvs"], [sh["rows"][k] for k in _SHADE_ROWS], zn, zf, noise.noise_r,
                                   noise.noise_a, noise.seeds, nat.C.addressof(p), int(sh["mode"]),
                                   bool(sh["directional"]), RAST_CACHE, _FUSED_FINALIZE)
    return _FusedPhongBlendFn.apply(dists, zbuf, bary, sh["verts"], sh["normals"], sh["tex"], sh["light"],
                                    sh["camera"], sigma, gamma, alpha, link, pix_to_face, znear, zfar, cfg, sh)


def image_from_winners(prob, zbuf, colors, p2f, winners, gamma, alpha, eps=1e-10, background=(1.0, 1.0, 1.0),
                       znear=1.0, zfar=100.0, vert_colors=None, faces=None):
    """The fused blend's image from given per-sample winners (P, Sa) (PR_BLEND_WINNERS_IN): the win
    counts and colour mix of the one-device kernel, so a sample-sharded blend whose shards' winners
    are gathered here gives the one-device image bit for bit.  `colors` are texels (N,H,W,K,3), or
    with vert_colors / faces the barycentrics (N,H,W,K,3) of the fused TexturesVertex sampling.
    Forward only (multidevice.sharded_blend routes the gradients through the shards)."""
    N, H, W, K = p2f.shape
    dev = p2f.device
    Sa = winners.shape[1]
    vertex = vert_colors is not None
    p2f_c = nat.dense(p2f, torch.int64)
    pr_c, z_c, c_c, w_c = _contig(prob), _contig(zbuf), _contig(colors), nat.dense(winners, torch.uint8)
    zn, zf = _planes(znear, N, dev), _planes(zfar, N, dev)
    sc, sc_dev = _scalars((1.0, gamma, alpha), dev)
    flags = nat.PR_BLEND_COLOR | nat.PR_BLEND_WINNERS_IN | (nat.PR_BLEND_VERTEX if vertex else 0)
    p = _params((N, H, W, K), 1, Sa, sc, sc_dev, float(eps), _background(background), Noise.philox(), zn, zf, flags)
    image = torch.empty((N, H, W, 4), dtype=F32, device=dev)
    a = nat.PRBlendFwdArgs()
    a.p = p
    a.pix_to_face, a.prob, a.zbuf = nat.ptr(p2f_c), nat.ptr(pr_c), nat.ptr(z_c)
    if vertex:
        f_c, v_c = nat.dense(faces, torch.int64), _contig(vert_colors)
        a.bary, a.faces, a.vert_colors = nat.ptr(c_c), nat.ptr(f_c), nat.ptr(v_c)
    else:
        a.colors = nat.ptr(c_c)
    a.image, a.winners, a.pix_count = nat.ptr(image), nat.ptr(w_c), nat.ptr(_counts_for(p2f))
    nat.call("pr_blend_fwd", "pr_blend_fwd", image, a)
    return image


def _fused(vertex, dists, zbuf, colors, vert_colors, sigma, gamma, alpha, link, p2f, faces, znear, zfar, cfg):
    """The fused blend node: the C++ layer's (host_layer.py) when it is in use, else the Python
    Function.  Both pack the same PRBlendParams and launch the same kernels."""
    ext = host_layer.get()
    if ext is not None:
        tensors = [dists, zbuf, colors, p2f] + ([vert_colors, faces] if vertex else [])
        if all(t.is_cuda for t in tensors):
            dev = p2f.device
            N = p2f.shape[0]
            sc, sc_dev = _scalars((sigma, gamma, alpha), dev)
            vals = (sigma, gamma, alpha)
            # device scalars are read by pointer in the backward too: only leaves whose own storage
            # the pointer addresses (float32 0-d) are kept alive by the node
            if sc_dev is None or all(d is None or d.data_ptr() == v.data_ptr() for d, v in zip(sc_dev, vals)):
                zn, zf = _planes(znear, N, dev), _planes(zfar, N, dev)
                noise = cfg["noise"].to(dev)
                flags = nat.PR_BLEND_RAST | nat.PR_BLEND_COLOR | cfg["vflags"]
                flags |= nat.PR_BLEND_VERTEX if vertex else 0
                p = _params(tuple(p2f.shape), cfg["Sr"], cfg["Sa"], sc, sc_dev, cfg["eps"], cfg["bg"], noise, zn, zf,
                            flags)
                t = lambda v: v if torch.is_tensor(v) else None
                return ext.blend(dists, zbuf, colors, vert_colors, t(sigma), t(gamma), t(alpha), link, p2f, faces,
                                 cfg["counts"], zn, zf, noise.noise_r, noise.noise_a, noise.seeds,
                                 nat.C.addressof(p), RAST_CACHE, _FUSED_FINALIZE)
    if vertex:
        return _FusedVertexBlendFn.apply(dists, zbuf, colors, vert_colors, sigma, gamma, alpha, link, p2f, faces,
                                         znear, zfar, cfg)
    return _FusedBlendFn.apply(dists, zbuf, colors, sigma, gamma, alpha, link, p2f, znear, zfar, cfg)


def perturbed_blend_vertex(vert_colors, faces, pix_to_face, bary, dists, zbuf, sigma, gamma, alpha,
                           nb_samples_rast, nb_samples_agg, eps=1e-10, background=(1.0, 1.0, 1.0), znear=1.0,
                           zfar=100.0, noise=None, fixed_noise=False, rast_kind="gaussian", rast_vr=True,
                           agg_kind="gaussian", agg_vr=True, live_only=False):
    """perturbed_blend(TexturesVertex(vert_colors).sample_textures(fragments), ...) as one native op:
    colours are interpolated only where a slot wins a Monte-Carlo sample (no texel tensor).
    vert_colors (V,3) and faces (F,3) are the packed mesh tensors; gradients flow to
    dists, zbuf, bary, vert_colors and the smoothing scalars."""
    shape = tuple(pix_to_face.shape)
    N, H, W, K = shape
    if tuple(bary.shape) != shape + (3,) or vert_colors.dim() != 2 or vert_colors.shape[-1] != 3:
        raise ValueError("bary must be (N,H,W,K,3) and vert_colors (V,3)")
    if tuple(dists.shape) != shape or tuple(zbuf.shape) != shape:
        raise ValueError("dists / zbuf must match pix_to_face's shape")
    vflags = variant_flags(rast_kind, rast_vr, agg_kind, agg_vr)
    if noise is None:
        pair = noise_mod.draw_pair(shape, nb_samples_rast, nb_samples_agg, pix_to_face.device, fixed_noise, rast_kind,
                                   agg_kind)
        if pair is None:
            pair = (noise_mod.draw_rast(shape, nb_samples_rast, pix_to_face.device, rast_kind),
                    noise_mod.draw_agg((N, H, W, K + 1), nb_samples_agg, pix_to_face.device, fixed_noise, agg_kind))
        noise = _merge(*pair)
    _check_injected(noise, nb_samples_rast, nb_samples_agg, shape, True, True)
    zbuf, linked = plane_link(zbuf, znear, zfar, pix_to_face)
    live_only = live_only and not linked  # the plane link reads d zbuf at every slot
    cfg = dict(Sr=int(nb_samples_rast), Sa=int(nb_samples_agg), eps=float(eps),
               bg=_background(background), noise=noise, vflags=vflags, counts=_counts_for(pix_to_face))
    if live_only and cfg["counts"] is not None:  # the caller reads the valid prefix only (backward: no zero rows)
        cfg["vflags"] |= nat.PR_BLEND_LIVE_ONLY
    (sigma, gamma, alpha), link = _link_scalars((sigma, gamma, alpha), pix_to_face.device)
    return _fused(True, dists, zbuf, bary, vert_colors, sigma, gamma, alpha, link, pix_to_face, faces, znear, zfar, cfg)


def perturbed_blend(colors, pix_to_face, dists, zbuf, sigma, gamma, alpha, nb_samples_rast,
                    nb_samples_agg, eps=1e-10, background=(1.0, 1.0, 1.0), znear=1.0, zfar=100.0,
                    noise=None, fixed_noise=False, rast_kind="gaussian", rast_vr=True, agg_kind="gaussian",
                    agg_vr=True, live_only=False):
    """smooth_rgb_blend(colors, fragments, <Rast>, <Agg>, ...) as one native op, for the
    Gaussian / Cauchy, with / without variance reduction operator pairs.

    Returns the (N,H,W,4) image; differentiable w.r.t. dists, zbuf, colors and the
    0-d smoothing tensors sigma, gamma, alpha."""
    shape = tuple(pix_to_face.shape)
    N, H, W, K = shape
    if tuple(colors.shape[:4]) != shape or colors.shape[-1] != 3:
        raise ValueError(f"colors must be (N,H,W,K,3) = {shape + (3,)}, got {tuple(colors.shape)}")
    if tuple(dists.shape) != shape or tuple(zbuf.shape) != shape:
        raise ValueError("dists / zbuf must match pix_to_face's shape")
    vflags = variant_flags(rast_kind, rast_vr, agg_kind, agg_vr)
    if noise is None:
        pair = noise_mod.draw_pair(shape, nb_samples_rast, nb_samples_agg, pix_to_face.device, fixed_noise, rast_kind,
                                   agg_kind)
        if pair is None:
            pair = (noise_mod.draw_rast(shape, nb_samples_rast, pix_to_face.device, rast_kind),
                    noise_mod.draw_agg((N, H, W, K + 1), nb_samples_agg, pix_to_face.device, fixed_noise, agg_kind))
        noise = _merge(*pair)
    _check_injected(noise, nb_samples_rast, nb_samples_agg, shape, True, True)
    zbuf, linked = plane_link(zbuf, znear, zfar, pix_to_face)
    live_only = live_only and not linked  # the plane link reads d zbuf at every slot
    cfg = dict(Sr=int(nb_samples_rast), Sa=int(nb_samples_agg), eps=float(eps),
               bg=_background(background), noise=noise, vflags=vflags, counts=_counts_for(pix_to_face))
    if live_only and cfg["counts"] is not None:  # the caller reads the valid prefix only (backward: no zero rows)
        cfg["vflags"] |= nat.PR_BLEND_LIVE_ONLY
    (sigma, gamma, alpha), link = _link_scalars((sigma, gamma, alpha), pix_to_face.device)
    return _fused(False, dists, zbuf, colors, None, sigma, gamma, alpha, link, pix_to_face, None, znear, zfar, cfg)


def soft_blend(colors, pix_to_face, dists, zbuf, sigma, gamma, alpha, eps=1e-10, background=(1.0, 1.0, 1.0),
               znear=1.0, zfar=100.0):
    """smooth_rgb_blend(colors, fragments, SoftRast(sigma), SoftAgg(gamma, alpha, eps), ...) as one
    native kernel pair (PR_BLEND_SOFT): P = sigmoid(-dists / sigma) (smoothrast.py:126-134),
    W = softmax(((gamma/alpha) log P + z_inv - zmax) / gamma) with the background logit
    (smoothagg.py:165-182), colour mix and alpha (random_rasterizer.py:34-56).  Deterministic;
    differentiable w.r.t. dists, zbuf, colors, sigma, gamma, alpha."""
    shape = tuple(pix_to_face.shape)
    if tuple(colors.shape[:4]) != shape or colors.shape[-1] != 3:
        raise ValueError(f"colors must be (N,H,W,K,3) = {shape + (3,)}, got {tuple(colors.shape)}")
    if tuple(dists.shape) != shape or tuple(zbuf.shape) != shape:
        raise ValueError("dists / zbuf must match pix_to_face's shape")
    zbuf, _ = plane_link(zbuf, znear, zfar, pix_to_face)
    cfg = dict(Sr=1, Sa=1, eps=float(eps), bg=_background(background), noise=Noise.philox(),
               vflags=nat.PR_BLEND_SOFT, counts=_counts_for(pix_to_face))
    (sigma, gamma, alpha), link = _link_scalars((sigma, gamma, alpha), pix_to_face.device)
    return _fused(False, dists, zbuf, colors, None, sigma, gamma, alpha, link, pix_to_face, None, znear, zfar, cfg)


# ==================================================== standalone heaviside
def _heaviside_args(shape, Sr, noise, sigma_val, sigma_dev, d_c, flags=0):
    N, H, W, K = shape
    a = nat.PRHeavisideArgs()
    a.flags = flags
    a.N, a.H, a.W, a.K, a.Sr = N, H, W, K, int(Sr)
    a.sample_offset_r, a.noise_mode, a.sigma = noise.offset_r, noise.mode, sigma_val
    a.seed_r, a.noise_r, a.dists = noise.seed_r & (2 ** 64 - 1), nat.ptr(noise.noise_r), nat.ptr(d_c)
    a.sigma_dev, a.seeds = nat.ptr(sigma_dev[0] if sigma_dev else None), nat.ptr(noise.seeds)
    return a


class _HeavisideFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dists, sigma, Sr, noise, flags):
        nat.require_device(dists)
        d_c = _contig(dists)
        noise = noise.to(d_c.device)
        (sv,), sdev = _scalars((sigma,), d_c.device)
        a = _heaviside_args(tuple(d_c.shape), Sr, noise, sv, sdev, d_c, flags)
        prob = torch.empty_like(d_c)
        a.prob = nat.ptr(prob)
        nat.call("pr_heaviside_fwd", "pr_heaviside_fwd", prob, a)
        ctx.save_for_backward(d_c)
        ctx.sdev = sdev
        ctx.noise, ctx.Sr, ctx.sv, ctx.sigma_ref, ctx.flags = noise, int(Sr), sv, sigma, flags
        return prob

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gP):
        d_c, = ctx.saved_tensors
        sdev = ctx.sdev
        lib = nat.load()
        a = _heaviside_args(tuple(d_c.shape), ctx.Sr, ctx.noise, ctx.sv, sdev, d_c, ctx.flags)
        g = nat.dense(gP, F32)
        gd = torch.empty_like(d_c)
        gs = torch.empty(1, dtype=F32, device=d_c.device)
        a.grad_prob, a.grad_dists, a.grad_sigma = nat.ptr(g), nat.ptr(gd), nat.ptr(gs)
        ws = torch.empty(max(1, lib.pr_heaviside_bwd_workspace_size(a)), dtype=torch.uint8, device=d_c.device)
        a.workspace, a.workspace_bytes = nat.ptr(ws), ws.numel()
        nat.call("pr_heaviside_bwd", "pr_heaviside_bwd", g, a)
        need = ctx.needs_input_grad
        ref = ctx.sigma_ref
        sg = gs[0].to(ref.dtype) if (need[1] and torch.is_tensor(ref)) else None
        return (gd if need[0] else None), sg, None, None, None


def perturbed_heaviside(dists, sigma, nb_samples, noise=None, kind="gaussian", variance_reduction=True):
    """GaussianRast / ArctanRast (kind="cauchy") / GaussianRast_wovr (variance_reduction=False)
    .rasterize(dists): P = mean_s H(-dists + sigma*eps_s) (smoothrast.py:144-173)."""
    if dists.dim() != 4:
        raise ValueError("dists must be (N,H,W,K)")
    flags = variant_flags(rast_kind=kind, rast_vr=variance_reduction)
    if noise is None:
        noise = noise_mod.draw_rast(tuple(dists.shape), nb_samples, dists.device, kind)
    _check_injected(noise, nb_samples, 0, tuple(dists.shape), True, False)
    return _HeavisideFn.apply(dists, sigma, int(nb_samples), noise, flags)


# ==================================================== standalone aggregate
class _AggregateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, zbuf, prob, gamma, alpha, mask, znear, zfar, cfg):
        nat.require_device(zbuf, prob, mask)
        N, H, W, K = zbuf.shape
        dev = zbuf.device
        z_c, p_c = _contig(zbuf), _contig(prob)
        m_c = nat.dense(mask, torch.uint8)
        zn, zf = _planes(znear, N, dev), _planes(zfar, N, dev)
        noise = cfg["noise"].to(dev)
        sc, sc_dev = _scalars((1.0, gamma, alpha), dev)
        p = _params((N, H, W, K), 1, cfg["Sa"], sc, sc_dev, cfg["eps"], (0.0, 0.0, 0.0), noise, zn, zf,
                    cfg["vflags"])
        weights = torch.empty((N, H, W, K + 1), dtype=F32, device=dev)
        winners = torch.empty((N * H * W, cfg["Sa"]), dtype=torch.uint8, device=dev)
        a = nat.PRBlendFwdArgs()
        a.p = p
        a.mask, a.prob, a.zbuf = nat.ptr(m_c), nat.ptr(p_c), nat.ptr(z_c)
        a.weights, a.winners = nat.ptr(weights), nat.ptr(winners)
        nat.call("pr_blend_fwd", "pr_blend_fwd(aggregate)", weights, a)
        ctx.save_for_backward(z_c, p_c, m_c, zn, zf, winners)
        ctx.sc_dev = sc_dev
        ctx.cfg, ctx.noise, ctx.sc, ctx.refs = cfg, noise, sc, (gamma, alpha)
        return weights

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gW):
        _no_uniform_grad(ctx.cfg["vflags"])
        z_c, p_c, m_c, zn, zf, winners = ctx.saved_tensors
        sc_dev = ctx.sc_dev
        cfg, noise, sc = ctx.cfg, ctx.noise, ctx.sc
        lib = nat.load()
        N, H, W, K = z_c.shape
        dev = z_c.device
        p = _params((N, H, W, K), 1, cfg["Sa"], sc, sc_dev, cfg["eps"], (0.0, 0.0, 0.0), noise, zn, zf,
                    cfg["vflags"])
        g = nat.dense(gW, F32)
        gz, gp = torch.empty_like(z_c), torch.empty_like(p_c)
        gsc = torch.empty(3, dtype=F32, device=dev)
        a = nat.PRBlendBwdArgs()
        a.p = p
        a.mask, a.prob, a.zbuf, a.winners = nat.ptr(m_c), nat.ptr(p_c), nat.ptr(z_c), nat.ptr(winners)
        a.grad_weights, a.grad_prob, a.grad_zbuf, a.grad_scalars = nat.ptr(g), nat.ptr(gp), nat.ptr(gz), nat.ptr(gsc)
        ws = torch.empty(max(1, lib.pr_blend_bwd_workspace_size(a)), dtype=torch.uint8, device=dev)
        a.workspace, a.workspace_bytes = nat.ptr(ws), ws.numel()
        nat.call("pr_blend_bwd", "pr_blend_bwd(aggregate)", g, a)
        need = ctx.needs_input_grad
        _, g_g, a_g = _scalar_grads(gsc, (False, need[2], need[3]), (None,) + ctx.refs)
        return (gz if need[0] else None, gp if need[1] else None, g_g, a_g, None, None, None, None)


def perturbed_aggregate(zbuf, zfar, znear, prob_map, mask, gamma, alpha, nb_samples, eps=1e-10,
                        noise=None, fixed_noise=False, kind="gaussian", variance_reduction=True):
    """GaussianAgg / CauchyAgg (kind="cauchy") / GaussianAgg_wovr (variance_reduction=False) /
    UniformAgg (kind="uniform", forward only) .aggregate(zbuf, zfar, znear, prob_map, mask) ->
    (N,H,W,K+1) weights (smoothagg.py:196-271)."""
    N, H, W, K = zbuf.shape
    vflags = variant_flags(agg_kind=kind, agg_vr=variance_reduction)
    if noise is None:
        noise = noise_mod.draw_agg((N, H, W, K + 1), nb_samples, zbuf.device, fixed_noise, kind)
    _check_injected(noise, 0, nb_samples, (N, H, W, K), False, True)
    mask = mask.expand(N, H, W, K) if mask.shape != zbuf.shape else mask
    prob_map = prob_map.expand(N, H, W, K) if prob_map.shape != zbuf.shape else prob_map
    cfg = dict(Sa=int(nb_samples), eps=float(eps), noise=noise, vflags=vflags)
    zbuf, _ = plane_link(zbuf, znear, zfar, mask=mask)
    return _AggregateFn.apply(zbuf, prob_map, gamma, alpha, mask, znear, zfar, cfg)
