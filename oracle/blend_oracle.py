"""CPU oracle for the perturbed blend hot path  —  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.  The product (``pertrenderer_amd``) never calls it.

A closed-form restatement, in float32 torch-CPU tensor arithmetic with INJECTED
noise, of the reference's perturbed soft rasterizer + perturbed aggregation:

* ``smoothrast.py:12-59``   randomHeaviside  (Gaussian / Cauchy noise, variance-reduced score)
* ``smoothrast.py:61-108``  randomHeaviside_wovr (no variance reduction)
* ``smoothagg.py:10-73``    randomArgmax     (Gaussian / Cauchy noise, variance-reduced score)
* ``smoothagg.py:75-141``   randomArgmax_wovr (Gaussian without variance reduction; its
  Cauchy branch keeps w - vr, as the reference does)
* ``smoothagg.py:185-205``  GaussianAgg.aggregate  (logit assembly incl. background)
* ``smoothagg.py:292-337``  log_corrected / prod_corrected  (inf/nan-safe backward)
* ``random_rasterizer.py:34-56``  smooth_rgb_blend  (mask, alpha product, colour mix)

The backward is written out explicitly (no autograd.Function replay); each line
cites the reference statement whose gradient it is.  Noise is passed in as the
tensors the reference would draw: ``noise_r`` (Sr,N,H,W,K) then ``noise_a``
(Sa,N,H,W,K+1) (``smoothrast.py:21``, ``smoothagg.py:21``).

Pinned: checked against golden vectors produced by the reference itself
(tests/golden/gen_golden.py -> tests/test_oracle_golden.py).
"""
import torch

F32 = torch.float32


def _t(x):
    return x if torch.is_tensor(x) else torch.tensor(x, dtype=F32)


# ----------------------------------------------------------------------------- rast
def heaviside_fwd(D, noise_r, sigma):
    """smoothrast.py:32-36: maps = H(D + sigma*eps) (H(0)=1), vr = H(D), P = mean_s maps."""
    sigma = _t(sigma)
    maps = torch.heaviside(D + sigma * noise_r, torch.ones((), dtype=F32))
    vr = torch.heaviside(D, torch.ones((), dtype=F32))
    return maps.mean(dim=0), maps, vr


def score(noise, kind):
    """d/d eps of -log density: eps (Gaussian, smoothrast.py:46) or 2 eps / (1 + eps^2)
    (Cauchy, smoothrast.py:49, smoothagg.py:60)."""
    return noise if kind == "gaussian" else (2 * noise) / (1 + torch.square(noise))


def heaviside_bwd(maps, vr, noise_r, sigma, gP, kind="gaussian", use_vr=True):
    """smoothrast.py:45-58 / :94-107: gmaps = mean_s(base*score/sigma) with base = maps-vr
    (variance-reduced) or maps (_wovr); d D = gmaps*gP ; d sigma = sum(gmaps*gP) (the
    quirk at :57-58 overwrites the sigma score of :47 with this sum)."""
    sigma = _t(sigma)
    base = (maps - vr) if use_vr else maps
    gmaps = (base * score(noise_r, kind) / sigma).mean(dim=0)
    gD = gmaps * gP
    return gD, gD.sum()


# ------------------------------------------------------------------------------ agg
def logits(zbuf, zfar, znear, prob, mask, gamma, alpha, eps):
    """smoothagg.py:197-202: z_inv, z_max (clamped), log prob, (gamma/alpha)*L + z_inv - z_max,
    background logit eps - z_max appended -> (N,H,W,K+1)."""
    gamma, alpha = _t(gamma), _t(alpha)
    maskf = mask
    z_inv = (zfar - zbuf) / (zfar - znear) * maskf
    zmax_raw, kmax = torch.max(z_inv, dim=-1)
    zmax = zmax_raw[..., None].clamp(min=eps)
    L = prob.log()
    gal = gamma / alpha
    zk = gal * L + z_inv - zmax
    N, H, W, _ = zk.shape
    z = torch.cat((zk, torch.ones((N, H, W, 1), dtype=F32) * eps - zmax), dim=-1)
    return z, dict(z_inv=z_inv, zmax_raw=zmax_raw, kmax=kmax, L=L, gal=gal)


def argmax_fwd(z, noise_a, gamma):
    """smoothagg.py:33-41: one-hot argmax of z + gamma*eps (first index on ties),
    mean over samples; vr' = one-hot argmax z."""
    gamma = _t(gamma)
    zp = z + gamma * noise_a
    idx = torch.max(zp, dim=-1, keepdim=True)[1]
    w = torch.zeros(zp.shape, dtype=F32).scatter_(-1, idx, 1)
    j0 = torch.max(z, dim=-1, keepdim=True)[1]
    vr = torch.zeros(z.shape, dtype=F32).scatter_(-1, j0, 1)
    return w.mean(dim=0), w, vr


def argmax_bwd(w, vr, noise_a, gamma, gW, kind="gaussian", use_vr=True):
    """smoothagg.py:50-56,71-72 (and :118-124 wovr): a_s = <gW, diff_s> with diff = w_s - vr'
    (variance-reduced, and always for Cauchy) or w_s (Gaussian _wovr);
    dz = mean_s(a_s*score(eps_s)/gamma) ;
    d gamma = mean_s sum_{pix,j} gW*diff_s*(n_s - 1)/gamma with n_s = |eps_s|^2 (Gaussian) or
    sum_j score(eps_sj)*eps_sj (Cauchy), over all K+1 logits, masked slots included."""
    gamma = _t(gamma)
    diff = (w - vr.unsqueeze(0)) if (use_vr or kind == "cauchy") else w
    a = (gW.unsqueeze(0) * diff).sum(-1, keepdim=True)
    sc = score(noise_a, kind)
    dz = (a * sc / gamma).mean(dim=0)
    if kind == "gaussian":
        n2 = torch.square(torch.norm(noise_a, dim=-1, keepdim=True))
    else:
        n2 = (sc * noise_a).sum(-1, keepdim=True)
    gg = (gW.unsqueeze(0) * (diff * (n2 - 1.0) / gamma)).sum(dim=(1, 2, 3, 4)).mean(dim=0)
    return dz, gg


def logits_bwd(dz, prob, mask, zfar, znear, gamma, alpha, eps, aux):
    """Gradient of smoothagg.py:197-202 w.r.t. zbuf, prob, gamma, alpha given dz (N,H,W,K+1)."""
    gamma, alpha = _t(gamma), _t(alpha)
    K = prob.shape[-1]
    dzk, dzK = dz[..., :K], dz[..., K:]
    # z_max enters both "- z_inv_max" (:201, broadcast over K) and "eps - z_inv_max" (:202)
    dzmax = -dzk.sum(-1, keepdim=True) - dzK
    dzmax = dzmax * (aux["zmax_raw"][..., None] >= eps)          # clamp(min=eps) (:199)
    dz_inv = dzk + torch.zeros_like(dzk).scatter_(-1, aux["kmax"][..., None], dzmax)  # max (:199)
    dzbuf = -(dz_inv * mask / (zfar - znear))                     # :198
    aux["dz_inv"] = dz_inv
    # prod_corrected backward (:329-336): x = gamma/alpha, y = log prob
    L = aux["L"]
    dL = aux["gal"] * dzk
    dL = torch.where(torch.isnan(dL), torch.zeros_like(dL), dL)
    dgal = (torch.where(torch.isinf(L), torch.zeros_like(L), L) * dzk).nansum()
    # log_corrected backward (:308-310)
    r = torch.ones(prob.shape, dtype=F32) / prob
    r = torch.where(torch.isinf(r), torch.zeros_like(r), r)
    dprob = r * dL
    dgamma = dgal / alpha
    dalpha = -dgal * ((gamma / alpha) / alpha)
    return dzbuf, dprob, dgamma, dalpha


def plane_grads(zbuf, zfar, znear, mask, dz_inv):
    """d znear, d zfar (each (N,1,1,1)) of smoothagg.py:198's z_inv = (zfar - zbuf) / (zfar - znear)
    * mask given dL/dz_inv: torch autograd of that expression, i.e. what the reference's graph
    gives camera planes that require grad (random_rasterizer.py:172-173)."""
    with torch.enable_grad():  # (also when called from an autograd Function's backward)
        zn = znear.detach().clone().requires_grad_(True)
        zf = zfar.detach().clone().requires_grad_(True)
        z_inv = (zf - zbuf.detach()) / (zf - zn) * mask
        return torch.autograd.grad(z_inv, (zn, zf), dz_inv.detach())


def _prod_backward(x, g):
    """torch's prod(dim=-1) backward as ATen implements it: grad*result/input when the
    whole input has no zero, exclusive prefix*suffix products otherwise."""
    if bool((x != 0).all()):
        return g[..., None] * (x.prod(-1, keepdim=True) / x)
    ones = torch.ones_like(x[..., :1])
    pre = torch.cat((ones, x[..., :-1]), -1).cumprod(-1)
    suf = torch.cat((ones, x[..., 1:].flip(-1)), -1).cumprod(-1).flip(-1)
    return g[..., None] * (pre * suf)


# ---------------------------------------------------------------------------- blend
def blend_forward(p2f, dists, zbuf, colors, noise_r, noise_a, sigma, gamma, alpha, eps,
                  background, znear, zfar, rast_kind="gaussian", rast_vr=True, agg_kind="gaussian",
                  agg_vr=True):
    """random_rasterizer.py:34-56 with GaussianRast/GaussianAgg, injected noise.

    znear/zfar: (N,1,1,1) float32 tensors (random_rasterizer.py:172-173).
    Returns (image (N,H,W,4), saved dict for blend_backward)."""
    N, H, W, K = p2f.shape
    bg = torch.as_tensor(background, dtype=F32)
    mask = p2f >= 0
    D = -dists                                                         # smoothrast.py:146
    P, maps, vr = heaviside_fwd(D, noise_r, sigma)
    prob = P * mask                                                    # :47
    one_minus = 1.0 - prob
    alpha_chan = torch.prod(one_minus, dim=-1)                         # :48
    z, aux = logits(zbuf, zfar, znear, prob, mask, gamma, alpha, eps)
    Wt, w, vra = argmax_fwd(z, noise_a, gamma)                         # :49
    wz, wb = Wt[..., :-1], Wt[..., -1:]
    img = torch.ones((N, H, W, 4), dtype=F32)
    img[..., :3] = (wz[..., None] * colors).sum(dim=-2) + wb * bg      # :50-53
    img[..., 3] = 1.0 - alpha_chan                                     # :54
    saved = dict(mask=mask, maps=maps, vr=vr, prob=prob, one_minus=one_minus, aux=aux, w=w, zbuf=zbuf,
                 vra=vra, W=Wt, colors=colors, bg=bg, zfar=zfar, znear=znear, noise_r=noise_r,
                 noise_a=noise_a, sigma=sigma, gamma=gamma, alpha=alpha, eps=eps, P=P,
                 kinds=(rast_kind, rast_vr, agg_kind, agg_vr))
    return img, saved


def blend_backward(gimg, s):
    """Closed-form backward of blend_forward.  Returns dict of grads
    (dists, zbuf, colors, sigma, gamma, alpha)."""
    K = s["prob"].shape[-1]
    g_rgb, g_a = gimg[..., :3], gimg[..., 3]
    # colour mix (:50-53)
    dW = torch.cat(((g_rgb[..., None, :] * s["colors"]).sum(-1),
                    (g_rgb * s["bg"]).sum(-1, keepdim=True)), dim=-1)
    dcolors = s["W"][..., :-1, None] * g_rgb[..., None, :]
    rk, rvr, ak, avr = s.get("kinds", ("gaussian", True, "gaussian", True))
    dz, dg1 = argmax_bwd(s["w"], s["vra"], s["noise_a"], s["gamma"], dW, ak, avr)
    dzbuf, dprob_l, dg2, dalpha = logits_bwd(dz, s["prob"], s["mask"], s["zfar"], s["znear"],
                                             s["gamma"], s["alpha"], s["eps"], s["aux"])
    # alpha channel: A = 1 - prod(1 - prob)  (:48,:54)
    dprob_a = -_prod_backward(s["one_minus"], -g_a)
    dprob = dprob_a + dprob_l
    dP = dprob * s["mask"]                                             # :47
    dD, dsigma = heaviside_bwd(s["maps"], s["vr"], s["noise_r"], s["sigma"], dP, rk, rvr)
    dzn, dzf = plane_grads(s["zbuf"], s["zfar"], s["znear"], s["mask"], s["aux"]["dz_inv"])
    return dict(dists=-dD, zbuf=dzbuf, colors=dcolors, sigma=dsigma, gamma=dg1 + dg2,
                alpha=dalpha, znear=dzn, zfar=dzf)


# --------------------------------------------------------------- standalone methods
def rasterize_forward_backward(dists, noise_r, sigma, gP, kind="gaussian", use_vr=True):
    """GaussianRast / ArctanRast / GaussianRast_wovr .rasterize (smoothrast.py:144-173) and
    the backward."""
    P, maps, vr = heaviside_fwd(-dists, noise_r, sigma)
    dD, dsigma = heaviside_bwd(maps, vr, noise_r, sigma, gP, kind, use_vr)
    return P, -dD, dsigma


def aggregate_forward_backward(zbuf, zfar, znear, prob, mask, noise_a, gamma, alpha, eps, gW,
                               kind="gaussian", use_vr=True, planes=False):
    """GaussianAgg / CauchyAgg / GaussianAgg_wovr .aggregate (smoothagg.py:196-250) and the
    backward (planes=True: also d znear, d zfar)."""
    z, aux = logits(zbuf, zfar, znear, prob, mask, gamma, alpha, eps)
    Wt, w, vra = argmax_fwd(z, noise_a, gamma)
    dz, dg1 = argmax_bwd(w, vra, noise_a, gamma, gW, kind, use_vr)
    dzbuf, dprob, dg2, dalpha = logits_bwd(dz, prob, mask, zfar, znear, gamma, alpha, eps, aux)
    if planes:
        return (Wt, dzbuf, dprob, dg1 + dg2, dalpha) + tuple(plane_grads(zbuf, zfar, znear, mask, aux["dz_inv"]))
    return Wt, dzbuf, dprob, dg1 + dg2, dalpha


# ---------------------------------------------------------- CPU baseline ("port")
def blend_step_cpu(p2f, dists, zbuf, colors, Sr, Sa, sigma, gamma, alpha, eps, background,
                   znear, zfar, gimg, generator=None):
    """One forward+backward of the blend on CPU, drawing the noise the way the reference
    does (randn(Sr,...) then randn(Sa,...,K+1)).  Used as bench.py's cpu_baseline."""
    N, H, W, K = p2f.shape
    nr = torch.randn((Sr, N, H, W, K), generator=generator)
    na = torch.randn((Sa, N, H, W, K + 1), generator=generator)
    img, saved = blend_forward(p2f, dists, zbuf, colors, nr, na, sigma, gamma, alpha, eps,
                               background, znear, zfar)
    return img, blend_backward(gimg, saved)


# ------------------------------------------------------ deterministic soft variants
class _LogC(torch.autograd.Function):
    """log whose backward maps 1/x = inf to 0 (semantics of smoothagg.py:303-311)."""
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return x.log()

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        r = 1.0 / x
        return torch.where(torch.isinf(r), torch.zeros_like(r), r) * g


class _ProdC(torch.autograd.Function):
    """scalar*tensor whose backward drops inf factors / nan products
    (semantics of smoothagg.py:325-337)."""
    @staticmethod
    def forward(ctx, x, y):
        ctx.save_for_backward(x, y)
        return x * y

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        dx = (torch.where(torch.isinf(y), torch.zeros_like(y), y) * g).nansum()
        dy = x * g
        return dx, torch.where(torch.isnan(dy), torch.zeros_like(dy), dy)


def soft_blend_forward_backward(p2f, dists, zbuf, colors, sigma, gamma, alpha, eps, background,
                                znear, zfar, gimg):
    """SoftRast (smoothrast.py:132-134) + SoftAgg (smoothagg.py:173-182) through
    smooth_rgb_blend (random_rasterizer.py:34-56); gradients by autograd on the restated graph."""
    sig, gam, alp = (torch.tensor(float(v), dtype=F32, requires_grad=True)
                     for v in (sigma, gamma, alpha))
    d = dists.clone().requires_grad_(True)
    zb = zbuf.clone().requires_grad_(True)
    col = colors.clone().requires_grad_(True)
    mask = p2f >= 0
    prob = torch.sigmoid(-d / sig) * mask
    alpha_chan = torch.prod(1.0 - prob, dim=-1)
    z_inv = (zfar - zb) / (zfar - znear) * mask
    zmax = torch.max(z_inv, dim=-1).values[..., None].clamp(min=eps)
    zk = _ProdC.apply(gam / alp, _LogC.apply(prob)) + z_inv - zmax
    N, H, W, K = p2f.shape
    z = torch.cat((zk, torch.ones((N, H, W, 1)) * eps - zmax), dim=-1)
    Wt = torch.softmax(_ProdC.apply(1.0 / gam, z), dim=-1)
    bg = torch.as_tensor(background, dtype=F32)
    img = torch.ones((N, H, W, 4), dtype=F32)
    img[..., :3] = (Wt[..., :-1, None] * col).sum(-2) + Wt[..., -1:] * bg
    img[..., 3] = 1.0 - alpha_chan
    (img * gimg).sum().backward()
    out = dict(dists=d.grad, zbuf=zb.grad, colors=col.grad, sigma=sig.grad, gamma=gam.grad, alpha=alp.grad)
    for name, z in (("znear", znear), ("zfar", zfar)):  # planes that require grad (leaves)
        if torch.is_tensor(z) and z.requires_grad:
            out[name] = z.grad
    return img.detach(), out
