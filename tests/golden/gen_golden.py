"""Golden-vector generator for the perturbed blend (randomras) hot path.

Runs ONLY in the build container, where the read-only reference checkout lives
at /root/reference.  It imports the reference's own ``randomras`` package
(smoothrast / smoothagg / random_rasterizer) unmodified, with placeholder
``pytorch3d`` modules in ``sys.modules`` because ``random_rasterizer.py:8-26``
imports PyTorch3D names at module scope that ``smooth_rgb_blend`` never uses.

For every case it records, into ``tests/golden/<case>.npz``:
  * the synthetic Fragments / colours / camera planes / smoothing parameters,
  * the exact Gaussian noise tensors the reference drew (re-drawn here from the
    same CPU generator state: ``randn(Sr,N,H,W,K)`` then ``randn(Sa,N,H,W,K+1)``,
    the order of ``smoothrast.py:21`` then ``smoothagg.py:21``),
  * a random upstream gradient and the reference's outputs and gradients
    (image / P / W, d dists, d zbuf, d colours, d sigma, d gamma, d alpha).

The fixtures are DATA (inputs and expected outputs); no reference source is
copied into this repository.  Re-run with::

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py            # all cases
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py uniform    # agg_uniform only
"""
import collections
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    p3d = types.ModuleType("pytorch3d")
    ren = types.ModuleType("pytorch3d.renderer")
    mesh = types.ModuleType("pytorch3d.renderer.mesh")
    shading = types.ModuleType("pytorch3d.renderer.mesh.shading")
    for name in ["look_at_view_transform", "OpenGLPerspectiveCameras", "PointLights",
                 "DirectionalLights", "Materials", "RasterizationSettings", "MeshRenderer",
                 "MeshRasterizer", "SoftPhongShader", "HardPhongShader", "SoftSilhouetteShader",
                 "hard_rgb_blend", "softmax_rgb_blend", "TexturesVertex"]:
        setattr(ren, name, type(name, (), {}))
    ren.BlendParams = collections.namedtuple("BlendParams", "sigma gamma background_color")
    shading.phong_shading = None
    sys.modules.update({"pytorch3d": p3d, "pytorch3d.renderer": ren,
                        "pytorch3d.renderer.mesh": mesh,
                        "pytorch3d.renderer.mesh.shading": shading})
    sys.path.insert(0, REF)
    from randomras import random_rasterizer, smoothagg, smoothrast  # noqa: E402
    return random_rasterizer, smoothrast, smoothagg, ren.BlendParams


Fragments = collections.namedtuple("Fragments", "pix_to_face zbuf bary_coords dists")


def synth_fragments(g, N, H, W, K, sigma, p_valid=0.6, packed=False):
    """Synthetic Fragments in PyTorch3D layout (N,H,W,K), K fastest.

    Valid slots: p2f in [0,1000), dists ~ U(-3s,3s), zbuf ~ 5+U(0,1);
    padded slots carry -1 everywhere (PyTorch3D's padding convention).
    """
    valid = torch.rand((N, H, W, K), generator=g) < p_valid
    if packed:  # valid slots first, like the rasterizer's output
        cnt = valid.sum(-1, keepdim=True)
        valid = torch.arange(K).expand(N, H, W, K) < cnt
    p2f = torch.randint(0, 1000, (N, H, W, K), generator=g)
    dists = (torch.rand((N, H, W, K), generator=g) - 0.5) * 6 * sigma
    zbuf = 5.0 + torch.rand((N, H, W, K), generator=g)
    if packed:
        zbuf, _ = zbuf.sort(-1)
    p2f = torch.where(valid, p2f, torch.full_like(p2f, -1))
    dists = torch.where(valid, dists, torch.full_like(dists, -1.0))
    zbuf = torch.where(valid, zbuf, torch.full_like(zbuf, -1.0))
    bary = torch.where(valid[..., None], torch.rand((N, H, W, K, 3), generator=g),
                       torch.full((N, H, W, K, 3), -1.0))
    return Fragments(p2f, zbuf, bary, dists)


def edge_fragments():
    """Hand-built edge cases (N=1, 4x4, K=6).

    row 0: all-masked pixel / single valid slot / P=1 slots (zero factor in the
           alpha product, twice in px(0,3)) ;
    row 1: exactly-equal zbuf (argmax tie on coplanar faces), D = +0 and -0 ;
    rows 2-3: random valid/invalid mix.
    """
    g = torch.Generator().manual_seed(7)
    N, H, W, K = 1, 4, 4, 6
    fr = synth_fragments(g, N, H, W, K, 1e-3, p_valid=0.7)
    p2f, zbuf, bary, dists = [t.clone() for t in fr]
    p2f[0, 0, 0] = -1; zbuf[0, 0, 0] = -1.0; dists[0, 0, 0] = -1.0
    p2f[0, 0, 1] = -1; zbuf[0, 0, 1] = -1.0; dists[0, 0, 1] = -1.0
    p2f[0, 0, 1, 0] = 3; zbuf[0, 0, 1, 0] = 5.5; dists[0, 0, 1, 0] = -1e-4
    p2f[0, 0, 2, :3] = torch.tensor([1, 2, 3]); dists[0, 0, 2, :3] = torch.tensor([-1.0, -1e-4, 2e-4])
    zbuf[0, 0, 2, :3] = torch.tensor([5.1, 5.2, 5.3])
    p2f[0, 0, 3, :] = torch.arange(6); dists[0, 0, 3, :] = torch.tensor([-1.0, -1.0, 1e-4, -2e-4, 3e-4, 0.0])
    zbuf[0, 0, 3, :] = torch.tensor([5.0, 5.0, 5.3, 5.3, 5.4, 5.5])
    p2f[0, 1, 0, :] = torch.arange(10, 16); zbuf[0, 1, 0, :] = 5.25; dists[0, 1, 0, :] = -2e-4
    p2f[0, 1, 1, :2] = torch.tensor([4, 5]); dists[0, 1, 1, :2] = torch.tensor([0.0, -0.0])
    zbuf[0, 1, 1, :2] = torch.tensor([5.5, 5.5])
    return Fragments(p2f, zbuf, bary, dists)


def leaves(sigma, gamma, alpha):
    return (torch.tensor(sigma, requires_grad=True), torch.tensor(gamma, requires_grad=True),
            torch.tensor(alpha, requires_grad=True))


def run_blend_case(name, ref, fr, colors, Sr, Sa, sigma, gamma, alpha, bg, znear, zfar,
                   seed, fixed_noise=False, eps=1e-10):
    rr, sr, sa, BlendParams = ref
    N, H, W, K = fr.pix_to_face.shape
    rast = sr.GaussianRast(nb_samples=Sr, sigma=sigma)
    agg = sa.GaussianAgg(nb_samples=Sa, gamma=gamma, alpha=alpha, eps=eps, fixed_noise=fixed_noise)
    dists = fr.dists.clone().requires_grad_(True)
    zbuf = fr.zbuf.clone().requires_grad_(True)
    cols = colors.clone().requires_grad_(True)
    frag = Fragments(fr.pix_to_face, zbuf, fr.bary_coords, dists)
    zn = torch.full((N,), znear)[:, None, None, None]
    zf = torch.full((N,), zfar)[:, None, None, None]
    bp = BlendParams(sigma, gamma, tuple(bg))
    torch.manual_seed(seed)
    img = rr.smooth_rgb_blend(cols, frag, rast, agg, bp, znear=zn, zfar=zf)
    gup = torch.randn(img.shape, generator=torch.Generator().manual_seed(seed + 1))
    (img * gup).sum().backward()
    torch.manual_seed(seed)
    er = torch.randn((Sr, N, H, W, K))
    if fixed_noise:
        torch.manual_seed(1)
    ea = torch.randn((Sa, N, H, W, K + 1))
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"),
        pix_to_face=fr.pix_to_face.numpy(), zbuf=fr.zbuf.numpy(), dists=fr.dists.numpy(),
        colors=colors.numpy(), znear=np.float32(znear), zfar=np.float32(zfar),
        background=np.asarray(bg, np.float32), sigma=np.float32(sigma), gamma=np.float32(gamma),
        alpha=np.float32(alpha), eps=np.float64(eps), Sr=np.int64(Sr), Sa=np.int64(Sa),
        seed=np.int64(seed), fixed_noise=np.bool_(fixed_noise),
        noise_r=er.numpy(), noise_a=ea.numpy(), grad_image=gup.numpy(),
        image=img.detach().numpy(), grad_dists=dists.grad.numpy(), grad_zbuf=zbuf.grad.numpy(),
        grad_colors=cols.grad.numpy(), grad_sigma=rast.sigma.grad.numpy(),
        grad_gamma=agg.gamma.grad.numpy(), grad_alpha=agg.alpha.grad.numpy())
    print("wrote", name, tuple(img.shape))


def run_rast_case(name, ref, fr, Sr, sigma, seed):
    _, sr, _, _ = ref
    N, H, W, K = fr.dists.shape
    rast = sr.GaussianRast(nb_samples=Sr, sigma=sigma)
    dists = fr.dists.clone().requires_grad_(True)
    torch.manual_seed(seed)
    P = rast.rasterize(dists)
    gup = torch.randn(P.shape, generator=torch.Generator().manual_seed(seed + 1))
    (P * gup).sum().backward()
    torch.manual_seed(seed)
    er = torch.randn((Sr, N, H, W, K))
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"), dists=fr.dists.numpy(), sigma=np.float32(sigma),
        Sr=np.int64(Sr), seed=np.int64(seed), noise_r=er.numpy(), grad_P=gup.numpy(),
        P=P.detach().numpy(), grad_dists=dists.grad.numpy(), grad_sigma=rast.sigma.grad.numpy())
    print("wrote", name, tuple(P.shape))


def run_agg_case(name, ref, fr, prob, Sa, gamma, alpha, znear, zfar, seed, eps=1e-10):
    _, _, sa, _ = ref
    N, H, W, K = fr.zbuf.shape
    agg = sa.GaussianAgg(nb_samples=Sa, gamma=gamma, alpha=alpha, eps=eps)
    zbuf = fr.zbuf.clone().requires_grad_(True)
    mask = fr.pix_to_face >= 0
    pr = (prob * mask).clone().requires_grad_(True)
    zn = torch.full((N,), znear)[:, None, None, None]
    zf = torch.full((N,), zfar)[:, None, None, None]
    torch.manual_seed(seed)
    Wt = agg.aggregate(zbuf, zf, zn, pr, mask)
    gup = torch.randn(Wt.shape, generator=torch.Generator().manual_seed(seed + 1))
    (Wt * gup).sum().backward()
    torch.manual_seed(seed)
    ea = torch.randn((Sa, N, H, W, K + 1))
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"), pix_to_face=fr.pix_to_face.numpy(), zbuf=fr.zbuf.numpy(),
        prob=(prob * mask).numpy(), znear=np.float32(znear), zfar=np.float32(zfar),
        gamma=np.float32(gamma), alpha=np.float32(alpha), eps=np.float64(eps), Sa=np.int64(Sa),
        seed=np.int64(seed), noise_a=ea.numpy(), grad_W=gup.numpy(), W=Wt.detach().numpy(),
        grad_zbuf=zbuf.grad.numpy(), grad_prob=pr.grad.numpy(),
        grad_gamma=agg.gamma.grad.numpy(), grad_alpha=agg.alpha.grad.numpy())
    print("wrote", name, tuple(Wt.shape))


def run_uniform_agg_case(name, ref, fr, prob, Sa, gamma, alpha, znear, zfar, seed, eps=1e-10):
    """UniformAgg.aggregate forward (smoothagg.py:252-271, noise :28-30); the reference has no
    backward for it (smoothagg.py:64-70), so only the weights are recorded."""
    _, _, sa, _ = ref
    N, H, W, K = fr.zbuf.shape
    agg = sa.UniformAgg(nb_samples=Sa, gamma=gamma, alpha=alpha, eps=eps)
    mask = fr.pix_to_face >= 0
    pr = prob * mask
    zn = torch.full((N,), znear)[:, None, None, None]
    zf = torch.full((N,), zfar)[:, None, None, None]
    torch.manual_seed(seed)
    with torch.no_grad():
        Wt = agg.aggregate(fr.zbuf, zf, zn, pr, mask)
    torch.manual_seed(seed)
    m = torch.distributions.uniform.Uniform(torch.tensor([-0.5]), torch.tensor([0.5]))
    ea = m.sample((Sa, N, H, W, K + 1)).squeeze(-1)
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"), pix_to_face=fr.pix_to_face.numpy(), zbuf=fr.zbuf.numpy(),
        prob=pr.numpy(), znear=np.float32(znear), zfar=np.float32(zfar),
        gamma=np.float32(gamma), alpha=np.float32(alpha), eps=np.float64(eps), Sa=np.int64(Sa),
        seed=np.int64(seed), noise_a=ea.numpy(), W=Wt.numpy())
    print("wrote", name, tuple(Wt.shape))


def main_uniform():
    """Only the UniformAgg case (added after the other fixtures: leaves them untouched)."""
    ref = _import_reference()
    torch.set_num_threads(1)
    g = torch.Generator().manual_seed(12)
    fr = synth_fragments(g, 2, 4, 5, 9, 1e-3, packed=True)
    prob = torch.rand((2, 4, 5, 9), generator=g)
    prob[0, 0, 0, :2] = 1.0
    run_uniform_agg_case("agg_uniform", ref, fr, prob, 6, 2e-2, 1.0, 1.0, 100.0, 91)


def redraw(kind, shape):
    """The reference's own noise draw (smoothrast.py:20-24, smoothagg.py:20-27) replayed
    from the same global generator state."""
    if kind == "gaussian":
        return torch.normal(mean=torch.zeros(shape), std=1.0)
    m = torch.distributions.cauchy.Cauchy(torch.tensor([0.0]), torch.tensor([1.0]))
    return torch.clamp(m.sample(shape).squeeze(-1), min=-1e7, max=1e7)


RAST_KIND = {"GaussianRast": ("gaussian", True), "GaussianRast_wovr": ("gaussian", False),
             "ArctanRast": ("cauchy", True)}
AGG_KIND = {"GaussianAgg": ("gaussian", True), "GaussianAgg_wovr": ("gaussian", False),
            "CauchyAgg": ("cauchy", True)}


def run_variant_blend_case(name, ref, fr, colors, rast_cls, agg_cls, Sr, Sa, sigma, gamma, alpha, bg,
                           znear, zfar, seed, eps=1e-10):
    """smooth_rgb_blend with a non-default (rast, agg) pair: Cauchy noise and/or no variance
    reduction."""
    rr, sr, sa, BlendParams = ref
    N, H, W, K = fr.pix_to_face.shape
    rast = getattr(sr, rast_cls)(nb_samples=Sr, sigma=sigma)
    agg = getattr(sa, agg_cls)(nb_samples=Sa, gamma=gamma, alpha=alpha, eps=eps)
    dists = fr.dists.clone().requires_grad_(True)
    zbuf = fr.zbuf.clone().requires_grad_(True)
    cols = colors.clone().requires_grad_(True)
    frag = Fragments(fr.pix_to_face, zbuf, fr.bary_coords, dists)
    zn = torch.full((N,), znear)[:, None, None, None]
    zf = torch.full((N,), zfar)[:, None, None, None]
    torch.manual_seed(seed)
    img = rr.smooth_rgb_blend(cols, frag, rast, agg, BlendParams(sigma, gamma, tuple(bg)), znear=zn, zfar=zf)
    gup = torch.randn(img.shape, generator=torch.Generator().manual_seed(seed + 1))
    (img * gup).sum().backward()
    torch.manual_seed(seed)
    rk, rvr = RAST_KIND[rast_cls]
    ak, avr = AGG_KIND[agg_cls]
    er = redraw(rk, (Sr, N, H, W, K))
    ea = redraw(ak, (Sa, N, H, W, K + 1))
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"),
        pix_to_face=fr.pix_to_face.numpy(), zbuf=fr.zbuf.numpy(), dists=fr.dists.numpy(),
        colors=colors.numpy(), znear=np.float32(znear), zfar=np.float32(zfar),
        background=np.asarray(bg, np.float32), sigma=np.float32(sigma), gamma=np.float32(gamma),
        alpha=np.float32(alpha), eps=np.float64(eps), Sr=np.int64(Sr), Sa=np.int64(Sa),
        seed=np.int64(seed), rast_cls=np.str_(rast_cls), agg_cls=np.str_(agg_cls),
        rast_kind=np.str_(rk), rast_vr=np.bool_(rvr), agg_kind=np.str_(ak), agg_vr=np.bool_(avr),
        noise_r=er.numpy(), noise_a=ea.numpy(), grad_image=gup.numpy(),
        image=img.detach().numpy(), grad_dists=dists.grad.numpy(), grad_zbuf=zbuf.grad.numpy(),
        grad_colors=cols.grad.numpy(), grad_sigma=rast.sigma.grad.numpy(),
        grad_gamma=agg.gamma.grad.numpy(), grad_alpha=agg.alpha.grad.numpy())
    print("wrote", name, tuple(img.shape))


def run_soft_case(name, ref, fr, colors, sigma, gamma, alpha, bg, znear, zfar, eps=1e-10):
    """Deterministic SoftRast + SoftAgg blend (eval.py's default "softras" renderer)."""
    rr, sr, sa, BlendParams = ref
    N, H, W, K = fr.pix_to_face.shape
    rast = sr.SoftRast(sigma=sigma)
    agg = sa.SoftAgg(gamma=gamma, alpha=alpha, eps=eps)
    dists = fr.dists.clone().requires_grad_(True)
    zbuf = fr.zbuf.clone().requires_grad_(True)
    cols = colors.clone().requires_grad_(True)
    frag = Fragments(fr.pix_to_face, zbuf, fr.bary_coords, dists)
    zn = torch.full((N,), znear)[:, None, None, None]
    zf = torch.full((N,), zfar)[:, None, None, None]
    img = rr.smooth_rgb_blend(cols, frag, rast, agg, BlendParams(sigma, gamma, tuple(bg)), znear=zn, zfar=zf)
    gup = torch.randn(img.shape, generator=torch.Generator().manual_seed(99))
    (img * gup).sum().backward()
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"), pix_to_face=fr.pix_to_face.numpy(), zbuf=fr.zbuf.numpy(),
        dists=fr.dists.numpy(), colors=colors.numpy(), znear=np.float32(znear), zfar=np.float32(zfar),
        background=np.asarray(bg, np.float32), sigma=np.float32(sigma), gamma=np.float32(gamma),
        alpha=np.float32(alpha), eps=np.float64(eps), grad_image=gup.numpy(),
        image=img.detach().numpy(), grad_dists=dists.grad.numpy(), grad_zbuf=zbuf.grad.numpy(),
        grad_colors=cols.grad.numpy(), grad_sigma=rast.sigma.grad.numpy(),
        grad_gamma=agg.gamma.grad.numpy(), grad_alpha=agg.alpha.grad.numpy())
    print("wrote", name, tuple(img.shape))


def main():
    ref = _import_reference()
    torch.set_num_threads(1)
    # F1: small, K=8, Sr=Sa=4, coloured background
    g = torch.Generator().manual_seed(0)
    fr = synth_fragments(g, 1, 4, 6, 8, 1e-3)
    cols = torch.rand((1, 4, 6, 8, 3), generator=g)
    run_blend_case("blend_small", ref, fr, cols, 4, 4, 1e-3, 1e-2, 1.0, (0.2, 0.5, 0.9), 1.0, 100.0, 123)
    # F2: eval.py plumbing ratio (GaussianRast default Sr=16, agg Sa=8), K=50, N=2, alpha != 1
    g = torch.Generator().manual_seed(1)
    fr = synth_fragments(g, 2, 6, 5, 50, 1e-3, packed=True)
    cols = torch.rand((2, 6, 5, 50, 3), generator=g)
    run_blend_case("blend_eval", ref, fr, cols, 16, 8, 1e-3, 1e-2, 1.5, (0.0, 0.0, 0.0), 1.0, 100.0, 321)
    # F3: edge cases, odd sample counts
    fr = edge_fragments()
    cols = torch.rand((1, 4, 4, 6, 3), generator=torch.Generator().manual_seed(3))
    run_blend_case("blend_edge", ref, fr, cols, 5, 3, 1e-3, 1e-2, 1.0, (1.0, 1.0, 1.0), 1.0, 100.0, 5)
    # F4: fixed_noise=True (reference reseeds the global generator with 1 before the agg draw)
    g = torch.Generator().manual_seed(4)
    fr = synth_fragments(g, 1, 3, 3, 5, 1e-3)
    cols = torch.rand((1, 3, 3, 5, 3), generator=g)
    run_blend_case("blend_fixed", ref, fr, cols, 4, 6, 1e-3, 2e-2, 1.0, (0.0, 0.0, 0.0), 0.5, 20.0, 77,
                   fixed_noise=True)
    # F5: K=100 (two 64-slot chunks), larger smoothing
    g = torch.Generator().manual_seed(5)
    fr = synth_fragments(g, 1, 3, 4, 100, 5e-3, p_valid=0.8, packed=True)
    cols = torch.rand((1, 3, 4, 100, 3), generator=g)
    run_blend_case("blend_k100", ref, fr, cols, 8, 8, 5e-3, 5e-2, 1.0, (0.3, 0.3, 0.3), 1.0, 100.0, 11)
    # standalone GaussianRast.rasterize / GaussianAgg.aggregate
    g = torch.Generator().manual_seed(6)
    fr = synth_fragments(g, 2, 4, 4, 7, 1e-3)
    run_rast_case("rast_only", ref, fr, 6, 1e-3, 31)
    prob = torch.rand((2, 4, 4, 7), generator=g)
    prob[0, 0, 0, :3] = 1.0
    prob[0, 1, 1, 1] = 0.0
    run_agg_case("agg_only", ref, fr, prob, 5, 1e-2, 1.0, 1.0, 100.0, 41)
    # noise variants (Cauchy / no variance reduction), fused blend
    g = torch.Generator().manual_seed(9)
    fr = synth_fragments(g, 2, 4, 5, 12, 1e-3, packed=True)
    cols = torch.rand((2, 4, 5, 12, 3), generator=g)
    run_variant_blend_case("var_arctan_cauchy", ref, fr, cols, "ArctanRast", "CauchyAgg", 8, 8, 1e-3, 1e-2, 1.0,
                           (0.1, 0.2, 0.3), 1.0, 100.0, 61)
    run_variant_blend_case("var_wovr", ref, fr, cols, "GaussianRast_wovr", "GaussianAgg_wovr", 8, 8, 1e-3, 1e-2,
                           1.0, (0.1, 0.2, 0.3), 1.0, 100.0, 62)
    run_variant_blend_case("var_mixed", ref, fr, cols, "ArctanRast", "GaussianAgg_wovr", 6, 5, 1e-3, 2e-2,
                           1.3, (0.0, 0.0, 0.0), 1.0, 100.0, 63)
    # deterministic soft path (eval.py "softras")
    g = torch.Generator().manual_seed(8)
    fr = synth_fragments(g, 1, 4, 5, 9, 1e-3)
    cols = torch.rand((1, 4, 5, 9, 3), generator=g)
    run_soft_case("soft_blend", ref, fr, cols, 1e-3, 1e-2, 1.0, (0.1, 0.2, 0.3), 1.0, 100.0)


if __name__ == "__main__":
    main_uniform() if sys.argv[1:] == ["uniform"] else main()
