"""BASELINE cfg5: experiments/eval.py's pose-optimisation benchmark on this package.

Mirrors, call for call, the reference's experiment driver:
  * ``load_cube``       eval.py:727-757  (textured rubiks cube, TexturesUV)
  * ``init_target``     eval.py:183-292  (cube centred / scaled, camera dist 6.7 elev 30 azim 120,
                                         PointLights at (0,2,-2), HardPhongShader K=1 target of a
                                         random_rotations pose)
  * ``init_renderers``  eval.py:124-180  (20 deg perturbation of the true pose; MeshRasterizer with
                                         blur = ln(1e4-1)*sigma, faces_per_pixel=50; RandomPhongShader
                                         with GaussianRast(sigma) [Sr = 16, its default] +
                                         GaussianAgg(nb_samples=MC), or SoftRast + SoftAgg)
  * ``optimize_pose``   eval.py:320-409  (Adam lr 5e-2, best-loss tracking, the grad-norm guard, and
                                         the adaptive schedule of :382-394: EMA of the smoothing
                                         gradients, every 50 iterations after 100 while v_gamma > 0:
                                         blur_radius / sigma / gamma / 1.1, nb_samples x2 up to 128,
                                         lr / 1.5 and a fresh Adam)
  * ``compare_pose_opt`` eval.py:576-661 (NUM_PROB problems x noise types; angle errors, solved
                                         fractions per threshold, the seven json tables)

Execution modes (``--mode``):
  * ``eager``:  the reference loop as written, including its per-iteration host reads (loss value,
                gradient norm, best-loss test).  This is what ``python eval.py`` does.
  * ``graph``:  the same iteration as a captured HIP graph (fwd + bwd + guard + Adam + best-loss
                tracking + the smoothing-gradient EMA, all on the device); the host only decides the
                adaptive schedule every 50 iterations, applies it in place (device smoothing leaves,
                blur radius, learning rate) and captures again only when it changes the sample
                counts.  compare_pose_opt keeps the captured iterations across its problems (one
                GraphSession per noise type; ``--no-graph-reuse`` captures per problem).
                Numerically the same algorithm (same Philox noise stream per iteration).

Multi-GPU (``torchrun --nproc-per-node G -m pertrenderer_amd.pose_opt``): the independent problems
are dealt round-robin to the ranks (one process per GPU), results are gathered on rank 0; no
collective on the data path.  Wall-clock = the slowest rank.
"""
import argparse
import json
import math
import os
import time

import numpy as np
import torch

from . import _native as nat
from . import host_layer
from . import random_rasterizer as rr
from .renderer import (BlendParams, HardPhongShader, Meshes, MeshRasterizer, MeshRenderer, OpenGLPerspectiveCameras,
                       PointLights, RasterizationSettings, Textures, load_obj, look_at_view_transform)
from .renderer.transforms import Rotate, random_rotations, so3_exponential_map, so3_log_map, so3_relative_angle
from .smoothagg import CauchyAgg, GaussianAgg, GaussianAgg_wovr, HardAgg, SoftAgg
from .smoothrast import AffineRast, ArctanRast, GaussianRast, GaussianRast_wovr, HardRast, SoftRast

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "tests", "golden")  # the reference's data/objs/rubiks files
THRESHOLDS = (1, 2, 5, 10, 15, 20, 25, 35, 45)  # eval.py:603
BLUR_FACTOR = math.log(1.0 / 1e-4 - 1.0)  # eval.py:137


def load_cube(device, data_dir=DATA):
    """eval.py:727-757: cube2.obj with its texture strip recoloured face by face from cube_p.npz."""
    with np.load(os.path.join(data_dir, "cube_p.npz")) as f:
        _, _, _, col = f.values()
    vtx_col = torch.from_numpy(col.astype(np.float32))
    green = vtx_col[3, :].clone()  # "reorder color to have same cube as softras"
    vtx_col[3, :] = vtx_col[0, :]
    vtx_col[0, :] = green
    verts, faces, aux = load_obj(os.path.join(data_dir, "cube2.obj"))
    img = aux.texture_images["cube"]
    band = img.size()[1] // 6
    for i in range(6):
        img[:, i * band:(i + 1) * band, :] = vtx_col[i, :][None, None].repeat(img.size()[0], band, 1)
    tex = Textures(verts_uvs=aux.verts_uvs[None], faces_uvs=faces.textures_idx[None], maps=img[None])
    return Meshes(verts=[verts], faces=[faces.verts_idx], textures=tex).to(device)


class Scene:
    """init_target's fixed part (eval.py:239-263): normalised cube, cameras, lights."""

    def __init__(self, device, imsize):
        mesh = load_cube(device)
        v = mesh.verts_packed()
        center = v.mean(0)
        scale = max((v - center).abs().max(0)[0])
        mesh.offset_verts_(-center.expand(v.shape[0], 3))
        mesh.scale_verts_(1.0 / float(scale))
        self.meshes = mesh.extend(1)
        R, T = look_at_view_transform(dist=6.7, elev=torch.linspace(30, 240, 1), azim=torch.linspace(120, 150, 1))
        R, T = R.to(device), T.to(device)
        self.cameras = [OpenGLPerspectiveCameras(device=device, R=R[None, 0], T=T[None, 0], fov=60)]
        self.camera = OpenGLPerspectiveCameras(device=device, R=R[None, 0], T=T[None, 0])
        self.lights = PointLights(device=device, location=[[0.0, 2.0, -2.0]])
        self.device, self.imsize = device, imsize
        self.hard = MeshRenderer(
            MeshRasterizer(cameras=self.camera, raster_settings=RasterizationSettings(
                image_size=imsize, blur_radius=0.0, faces_per_pixel=1, max_faces_per_bin=100000)),
            HardPhongShader(device=device, blend_params=BlendParams(background_color=(0.0, 0.0, 0.0))))

    def target(self):
        """One test problem's target (eval.py:284-292): a random_rotations pose, hard render."""
        R_true = random_rotations(1).to(self.device)
        m = self.meshes.update_padded(Rotate(R_true).transform_points(self.meshes.verts_padded()))
        img = self.hard(m, cameras=self.cameras[0], lights=self.lights)
        return [img[0, ..., :3].detach()], R_true


def init_renderers(scene, R_true, pert_init_intensity=20.0, sigma=1e-3, gamma=1e-2, alpha=1.0, nb_samples=8,
                   noise_type=("softras", "gaussian")):
    """eval.py:124-180 -> (log_rot_init, [MeshRenderer per noise type])."""
    dev = scene.device
    if pert_init_intensity == 0.0:
        R_init = random_rotations(1).to(dev)
    else:
        R_pert = torch.normal(torch.zeros((1, 3), device=dev))
        R_pert = so3_exponential_map((pert_init_intensity * np.pi / 180.0) * R_pert / R_pert.norm(dim=1))
        R_init = torch.bmm(R_true.clone(), R_pert).detach().clone()
    log_rot_init = so3_log_map(R_init)
    blend = BlendParams(sigma=sigma, gamma=gamma, background_color=(0.0, 0.0, 0.0))
    renderers = []
    for nt in noise_type:
        settings = RasterizationSettings(image_size=scene.imsize, blur_radius=BLUR_FACTOR * blend.sigma,
                                         faces_per_pixel=50, max_faces_per_bin=50000, perspective_correct=False)
        rast, agg = {
            "cauchy": lambda: (ArctanRast(sigma=sigma), CauchyAgg(gamma=gamma, alpha=1.0, nb_samples=nb_samples)),
            "gaussian": lambda: (GaussianRast(sigma=sigma), GaussianAgg(gamma=gamma, alpha=1.0, nb_samples=nb_samples)),
            "gaussian_wovr": lambda: (GaussianRast_wovr(sigma=sigma),
                                      GaussianAgg_wovr(gamma=gamma, alpha=1.0, nb_samples=nb_samples)),
            "uniform": lambda: (AffineRast(sigma=sigma), HardAgg()),
            "hard": lambda: (HardRast(), HardAgg()),
            "softras": lambda: (SoftRast(sigma=sigma), SoftAgg(gamma=gamma, alpha=1.0)),
        }[nt]()
        renderers.append(MeshRenderer(
            MeshRasterizer(cameras=scene.camera, raster_settings=settings),
            rr.RandomPhongShader(device=dev, cameras=scene.camera, lights=scene.lights, blend_params=blend,
                                 smoothrast=rast, smoothagg=agg)))
    return log_rot_init, renderers


def _adapt(renderer, i, v, adapt_params, lr, log_rot):
    """eval.py:382-394 for iteration i (> 100); v = [v_sigma, v_gamma, v_alpha] (CPU tensors).
    Returns (new lr or None, v)."""
    sigma, gamma, alpha = renderer.shader.get_smoothing()
    grads = [t.grad if t.grad is not None else torch.zeros_like(t) for t in (sigma, gamma, alpha)]
    v = [0.9 * vi.detach().clone() + 0.1 * g.detach().clone().reshape(vi.shape).cpu() for vi, g in zip(v, grads)]
    for t in (sigma, gamma, alpha):
        if t.grad is not None:
            t.grad = torch.zeros_like(t.grad)
    new_sigma = sigma.detach().clone() / adapt_params[0]
    new_gamma = gamma.detach().clone() / adapt_params[1]
    nb = renderer.shader.get_nb_samples()
    if v[1] > 0 and (i + 1) % 50 == 0:
        s = max(float(new_sigma), 5e-5)
        renderer.rasterizer.raster_settings.blur_radius = BLUR_FACTOR * s
        renderer.shader.update_smoothing(sigma=s, gamma=max(float(new_gamma), 5e-4))
        renderer.shader.update_nb_samples(nb_samples=min(2 * nb, 128))
        return max(lr / 1.5, 1e-4), v
    return None, v


def optimize_pose(scene, init_pose, renderer, target_rgb, lr_init=5e-2, Niter=800, adapt_reg=True,
                  adapt_params=(1.1, 1.1)):
    """eval.py:320-409 (eager, as written).  Returns (best_log_rot, info)."""
    losses, gradient_values = [], []
    log_rot = init_pose.clone().requires_grad_(True)
    lr = lr_init
    optimizer = torch.optim.Adam([log_rot], lr=lr)
    v = [torch.zeros(1), torch.zeros(1), torch.zeros(1)]
    best_log_rot, best_loss = log_rot.clone(), np.inf
    mesh, cams, lights = scene.meshes, scene.cameras, scene.lights
    runtimes = {"forward": [], "backward": []}
    for i in range(Niter):
        R = so3_exponential_map(log_rot)
        predicted = mesh.update_padded(Rotate(R).transform_points(mesh.verts_padded()))
        t1 = time.time()
        images = renderer(predicted, cameras=cams[0], lights=lights)
        loss_rgb = ((images[..., :3] - target_rgb[0]) ** 2).mean()
        t2 = time.time()
        losses.append(loss_rgb.detach().cpu().item())
        optimizer.zero_grad()
        t3 = time.time()
        loss_rgb.backward()
        t4 = time.time()
        lv = loss_rgb.detach().cpu().numpy()
        if lv < best_loss:
            best_loss, best_log_rot = lv, log_rot.clone()
        gradient_values.append(torch.norm(log_rot.grad).detach().cpu().item())
        if gradient_values[-1] > 1000.0:
            log_rot.grad = 1e-5 * torch.normal(torch.zeros_like(log_rot.grad))
        optimizer.step()
        runtimes["forward"].append(t2 - t1)
        runtimes["backward"].append(t4 - t3)
        if adapt_reg and i > 100:
            new_lr, v = _adapt(renderer, i, v, adapt_params, lr, log_rot)
            if new_lr is not None:
                lr = new_lr
                optimizer = torch.optim.Adam([log_rot], lr=lr)
    return best_log_rot, dict(loss_values=losses, gradient_values=gradient_values, runtimes=runtimes,
                              nb_samples=renderer.shader.get_nb_samples())


# ------------------------------------------------------------------ graph mode
def _device_leaves(shader, device):
    """The smoothing leaves as device tensors (same values, requires_grad, zero grads): the
    captured step passes them to the kernels by pointer and accumulates their gradients in place."""
    sr, sa = shader.smoothrast, shader.smoothagg
    for obj, names in ((sr, ("sigma",)), (sa, ("gamma", "alpha"))):
        for name in names:
            t = getattr(obj, name, None)
            if torch.is_tensor(t):
                leaf = torch.tensor(float(t.detach()), device=device, requires_grad=True)
                leaf.grad = torch.zeros_like(leaf)
                setattr(obj, name, leaf)


def _fresh_adam(log_rot, lr):
    """torch.optim.Adam([log_rot], lr) with its state initialised up front (capturable, fused, the
    learning rate a device tensor): the same state a new optimizer starts from (eval.py:337)."""
    lr_t = torch.tensor(float(lr), dtype=torch.float32, device=log_rot.device)
    opt = torch.optim.Adam([log_rot], lr=lr_t, capturable=True, fused=True)
    opt.state[log_rot] = {"step": torch.zeros((), dtype=torch.float32, device=log_rot.device),
                          "exp_avg": torch.zeros_like(log_rot), "exp_avg_sq": torch.zeros_like(log_rot)}
    return opt


def _renew_adam(opt, log_rot, lr):
    """eval.py:394's new torch.optim.Adam(lr) in place: the state zeroed and the device learning
    rate rewritten, so a captured step keeps addressing the same tensors."""
    with torch.no_grad():
        for t in opt.state[log_rot].values():
            t.zero_()
        opt.param_groups[0]["lr"].fill_(float(lr))


def rgb_mse(images, target):
    """eval.py:352-353's loss on the native kernels: the C++ autograd node (host_layer.py) when it
    is in use, else the Python Function (_RgbMse); the same launches either way.  The native
    nodes differentiate the images only: a target that requires grad takes eval.py's torch
    expression, so its gradient is not dropped."""
    if torch.is_tensor(target) and target.requires_grad and torch.is_grad_enabled():
        return ((images[..., :3] - target) ** 2).mean()
    ext = host_layer.get()
    if ext is not None and images.is_cuda and target.is_cuda:
        return ext.rgb_mse(images, target)
    return _RgbMse.apply(images, target)


class _RgbMse(torch.autograd.Function):
    """((images[..., :3] - target) ** 2).mean() (experiments/eval.py:352-353) on the native kernels
    pr_rgb_mse_fwd / pr_rgb_mse_bwd: images (N,H,W,C>=3) float32, target (H,W,3) broadcast over
    the batch or (N,H,W,3).  Sums in a fixed order (deterministic); gradient (g / 3P) * 2 (x - t)."""

    @staticmethod
    def _args(img, t):
        N, H, W, C = img.shape
        if img.dtype != torch.float32 or t.dtype != torch.float32 or C < 3 or t.shape[-1] != 3:
            raise ValueError("rgb_mse: float32 (N,H,W,C>=3) images and (..,H,W,3) target expected")
        if t.numel() not in (H * W * 3, N * H * W * 3):
            raise ValueError(f"rgb_mse: target {tuple(t.shape)} does not broadcast to {(N, H, W, 3)}")
        a = nat.PRRgbMseArgs()
        a.P, a.C, a.HW = N * H * W, C, H * W
        a.target_batched = int(t.numel() == N * H * W * 3 and N > 1)
        a.image, a.target = nat.ptr(img), nat.ptr(t)
        return a

    @staticmethod
    def forward(ctx, images, target):
        img, t = images.detach().contiguous(), target.detach().contiguous()
        a = _RgbMse._args(img, t)
        loss = torch.empty((), dtype=torch.float32, device=img.device)
        part = torch.empty(nat.load().pr_rgb_mse_workspace(a.P), dtype=torch.float32, device=img.device)
        a.loss, a.partials = nat.ptr(loss), nat.ptr(part)
        nat.call("pr_rgb_mse_fwd", "rgb_mse_fwd", img, a)
        ctx.save_for_backward(img, t)
        return loss

    @staticmethod
    def backward(ctx, g):
        img, t = ctx.saved_tensors
        a = _RgbMse._args(img, t)
        gi = torch.empty_like(img)
        gl = g.detach().to(torch.float32).contiguous()
        a.grad_loss, a.grad_image = nat.ptr(gl), nat.ptr(gi)
        nat.call("pr_rgb_mse_bwd", "rgb_mse_bwd", img, a)
        return gi, None


class _CapturedIteration:
    """One optimize_pose iteration (eval.py:343-388) as a HIP graph for a fixed schedule state
    (nb_samples, blur_radius, lr): noise key advance, so3 pose, render, L2 loss, backward,
    loss / grad-norm records, best-loss tracking, the grad-norm guard, Adam, and (post) the EMA
    of the smoothing gradients with their zeroing."""

    def __init__(self, scene, renderer, target, log_rot, st, opt, post, seed, pool):
        self.scene, self.renderer, self.target, self.log_rot = scene, renderer, target, log_rot
        self.st, self.opt, self.post, self.seed = st, opt, post, seed
        leaves = list(renderer.shader.get_smoothing())
        self.leaves = leaves
        # warm-up pass on a side stream (lazy allocations and caches outside the graph); it must
        # not change the optimisation state, which lives in st (the smoothing gradients' running
        # sum is st["acc"]): the gradients it leaves are dropped
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self.seed.advance()
            self._forward().backward()
        torch.cuda.current_stream().wait_stream(side)
        for l in leaves:
            if torch.is_tensor(l):
                l.grad = None
        log_rot.grad = None
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, pool=pool):
            self._body()

    def _forward(self):
        mesh = self.scene.meshes
        R = so3_exponential_map(self.log_rot)
        predicted = mesh.update_padded(Rotate(R).transform_points(mesh.verts_padded()))
        images = self.renderer(predicted, cameras=self.scene.cameras[0], lights=self.scene.lights)
        # eval.py:352-353's ((images[..., :3] - target) ** 2).mean() as two native kernels forward
        # and one backward (pr_rgb_mse_*) instead of ~10 torch kernels.  It also keeps the loss off
        # torch's one-pass cross-workgroup mean, which on this PyTorch-ROCm build an eager BLAS
        # call (init_renderers' bmm, angle_deg) between the replays of a kept graph leaves wrong:
        # GraphSession's reused graphs recorded stale losses with it and tracked the wrong best
        # pose (tools/scratch/graph_mean_repro.py, profiles/r5/cfg5_graph_reuse.md).
        return rgb_mse(images, self.target)

    def _body(self):
        st, log_rot = self.st, self.log_rot
        self.seed.advance()
        loss = self._forward()
        # optimizer.zero_grad() as set_to_none, and the smoothing leaves' gradients too: the
        # backward's own buffers become the gradients (AccumulateGrad takes them) instead of a fill
        # and an add per leaf; pr_pose_step keeps the leaves' running sum (eval.py accumulates
        # sigma.grad etc. until the EMA reads and zeroes them) in st["acc"]
        log_rot.grad = None
        for l in self.leaves:
            if torch.is_tensor(l):
                l.grad = None
        loss.backward()
        if log_rot.grad is None:
            raise RuntimeError("pose step: the loss does not reach log_rot")
        # the records, best-loss pose, grad-norm guard, (post) smoothing-gradient EMA and the
        # iteration counter in one native kernel (pr_pose_step) instead of ~20 one-element torch ops
        a = nat.PRPoseStepArgs()
        a.loss, a.log_rot, a.grad, a.it = nat.ptr(loss), nat.ptr(log_rot), nat.ptr(log_rot.grad), nat.ptr(st["it"])
        a.losses, a.gnorms = nat.ptr(st["losses"]), nat.ptr(st["gnorms"])
        a.best_loss, a.best, a.v, a.acc = nat.ptr(st["best_loss"]), nat.ptr(st["best"]), nat.ptr(st["v"]), nat.ptr(st["acc"])
        for i, l in enumerate(self.leaves[:3]):
            g = l.grad if torch.is_tensor(l) else None
            if g is not None and (g.dtype != torch.float32 or g.numel() != 1 or not g.is_cuda):
                raise RuntimeError("pose step: smoothing gradients must be one-element float32 device tensors")
            a.leaf_grad[i] = nat.ptr(g)
        a.seed = nat.ptr(self.seed.tensor)
        # and optimizer.step(): the Adam update on the same thread (self.opt holds the state and the
        # device learning rate; _renew_adam resets them in place)
        ost = self.opt.state[log_rot]
        a.exp_avg, a.exp_avg_sq, a.step = nat.ptr(ost["exp_avg"]), nat.ptr(ost["exp_avg_sq"]), nat.ptr(ost["step"])
        a.lr, a.adam = nat.ptr(self.opt.param_groups[0]["lr"]), 1
        a.niter, a.n, a.post = st["losses"].numel(), log_rot.numel(), int(self.post)
        nat.call("pr_pose_step", "pose_step", loss, a)

    def replay(self, n):
        for _ in range(n):
            self.graph.replay()


def _nb(sh):
    """(Sr, Sa) of a perturbed shader: the launch-time sample counts a captured step bakes in."""
    return (getattr(sh.smoothrast, "nb_samples", None), getattr(sh.smoothagg, "nb_samples", None))


class GraphSession:
    """The captured iterations of optimize_pose_graph kept across the problems of one benchmark
    run (compare_pose_opt / compare_runtime: one session per renderer configuration).  The first
    call adopts its renderer and sizes every tensor a captured step addresses (the pose and its
    gradient, the target, the loss records, Adam's state and learning rate, the noise key, the
    blur radius, the smoothing leaves); later calls reset those in place to their problem's start
    and replay the graphs already captured for each (phase, Sr, Sa) -- a problem then captures only
    at sample counts no earlier problem reached.  The later calls' own renderers must be configured
    as the adopted one (init_renderers with the same arguments); only their starting values are
    taken from the call."""

    def __init__(self):
        self.renderer = None
        self.graphs = {}

    def bind(self, scene, init_pose, renderer, target_rgb, lr_init, Niter):
        from . import noise
        dev = scene.device
        if self.renderer is None:
            sh = renderer.shader
            self.renderer, self.scene, self.Niter = renderer, scene, Niter
            sr, sa = sh.smoothrast, sh.smoothagg
            f = lambda t: float(t.detach()) if torch.is_tensor(t) else float(t)
            self.start = dict(sigma=f(sr.sigma), gamma=f(sa.gamma), alpha=f(sa.alpha), nb=_nb(sh),
                              blur=float(renderer.rasterizer.raster_settings.blur_radius))
            _device_leaves(sh, dev)
            self.seed = noise.DeviceSeed(dev)
            self.log_rot = init_pose.clone().detach().to(dev).requires_grad_(True)
            self.log_rot.grad = torch.zeros_like(self.log_rot)
            self.target = target_rgb[0].clone()
            self.st = dict(it=torch.zeros((), dtype=torch.int64, device=dev), losses=torch.zeros(Niter, device=dev),
                           gnorms=torch.zeros(Niter, device=dev), best_loss=torch.full((), float("inf"), device=dev),
                           best=self.log_rot.detach().clone(), v=torch.zeros(3, device=dev),
                           acc=torch.zeros(3, device=dev))
            self.opt = _fresh_adam(self.log_rot, lr_init)
            self.blur = torch.tensor(self.start["blur"], dtype=torch.float32, device=dev)
        else:
            if scene is not self.scene or Niter != self.Niter or type(renderer.shader) is not type(self.renderer.shader):
                raise ValueError("GraphSession: a call with another scene, iteration count or shader")
            sh = self.renderer.shader
            z = self.start
            with torch.no_grad():
                for t, v in ((sh.smoothrast.sigma, z["sigma"]), (sh.smoothagg.gamma, z["gamma"]),
                             (sh.smoothagg.alpha, z["alpha"])):
                    if torch.is_tensor(t):
                        t.fill_(v)
                        t.grad = None
                if z["nb"][0] is not None:
                    sh.smoothrast.nb_samples = z["nb"][0]
                if z["nb"][1] is not None:
                    sh.smoothagg.nb_samples = z["nb"][1]
                self.blur.fill_(z["blur"])
                self.log_rot.copy_(init_pose.to(dev))
                if self.log_rot.grad is not None:
                    self.log_rot.grad.zero_()
                self.target.copy_(target_rgb[0])
                st = self.st
                st["it"].zero_()
                st["losses"].zero_()
                st["gnorms"].zero_()
                st["best_loss"].fill_(float("inf"))
                st["best"].copy_(self.log_rot)
                st["v"].zero_()
                st["acc"].zero_()
                self.seed.tensor.fill_(noise.draw_key())  # a new problem's key, as a new DeviceSeed draws
                self.seed._next, self.seed._pending = 1, 0
            _renew_adam(self.opt, self.log_rot, lr_init)
        self.renderer.rasterizer.raster_settings.blur_radius = self.blur
        noise.use_device_seed(self.seed)

    def step(self, post):
        """The captured iteration for the current phase and sample counts (captured on first use)."""
        key = (post,) + _nb(self.renderer.shader)
        cur = self.graphs.get(key)
        if cur is None:
            # each graph its own memory pool: graphs sharing a pool may only replay in capture order,
            # and a session replays its first-phase graph again after the later ones were captured
            cur = _CapturedIteration(self.scene, self.renderer, self.target, self.log_rot, self.st, self.opt, post,
                                     self.seed, torch.cuda.graph_pool_handle())
            self.graphs[key] = cur
        return cur


def optimize_pose_graph(scene, init_pose, renderer, target_rgb, lr_init=5e-2, Niter=800, adapt_reg=True,
                        adapt_params=(1.1, 1.1), session=None):
    """optimize_pose (eval.py:320-409) with every iteration a graph replay.  The host only acts at
    the schedule's decision points (i > 100 with (i+1) % 50 == 0, eval.py:389): it reads v_gamma
    and applies the smoothing / blur / lr update in place -- the smoothing leaves, the blur radius
    (a device float the rasterizer reads, PRRastArgs.blur_radius_dev) and Adam's learning rate
    and state are device tensors the captured step addresses -- so it captures again only when
    the sample counts change (launch arguments).  `session` (GraphSession) keeps the captured
    iterations for the next problem.  Returns (best_log_rot, info)."""
    from . import noise
    ses = GraphSession() if session is None else session
    ses.bind(scene, init_pose, renderer, target_rgb, lr_init, Niter)
    sh, st, rs = ses.renderer.shader, ses.st, ses.renderer.rasterizer.raster_settings
    lr = lr_init
    i = 0
    try:
        while i < Niter:
            post = adapt_reg and i > 100
            if post:
                end = min(Niter, i + (49 - i % 50) + 1)  # through the next i with (i+1) % 50 == 0
            else:
                end = min(Niter, 101) if adapt_reg else Niter
            ses.step(post).replay(end - i)
            i = end
            if post and i % 50 == 0:  # the last replayed iteration had (i+1) % 50 == 0
                v_gamma = float(st["v"][1])
                if v_gamma > 0:
                    sigma, gamma, _ = sh.get_smoothing()
                    s = max(float(sigma.detach()) / adapt_params[0], 5e-5)
                    g = max(float(gamma.detach()) / adapt_params[1], 5e-4)
                    with torch.no_grad():
                        ses.blur.fill_(BLUR_FACTOR * s)
                        sh.smoothrast.sigma.fill_(s)
                        sh.smoothagg.gamma.fill_(g)
                        sh.smoothagg.alpha.fill_(1.0)
                    sh.update_nb_samples(nb_samples=min(2 * sh.get_nb_samples(), 128))
                    lr = max(lr / 1.5, 1e-4)
                    _renew_adam(ses.opt, ses.log_rot, lr)
    finally:
        noise.use_device_seed(None)
        rs.blur_radius = float(ses.blur)  # back to PyTorch3D's float (one host read, at the end)
    torch.cuda.synchronize()
    info = dict(loss_values=st["losses"].cpu().tolist(), gradient_values=st["gnorms"].cpu().tolist(),
                nb_samples=sh.get_nb_samples())
    return st["best"].detach().clone(), info


def angle_deg(log_rot, R_true):
    return so3_relative_angle(so3_exponential_map(log_rot), R_true).detach().cpu().item() * 180.0 / np.pi


def make_problems(scene, num_prob, noise_type, pert):
    """compare_pose_opt's test problems (eval.py:605-609): targets and initial poses."""
    problems = []
    for _ in range(num_prob):
        target_rgb, R_true = scene.target()
        log_rot_init, _ = init_renderers(scene, R_true, pert_init_intensity=pert, sigma=0.1, gamma=0.1, nb_samples=1,
                                         noise_type=noise_type)
        problems.append(([t.clone() for t in target_rgb], R_true.clone(), log_rot_init.detach().clone()))
    return problems


def run_problem(scene, problem, noise_type, sigma, gamma, nb_mc, pert, niter, adapt_reg, adapt_params, mode,
                sessions=None):
    """One compare_pose_opt problem for every noise type.  `sessions` (a dict kept by the caller
    across problems; graph mode): one GraphSession per noise type, so the captured iterations of
    earlier problems are replayed instead of captured again."""
    target_rgb, R_true, log_rot_init = problem
    _, renderers = init_renderers(scene, R_true, pert_init_intensity=pert, sigma=sigma, gamma=gamma,
                                  nb_samples=nb_mc, noise_type=noise_type)
    out = {}
    for nt, renderer in zip(noise_type, renderers):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "graph":
            ses = None if sessions is None else sessions.setdefault(nt, GraphSession())
            log_rot, info = optimize_pose_graph(scene, log_rot_init, renderer, target_rgb, Niter=niter,
                                                adapt_reg=adapt_reg, adapt_params=adapt_params, session=ses)
        else:
            log_rot, info = optimize_pose(scene, log_rot_init, renderer, target_rgb, Niter=niter, adapt_reg=adapt_reg,
                                          adapt_params=adapt_params)
        torch.cuda.synchronize()
        out[nt] = dict(seconds=time.perf_counter() - t0, init_error=angle_deg(log_rot_init, R_true),
                       final_error=angle_deg(log_rot, R_true), final_nb_samples=info["nb_samples"],
                       final_loss=info["loss_values"][-1], iterations=niter)
    return out


def compare_runtime(scene, num_prob, noise_type, smoothing_list, mc_list, pert=20.0, niter=800, adapt_reg=True,
                    adapt_params=(1.1, 1.1), lr_list=(5e-2,), mode="eager", out=None):
    """eval.py compare_runtime (experiments/eval.py:506-574) on the cube scene (ShapeNet is not
    available here; eval.py's pose benchmark uses the same cube): for every (lr, (sigma, gamma),
    MC) setting and test problem, the wall time of one whole optimize_pose run and the peak
    device memory (torch.cuda.max_memory_allocated, MB) per noise type.  Returns (mean_runtimes,
    mean_memory, params) shaped as eval.py's runtimes.txt / memory.txt: {noise: [[per problem]
    per setting]}; writes them (results.write_runtime_results) when `out` is given."""
    device = scene.device
    problems = make_problems(scene, num_prob, noise_type, pert)
    mean_runtimes = {nt: [] for nt in noise_type}
    mean_memory = {nt: [] for nt in noise_type}
    params = {"lr-smoothing-MC": [], "lr": [], "sigma": [], "gamma": [], "MC": [], "adapt_params": []}
    for lr in lr_list:
        for sigma, gamma in smoothing_list:
            for nb_mc in mc_list:
                runtimes = {nt: [] for nt in noise_type}
                memory = {nt: [] for nt in noise_type}
                for target_rgb, R_true, log_rot_init in problems:
                    _, renderers = init_renderers(scene, R_true, pert_init_intensity=pert, sigma=sigma, gamma=gamma,
                                                  nb_samples=nb_mc, noise_type=noise_type)
                    for nt, renderer in zip(noise_type, renderers):
                        torch.cuda.synchronize(device)
                        torch.cuda.reset_peak_memory_stats(device)  # eval.py:548
                        t0 = time.perf_counter()
                        run = optimize_pose_graph if mode == "graph" else optimize_pose
                        run(scene, log_rot_init, renderer, target_rgb, lr_init=lr, Niter=niter, adapt_reg=adapt_reg,
                            adapt_params=adapt_params)
                        torch.cuda.synchronize(device)
                        runtimes[nt].append(time.perf_counter() - t0)
                        memory[nt].append(torch.cuda.max_memory_allocated(device) * 1e-6)  # MB, eval.py:555
                for nt in noise_type:
                    mean_runtimes[nt].append(runtimes[nt])
                    mean_memory[nt].append(memory[nt])
                params["lr-smoothing-MC"].append((lr, sigma, gamma, nb_mc))
                params["lr"].append(lr)
                params["sigma"].append(sigma)
                params["gamma"].append(gamma)
                params["MC"].append(nb_mc)
                params["adapt_params"].append(adapt_params)
    if out:
        from . import results as res
        res.write_runtime_results(out, mean_runtimes, mean_memory)
    return mean_runtimes, mean_memory, params


def tables(per_problem, noise_type, params, exp_setup):
    """compare_pose_opt's json tables (eval.py:632-661) for one parameter setting."""
    mean_errors, var_errors, init_errors, final_errors = {}, {}, {}, {}
    mean_solved = {}
    for nt in noise_type:
        err = [p[nt]["final_error"] for p in per_problem]
        mean_errors[nt] = [sum(err) / len(err)]
        var_errors[nt] = [float(np.std(err))]
        init_errors[nt] = [[p[nt]["init_error"] for p in per_problem]]
        final_errors[nt] = [err]
        mean_solved[nt] = {th: [sum(1 if a < th else 0 for a in err) / len(err)] for th in THRESHOLDS}
    return dict(mean_errors=mean_errors, final_errors=final_errors, init_errors=init_errors, var_errors=var_errors,
                mean_solved=mean_solved, params=params, exp_setup=exp_setup)


def main(argv=None):
    ap = argparse.ArgumentParser(description="eval.py compare_pose_opt (BASELINE cfg5) on pertrenderer_amd")
    ap.add_argument("-np", "--num-prob", type=int, default=100)
    ap.add_argument("-ni", "--num-iterations", type=int, default=800)
    ap.add_argument("-is", "--image-size", type=int, default=256)
    ap.add_argument("-sn", "--smoothing-noise", nargs="+", default=["softras", "gaussian"])
    ap.add_argument("-mc", "--mc-samples", type=int, default=8)
    ap.add_argument("-sv", "--smoothing", type=float, nargs=2, default=(1e-3, 1e-2))
    ap.add_argument("-ip", "--initial-perturbation", type=float, default=20.0)
    ap.add_argument("-ar", "--adaptive-regularization", type=int, default=1)
    ap.add_argument("-s", "--seed", type=int, default=1)
    ap.add_argument("--mode", choices=["eager", "graph"], default="eager")
    ap.add_argument("--no-graph-reuse", action="store_true",
                    help="graph mode: capture every problem's iterations anew instead of keeping them across "
                         "problems (GraphSession; profiles/r5/cfg5_graph_reuse.md)")
    ap.add_argument("--out", default=None, help="directory for eval.py's tables + summary.json")
    ap.add_argument("--runtime", action="store_true",
                    help="eval.py compare_runtime instead: runtimes.txt / memory.txt per MC setting")
    ap.add_argument("-mcl", "--mc-list", type=int, nargs="+", default=None, help="--runtime: MC settings")
    args = ap.parse_args(argv)
    if args.runtime:
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(device)
        torch.manual_seed(args.seed)
        scene = Scene(device, args.image_size)
        rt, mem, params = compare_runtime(scene, args.num_prob, list(args.smoothing_noise), [tuple(args.smoothing)],
                                          args.mc_list or [args.mc_samples], pert=args.initial_perturbation,
                                          niter=args.num_iterations, adapt_reg=bool(args.adaptive_regularization),
                                          mode=args.mode, out=args.out)
        print(json.dumps({"runtimes": rt, "memory_mb": mem, "params": params}), flush=True)
        return 0

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # results only: a handful of floats per problem
    torch.manual_seed(args.seed)
    t_setup = time.perf_counter()
    scene = Scene(device, args.image_size)
    noise_type = list(args.smoothing_noise)
    problems = make_problems(scene, args.num_prob, noise_type, args.initial_perturbation)
    sigma, gamma = args.smoothing
    adapt_params = (1.1, 1.1)
    mine = list(range(rank, args.num_prob, world))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    results = {}
    sessions = None if args.no_graph_reuse else {}  # graph mode: captured iterations kept across problems
    for i in mine:
        results[i] = run_problem(scene, problems[i], noise_type, sigma, gamma, args.mc_samples,
                                 args.initial_perturbation, args.num_iterations, bool(args.adaptive_regularization),
                                 adapt_params, args.mode, sessions=sessions)
        if rank == 0:
            print(json.dumps({"problem": i, **{nt: {k: round(v, 4) if isinstance(v, float) else v
                                                    for k, v in r.items()} for nt, r in results[i].items()}}),
                  flush=True)
    wall = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        gathered = [None] * world
        dist.all_gather_object(gathered, (results, wall))
        results = {k: v for res, _ in gathered for k, v in res.items()}
        wall = max(w for _, w in gathered)
        dist.destroy_process_group()
    if rank != 0:
        return 0
    per_problem = [results[i] for i in sorted(results)]
    params = {"lr-smoothing-MC": [(5e-2, sigma, gamma, args.mc_samples)], "lr": [5e-2], "sigma": [sigma],
              "gamma": [gamma], "MC": [args.mc_samples], "adapt_params": [adapt_params]}
    exp_setup = {"perturbation": args.initial_perturbation, "Niter": args.num_iterations, "optimizer": "adam",
                 "N_benchmark": args.num_prob, "adaptive_regularization": args.adaptive_regularization,
                 "category": ["cube"]}
    tab = tables(per_problem, noise_type, params, exp_setup)
    summary = {
        "workload": f"eval.py compare_pose_opt: cube (TexturesUV) + RandomPhongShader, {args.image_size}^2, "
                    f"faces_per_pixel=50, {args.num_prob} problems x {args.num_iterations} iterations, "
                    f"noise {noise_type}, MC={args.mc_samples} (GaussianRast Sr=16 default), adaptive schedule "
                    f"{'on' if args.adaptive_regularization else 'off'}",
        "mode": args.mode, "n_gpus": world, "wall_clock_s": round(wall, 3), "setup_s": round(t0 - t_setup, 3),
        "per_noise": {}}
    for nt in noise_type:
        secs = [p[nt]["seconds"] for p in per_problem]
        summary["per_noise"][nt] = {
            "mean_seconds_per_problem": round(float(np.mean(secs)), 4),
            "ms_per_iteration": round(1e3 * float(np.mean(secs)) / args.num_iterations, 4),
            "mean_final_error_deg": round(tab["mean_errors"][nt][0], 4),
            "std_final_error_deg": round(tab["var_errors"][nt][0], 4),
            "mean_init_error_deg": round(float(np.mean(tab["init_errors"][nt][0])), 4),
            "solved": {str(th): tab["mean_solved"][nt][th][0] for th in THRESHOLDS},
            "final_nb_samples": sorted({p[nt]["final_nb_samples"] for p in per_problem}),
        }
    print(json.dumps(summary), flush=True)
    if args.out:
        from . import results as res
        res.write_pose_results(args.out, **tab)
        with open(os.path.join(args.out, "summary.json"), "w") as f:
            json.dump({"summary": summary, "per_problem": per_problem}, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
