"""Benchmark of the perturbed-renderer hot path (BASELINE.json configs[1]).

One step = one pose-optimisation iteration of experiments/eval.py:343-376: rotate the mesh
(so3 exp map), MeshRasterizer (native K-nearest rasterizer, 256x256, faces_per_pixel=50,
blur = ln(1/1e-4 - 1)*sigma), RandomSimpleShader with GaussianRast(nb_samples=8) +
GaussianAgg(nb_samples=8) (fused native blend with TexturesVertex sampling), L2 loss to a fixed
synthetic target, backward through blend -> rasterizer -> vertices -> pose, Adam step on the
pose (lr 5e-2, eval.py:337).  The whole step is one captured HIP graph.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|eval]
    python bench.py --gpus N ...                        (starts N rank processes itself, RCCL)
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL; --gpus must equal N)

Multi-GPU (--shard):
  samples (default at N > 1, the north star's partition, strong scaling): every rank renders the
          same frame with its shard of the config's Monte-Carlo samples (parallel.sample_shard:
          global sample offsets, shared Philox keys) and one RCCL all-reduce forms the full-S
          gradient estimate (weights n_r / S).  value = distinct frames / s (each frame counted
          once).  The rasterizer and pose kernels are replicated on every rank: the line reports
          their per-rank time ("strong_scaling": replicated vs sharded ms, and the speed-up bound).
  frames  (weak scaling): every rank renders its OWN view of the shared pose (camera azimuth
          120 + 360 r / N: a multi-view pose optimisation step) and one RCCL all-reduce averages
          the pose / smoothing gradients.  value = distinct frames / s.

Prints ONE JSON line on rank 0: `value` = frames/s (forward + backward per frame) over all
ranks; `ms_forward` / `ms_backward` = HIP events around separately captured forward and
backward(+Adam) graphs replayed right after the timed region; `roofline` is the dominant native
call's algorithmic HBM bytes / its HIP-event duration; `cpu_baseline` times the CPU oracle
(test-infrastructure restatement of the reference + PyTorch3D rasterizer) on a bounded sample of
the same workload, on rank 0 at N=1, with every CPU this process may use.
"""
import argparse
import json
import math
import os
import sys
import time


def _launch_ranks():
    """`python bench.py --gpus N` (N > 1) without a launcher: start N rank processes, one per GPU,
    as torchrun would (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), and exit
    with the first failing rank's code.  This parent imports neither torch nor the package, so it
    never touches the device; each child dies with it (PR_SET_PDEATHSIG).  Under a launcher
    (WORLD_SIZE set) a --gpus that differs from WORLD_SIZE is an error: the line would misreport
    n_gpus."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    n = pre.parse_known_args()[0].gpus
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != n:
            sys.stderr.write(f"bench.py: --gpus {n} but the launcher started WORLD_SIZE="
                             f"{os.environ['WORLD_SIZE']} ranks\n")
            sys.exit(2)
        return
    if n <= 1:
        return
    import ctypes
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    libc = ctypes.CDLL(None, use_errno=True)

    def _die_with_parent():
        libc.prctl(1, signal.SIGKILL)  # PR_SET_PDEATHSIG

    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      preexec_fn=_die_with_parent))
    code = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0 and code == 0:
                    code = rc if rc > 0 else 128 - rc
                    for q in live:  # one rank failed: the collectives of the others would hang
                        q.kill()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    sys.exit(code)


if __name__ == "__main__":
    _launch_ranks()

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import pertrenderer_amd as pa  # noqa: E402
from pertrenderer_amd.renderer import (FoVPerspectiveCameras, MeshRasterizer, MeshRenderer, Meshes,  # noqa: E402
                                       RasterizationSettings, TexturesVertex, load_obj, look_at_view_transform)
from pertrenderer_amd.renderer.transforms import Rotate, so3_exponential_map  # noqa: E402
from pertrenderer_amd.parallel import average_gradients, sample_shard  # noqa: E402
from pertrenderer_amd.timing import KernelTimer  # noqa: E402
from pertrenderer_amd.build_native import source_sha  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def load_mesh(device, name="sphere_642.obj"):
    """A reference data mesh (data/objs, copied to tests/golden), centred, max |coord| = 1."""
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", name))
    center = verts.mean(0)
    verts = verts - center
    verts = verts / verts.abs().max()
    return verts.to(device), faces.verts_idx.to(device)


def load_sphere(device):
    return load_mesh(device, "sphere_642.obj")


# BASELINE.json configs: cfg2 is the headline (metric's) workload; cfg3/cfg4 are the batch
# configurations (16 meshes alternating sphere_642 / cube2, each with its own pose); "eval" is
# eval.py's own renderer (textured cube, RandomPhongShader, GaussianRast's default Sr=16, Sa=8)
RNG_PEAK_NORMALS_PER_S = 2.76e12  # measured generator throughput per MI355X, Philox4x32-7 + Box-Muller (DESIGN.md §4 Noise)

CONFIGS = {
    "cfg2": dict(batch=1, image_size=256, K=50, samples=8),
    "cfg3": dict(batch=16, image_size=256, K=100, samples=16),
    "cfg4": dict(batch=16, image_size=512, K=150, samples=64),
    "eval": dict(batch=1, image_size=256, K=50, samples=8, rast_samples=16),
}


class Workload:
    def __init__(self, device, image_size=256, K=50, samples=8, sigma=1e-3, gamma=1e-2, dist_cam=2.7, seed=0,
                 batch=1, azim=120.0, rast_samples=None, eval_scene=False, loss="native"):
        self.device = device
        self.loss_kind = loss
        g = torch.Generator().manual_seed(seed)
        Sr = samples if rast_samples is None else rast_samples
        blend = pa.random_rasterizer.BlendParams(sigma, gamma, (0.0, 0.0, 0.0))
        self.rast = pa.GaussianRast(nb_samples=Sr, sigma=sigma)
        self.agg = pa.GaussianAgg(nb_samples=samples, gamma=gamma, alpha=1.0)
        self.settings = RasterizationSettings(image_size=image_size,
                                              blur_radius=math.log(1.0 / 1e-4 - 1.0) * sigma,
                                              faces_per_pixel=K, max_faces_per_bin=50000,
                                              perspective_correct=False)
        if eval_scene:  # eval.py:124-180, 727-757: textured cube, Phong, camera at 6.7
            from pertrenderer_amd import pose_opt
            scene = pose_opt.Scene(device, image_size)
            self.base, self.lights = scene.meshes, scene.lights
            R, T = look_at_view_transform(6.7, 30.0, azim, device=device)
            self.cameras = FoVPerspectiveCameras(R=R, T=T, device=device, fov=60.0)
            shader = pa.RandomPhongShader(device=device, cameras=self.cameras, lights=self.lights,
                                          smoothrast=self.rast, smoothagg=self.agg, blend_params=blend)
            faces = self.base.faces_packed()
        else:
            vl, fl, cl = [], [], []
            for i in range(batch):
                verts, faces = load_mesh(device, "sphere_642.obj" if i % 2 == 0 else "cube2.obj")
                vl.append(verts)
                fl.append(faces)
                cl.append(torch.rand((verts.shape[0], 3), generator=g).to(device))
            self.base = Meshes(vl, fl, TexturesVertex(cl))
            faces = torch.cat(fl)
            R, T = look_at_view_transform(dist_cam, 30.0, azim, device=device)
            self.cameras = FoVPerspectiveCameras(R=R, T=T, device=device, fov=60.0)
            self.lights = None
            shader = pa.RandomSimpleShader(device=device, cameras=self.cameras, smoothrast=self.rast,
                                           smoothagg=self.agg, blend_params=blend)
        self.renderer = MeshRenderer(rasterizer=MeshRasterizer(cameras=self.cameras, raster_settings=self.settings),
                                     shader=shader)
        self.log_rot = (0.3 * torch.randn((batch, 3), generator=g)).to(device).requires_grad_(True)
        self.target = torch.rand((batch, image_size, image_size, 3), generator=g).to(device)
        # loss.backward()'s seed gradient, made once (a captured step then holds no fill kernel for it)
        self.one = torch.ones((), device=device)
        self.K, self.S, self.Sr, self.H, self.batch = K, samples, Sr, image_size, batch
        self.F = faces.shape[0]

    def params(self):
        return [self.log_rot, self.rast.sigma, self.agg.gamma, self.agg.alpha]

    def device_scalars(self):
        """Smoothing leaves on the device (graph mode): no host sync inside the step."""
        mk = lambda t: torch.tensor(float(t.detach()), device=self.device, requires_grad=True)
        self.rast.sigma, self.agg.gamma, self.agg.alpha = mk(self.rast.sigma), mk(self.agg.gamma), mk(self.agg.alpha)

    def forward(self):
        R = so3_exponential_map(self.log_rot)
        mesh = self.base.update_padded(Rotate(R).transform_points(self.base.verts_padded()))
        kw = {"lights": self.lights} if self.lights is not None else {}
        images = self.renderer(mesh, cameras=self.cameras, **kw)
        if self.loss_kind == "native":
            # eval.py:352-353's ((images[..., :3] - target) ** 2).mean() on the package's fused loss
            # kernels (pose_opt._RgbMse, pr_rgb_mse_*: 2 forward + 1 backward launches, fp32 summation
            # order only) -- cfg 5's captured step uses the same; --loss torch: the 11-kernel torch
            # composition
            from pertrenderer_amd.pose_opt import rgb_mse
            return rgb_mse(images, self.target)
        return ((images[..., :3] - self.target) ** 2).mean()

    def zero_grad(self):
        for p in self.params():
            p.grad = None


def kernel_bytes(name, P, K, S, F):
    """Algorithmic HBM bytes per launch (int64 pix_to_face)."""
    slots = P * K
    return {
        "blend_fwd": slots * (8 + 4 + 4 + 12) + P * 16 + P * S,           # p2f,dists,zbuf,colors | image, winners
        "blend_bwd": slots * (8 + 4 + 4 + 12 + 4 + 4 + 12) + P * 16 + P * S,  # + d dists,d zbuf,d colors | d image
        "rast_fwd": slots * (8 + 4 + 12 + 4) + F * 36,                   # p2f,zbuf,bary,dists | face verts
        "rast_bwd": slots * (8 + 4 + 12 + 4) + F * 36 * 2,               # p2f + 3 upstream grads | verts, grads
    }.get(name)


def dense_roofline(device, P_side=256, K=50, S=8, iters=20, N=1, Sr=None):
    """Blend kernels on dense synthetic fragments (every slot valid) at a configuration's shape
    (N images of P_side^2, K, Sr / Sa samples) — the bandwidth microbench of SURVEY §8(d); the
    real meshes' fragments are mostly padding (2/3 of the slots at cfg 2, 93 % at cfg 4), which
    the kernels never read, so only dense fragments give a meaningful fraction of HBM peak."""
    g = torch.Generator(device).manual_seed(0)
    H = W = P_side
    Sr = S if Sr is None else Sr
    p2f = torch.randint(0, 5000, (N, H, W, K), generator=g, device=device)
    dists = ((torch.rand((N, H, W, K), generator=g, device=device) - 0.5) * 6e-3).requires_grad_(True)
    zbuf = (5.0 + 2.0 * torch.rand((N, H, W, K), generator=g, device=device)).sort(-1).values.requires_grad_(True)
    colors = torch.rand((N, H, W, K, 3), generator=g, device=device).requires_grad_(True)
    sig, gam, alp = (torch.tensor(v, device=device, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
    gimg = torch.randn((N, H, W, 4), device=device, generator=g)
    with KernelTimer(lead_cycles=LEAD_CYCLES) as kt:
        for it in range(iters + 3):
            if it == 3:
                torch.cuda.synchronize()
                kt.reset()
            img = pa.perturbed_blend(colors, p2f, dists, zbuf, sig, gam, alp, Sr, S, background=(0, 0, 0))
            img.backward(gimg)
        torch.cuda.synchronize()
    # the kernel's own duration: the library's event pair immediately around it (pr_ktimer_arm), as
    # for the headline roofline; the call-level pair (kt.summary) also holds that inner pair and the
    # launch gaps, and read 10-15 % long (VERDICT r4 "What's weak" 4)
    kmean, kmin, calls = kt.kernel_summary("mean"), kt.kernel_summary("min"), kt.summary("min")
    shape = f"{N}x{P_side}^2, K={K}, Sr={Sr}, Sa={S}, every slot valid"
    sha = source_sha()
    headline = (N, P_side, K, S, Sr) == (1, 256, 50, 8, 8)
    prof = committed_record("rocprof_dense.json", sha) if headline else None
    pmc = committed_record("pmc_dense.json", sha) if headline else None
    out = {}
    for name, (kname, n, ms) in kmean.items():
        b = kernel_bytes(name, N * H * W, K, S, 0)
        out[name] = {"kernel": kname, "achieved": round(b / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "ms": round(ms, 4),
                     "ms_min": round(kmin[name][2], 4), "call_ms_min": round(calls[name][1], 4) if name in calls else None,
                     "bytes": b, "launches": n, "shape": shape,
                     "timing": "mean of the library's event pair around the kernel (pr_ktimer_arm)"}
        if prof and kname in prof.get("kernels", {}):
            avg_us = prof["kernels"][kname]["avg_us"]
            out[name]["rocprof"] = {"avg_us": avg_us, "frac": round(b / (avg_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                                    "source": f"profiles/rocprof_dense.json ({prof.get('run', '')}), same source_sha"}
        if pmc and pmc.get(name):
            tr = pmc[name]
            out[name]["traffic"] = tr.get("bytes_per_launch")
            if tr.get("valu_issue_us"):
                out[name]["valu_issue_us"] = tr["valu_issue_us"]
                out[name]["valu_frac"] = round(tr["valu_issue_us"] / (1e3 * ms), 4)
    return out


# ------------------------------------------------------------------ CPU baseline
def host_cpus():
    """(threads this process may use, logical CPUs of the machine, CPU model): the affinity
    set, capped by the cgroup CPU quota when one is set."""
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            avail = max(1, min(avail, int(math.ceil(int(quota) / int(period)))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return avail, os.cpu_count() or avail, model


def cpu_baseline(frames, threads):
    """CPU oracle of one step of the same workload (rasterizer in C/OpenMP, blend in torch-CPU)."""
    os.environ["OMP_NUM_THREADS"] = str(threads)  # the C oracle's OpenMP runtime reads it when loaded
    from oracle import blend_oracle as bo
    from oracle import rast_ref
    torch.set_num_threads(threads)
    wl = WorkloadCPU()
    wl.step(bo, rast_ref, 0)  # warm-up (library load, allocations): not timed
    t0 = time.perf_counter()
    for i in range(frames):
        wl.step(bo, rast_ref, i)
    dt = time.perf_counter() - t0
    return frames / dt, dt


class WorkloadCPU:
    """Same frame as Workload, on the CPU oracles (no torch device code)."""

    def __init__(self, image_size=256, K=50, samples=8, sigma=1e-3, gamma=1e-2):
        dev = torch.device("cpu")
        g = torch.Generator().manual_seed(0)
        verts, faces = load_sphere(dev)
        self.colors_v = torch.rand((verts.shape[0], 3), generator=g)
        R, T = look_at_view_transform(2.7, 30.0, 120.0)
        self.cams = FoVPerspectiveCameras(R=R, T=T, fov=60.0)
        self.verts, self.faces = verts, faces
        self.log_rot = 0.3 * torch.randn((1, 3), generator=g)
        self.target = torch.rand((1, image_size, image_size, 3), generator=g)
        self.H, self.K, self.S, self.sigma, self.gamma = image_size, K, samples, sigma, gamma
        self.blur = math.log(1.0 / 1e-4 - 1.0) * sigma

    def step(self, bo, rast_ref, i):
        H, K, S = self.H, self.K, self.S
        R = so3_exponential_map(self.log_rot)
        v = Rotate(R).transform_points(self.verts[None])
        vv = self.cams.get_world_to_view_transform().transform_points(v)
        vn = self.cams.get_projection_transform().transform_points(vv)
        vn = torch.cat([vn[..., :2], vv[..., 2:3]], -1)[0]
        fv = vn[self.faces].numpy()
        p2f, zbuf, bary, dists = rast_ref.rast_fwd(fv, [0], [fv.shape[0]], H, H, K, self.blur, False, True, False)
        attr = self.colors_v[self.faces].numpy()
        texels = torch.from_numpy(rast_ref.interp(p2f, bary, attr))
        zn, zf = torch.ones((1, 1, 1, 1)), torch.full((1, 1, 1, 1), 100.0)
        nr = torch.randn((S, 1, H, H, K))
        na = torch.randn((S, 1, H, H, K + 1))
        img, saved = bo.blend_forward(torch.from_numpy(p2f), torch.from_numpy(dists), torch.from_numpy(zbuf), texels,
                                      nr, na, torch.tensor(self.sigma), torch.tensor(self.gamma), torch.tensor(1.0),
                                      1e-10, (0.0, 0.0, 0.0), zn, zf)
        gimg = torch.zeros_like(img)
        gimg[..., :3] = 2.0 * (img[..., :3] - self.target) / self.target.numel()
        g = bo.blend_backward(gimg, saved)
        gbary = np.einsum("...kc,...kvc->...kv", g["colors"].numpy(),
                          attr[np.where(p2f >= 0, p2f, 0)]) * (p2f >= 0)[..., None]
        rast_ref.rast_bwd(fv, p2f, g["zbuf"].numpy(), gbary.astype(np.float32), g["dists"].numpy(), False, True)


# ------------------------------------------------------------------ the step
def build_step(wl, world, mode, device, grad_weight, dist_on=None):
    """Returns step() for eager or HIP-graph mode.  A step is one full pose-optimisation
    iteration of eval.py:343-376: forward, loss, backward, (N>1: the gradient all-reduce),
    Adam step on the pose (lr 5e-2, eval.py:320,337).  In graph mode forward+backward
    (incl. the Philox key advance) and the Adam step are captured HIP graphs (one graph at
    N=1); sigma/gamma/alpha live on the device so no host synchronisation remains.  dist_on (default
    world > 1): the gradient all-reduce between the captured forward/backward and Adam graphs."""
    dist_on = world > 1 if dist_on is None else dist_on
    if mode == "eager":
        # the same Adam update as eval.py:320's torch.optim.Adam, as one fused kernel (the default
        # multi-tensor path spends ~120 us of host time per step on a single (N,3) parameter)
        wl.opt = torch.optim.Adam([wl.log_rot], lr=5e-2, fused=True)

        def step():
            wl.forward().backward(wl.one)
            if dist_on:
                average_gradients(wl.params(), weight=grad_weight)
            wl.opt.step()
            wl.zero_grad()
        return step

    ds = pa.noise.DeviceSeed(device)
    pa.noise.use_device_seed(ds)
    wl.device_scalars()
    wl.seed = ds
    wl.opt = torch.optim.Adam([wl.log_rot], lr=5e-2, capturable=True, fused=True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            ds.advance()
            wl.forward().backward(wl.one)
            wl.opt.step()
            wl.zero_grad()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    # thread_local: CUDA calls of other threads (the RCCL watchdog at N>1) must not void the capture
    with torch.cuda.graph(graph, capture_error_mode="thread_local"):
        ds.advance()
        wl.forward().backward(wl.one)
        if not dist_on:
            wl.opt.step()
    wl.graph = graph
    if not dist_on:
        return graph.replay
    opt_graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(opt_graph, capture_error_mode="thread_local"):
        wl.opt.step()
    wl.opt_graph = opt_graph

    def step():
        graph.replay()
        average_gradients(wl.params(), weight=grad_weight)
        opt_graph.replay()
    return step


def split_fwd_bwd(wl, steps, world, dist_on=None):
    """Forward and backward(+Adam) as two separately captured graphs sharing one pool, replayed
    in order with events recorded between the replays: (ms_forward, ms_backward)."""
    pool = torch.cuda.graph_pool_handle()
    gf, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gf, pool=pool, capture_error_mode="thread_local"):
        wl.seed.advance()
        loss = wl.forward()
    with torch.cuda.graph(gb, pool=pool, capture_error_mode="thread_local"):
        loss.backward(wl.one, retain_graph=True)
        if not (world > 1 if dist_on is None else dist_on):
            wl.opt.step()
    for _ in range(3):
        gf.replay()
        gb.replay()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    torch.cuda.synchronize()
    for e in ev:
        e[0].record()
        gf.replay()
        e[1].record()
        gb.replay()
        e[2].record()
    torch.cuda.synchronize()
    return (float(np.mean([a.elapsed_time(b) for a, b, _ in ev])),
            float(np.mean([b.elapsed_time(c) for _, b, c in ev])))


# device-side spin before each timed launch's start event (~80 us at the 2.4 GHz shader
# clock): the host submits the launch while the GPU spins, so the event pair brackets the
# call's kernels only, not the eager pass's Python time (timing.KernelTimer)
LEAD_CYCLES = 200_000
# full-chip warm-up pass between the spin and the start event (clocks back up): 64 MB
WARM_BYTES = 64 << 20


def instrumented_pass(wl, steps):
    """Eager replica of the timed step with HIP events around every native launch (on its
    stream, each behind a device-side lead spin): per-call kernel durations.  (ROCm cannot
    record events inside a captured graph.)"""
    seed = getattr(wl, "seed", None)
    grads = [p.grad for p in wl.params()]
    torch.cuda.synchronize()
    with KernelTimer(lead_cycles=LEAD_CYCLES, warm_bytes=WARM_BYTES) as kt:
        for _ in range(steps):
            if seed is not None:
                seed.advance()
            wl.forward().backward(wl.one)
            for p in wl.params():
                p.grad = None
        torch.cuda.synchronize()
    for p, g in zip(wl.params(), grads):
        p.grad = g
    return kt.summary("min"), kt.summary("median"), kt.kernel_summary("mean"), kt.kernel_summary("min")


def committed_record(name, sha):
    """profiles/<name> when it was measured on these native sources (its "source_sha"), else None."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    rec = json.load(open(path))
    return rec if rec.get("source_sha") == sha else None


def eager_split(wl, steps):
    """ms forward / ms backward of the eager step (events around forward and loss.backward())."""
    fb = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for i in range(steps):
        fb[i][0].record()
        loss = wl.forward()
        fb[i][1].record()
        loss.backward(wl.one)
        fb[i][2].record()
        wl.zero_grad()
    torch.cuda.synchronize()
    return (float(np.mean([a.elapsed_time(b) for a, b, _ in fb])),
            float(np.mean([b.elapsed_time(c) for _, b, c in fb])))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--mode", choices=["graph", "eager"], default="graph")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="cfg2",
                    help="BASELINE.json configuration (cfg2 = the metric's headline workload)")
    ap.add_argument("--shard", choices=["frames", "samples"], default="samples",
                    help="N > 1: the Monte-Carlo samples (strong, default) or distinct views per rank (weak)")
    ap.add_argument("--image-size", type=int, default=None)
    ap.add_argument("--faces-per-pixel", type=int, default=None)
    ap.add_argument("--samples", type=int, default=None, help="Monte-Carlo samples (global in --shard samples)")
    ap.add_argument("--batch", type=int, default=None, help="meshes per rank")
    ap.add_argument("--loss", choices=["native", "torch"], default="native",
                    help="the step's L2 loss: the package's fused kernels (default) or torch ops")
    ap.add_argument("--cpu-frames", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dense", action="store_true")
    ap.add_argument("--launch-check", action="store_true",
                    help="no GPU work: join a gloo group, count the ranks by an all-reduce, print them (tests)")
    args = ap.parse_args()
    if args.launch_check:
        dist.init_process_group("gloo")
        seen = torch.ones(1)
        dist.all_reduce(seen)
        if dist.get_rank() == 0:
            print(json.dumps({"n_gpus": args.gpus, "world_size": dist.get_world_size(), "ranks_seen": int(seen.item()),
                              "master": f"{os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}"}), flush=True)
        dist.destroy_process_group()
        return
    cfg = dict(CONFIGS[args.config])
    for key, val in (("image_size", args.image_size), ("K", args.faces_per_pixel), ("samples", args.samples),
                     ("batch", args.batch)):
        if val is not None:
            cfg[key] = val
    headline = args.config == "cfg2" and cfg == CONFIGS["cfg2"]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # PR_BENCH_BACKEND=gloo rehearses the N>1 path with several ranks on fewer GPUs
    # (rank -> GPU local % device_count); the measured configuration is nccl (RCCL)
    backend = os.environ.get("PR_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    # PR_BENCH_DIST=1: the process group, the gradient all-reduce and the max-over-ranks timing at
    # N = 1 too (one RCCL rank: the N > 1 code path on a one-GPU box, tests/test_gpu_rccl.py)
    dist_on = world > 1 or os.environ.get("PR_BENCH_DIST", "0") == "1"
    if dist_on:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    ranks = dist.get_world_size() if dist_on else 1  # the ranks the process group (RCCL) saw
    if ranks != world:
        raise RuntimeError(f"process group has {ranks} ranks, WORLD_SIZE={world}")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    torch.manual_seed(1234)  # same Philox keys on every rank
    pa.native_library()

    S, Sr = cfg["samples"], cfg.get("rast_samples", cfg["samples"])
    shard = args.shard if world > 1 else "frames"
    grad_weight = None
    azim = 120.0
    if shard == "samples":
        off_a, n_a = sample_shard(S, rank, world)
        off_r, n_r = sample_shard(Sr, rank, world)
        pa.noise.set_sample_offset(off_r, off_a)
        grad_weight = n_a / S
        S_local, Sr_local = n_a, n_r
    else:
        azim = 120.0 + 360.0 * rank / world
        S_local, Sr_local = S, Sr

    mk_wl = lambda: Workload(device, cfg["image_size"], cfg["K"], S_local, seed=0, batch=cfg["batch"], azim=azim,
                             rast_samples=Sr_local, eval_scene=args.config == "eval", loss=args.loss)
    wl = mk_wl()
    P = cfg["batch"] * cfg["image_size"] * cfg["image_size"]
    mode, note = args.mode, None
    try:
        step = build_step(wl, world, mode, device, grad_weight, dist_on)
    except Exception as e:  # graph capture unavailable: measure eagerly and say so
        note = f"graph capture failed ({type(e).__name__}: {e}); eager fallback"
        pa.noise.use_device_seed(None)
        wl = mk_wl()
        mode = "eager"
        step = build_step(wl, world, mode, device, grad_weight, dist_on)

    for _ in range(args.warmup):
        step()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    n_split = min(args.steps, 20)
    if mode == "graph":
        ms_fwd, ms_bwd = split_fwd_bwd(wl, n_split, world, dist_on)
        split_from = ("HIP events around separately captured forward and backward(+Adam) graphs, replayed "
                      "after the timed region")
    else:
        ms_fwd, ms_bwd = eager_split(wl, n_split)
        split_from = "HIP events around the eager forward / loss.backward()"
    ksum, kmed, kk, kkmin = instrumented_pass(wl, n_split)
    kern = {}
    for name, (n, ms) in ksum.items():
        bts = kernel_bytes(name, P, wl.K, S_local, wl.F)
        kern[name] = {"launches": n, "ms": round(ms, 4), "ms_median": round(kmed[name][1], 4), "bytes": bts,
                      "GBps": round(bts / (ms * 1e-3) / 1e9, 1)}
        if name in kk:  # the call's dominant kernel alone (the library's own event pair around it)
            kname, _, kms = kk[name]
            kern[name].update({"kernel": kname, "kernel_ms": round(kms, 4), "kernel_ms_min": round(kkmin[name][2], 4)})
    sha = source_sha()
    prof = committed_record("rocprof_kernels.json", sha) if headline else None
    pmc = committed_record("pmc_traffic.json", sha) if headline else None
    # every call's algorithmic fraction (live kernel events), beside it the committed rocprofv3 average
    # and the PMC-traffic fraction when those records were measured on these native sources
    for name, e in kern.items():
        k_ms_e = e.get("kernel_ms", e["ms"])
        e["frac"] = round(e["bytes"] / (k_ms_e * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        t_ms = k_ms_e
        if prof and e.get("kernel") in prof.get("kernels", {}):
            t_ms = prof["kernels"][e["kernel"]]["avg_us"] * 1e-3
            e["rocprof_ms"] = round(t_ms, 4)
            e["frac_rocprof"] = round(e["bytes"] / (t_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        if pmc and pmc.get(name, {}).get("bytes_per_launch"):
            e["traffic"] = pmc[name]["bytes_per_launch"]
            e["frac_traffic"] = round(e["traffic"] / (t_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    # roofline: the longest kernel as rocprofv3 names it -- by the committed rocprofv3 average when it
    # was measured on these sources (box noise flips the live order of near-equal kernels), else by
    # its live per-launch duration
    timed = [k for k in kern if "kernel_ms" in kern[k]] or list(kern)
    if prof and all("rocprof_ms" in kern[k] for k in timed):
        dom = max(timed, key=lambda k: kern[k]["rocprof_ms"] * kern[k]["launches"])
        dom_from = "longest committed rocprofv3 average (profiles/rocprof_kernels.json, same source_sha)"
    else:
        dom = max(timed, key=lambda k: kern[k].get("kernel_ms", kern[k]["ms"]) * kern[k]["launches"])
        dom_from = "longest live kernel event time (no rocprofv3 record for these sources)"
    d = kern[dom]
    k_ms = d.get("kernel_ms", d["ms"])
    achieved = d["bytes"] / (k_ms * 1e-3) / 1e9
    roof = {"kernel": d.get("kernel", dom), "call": dom, "bound": "hbm", "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "bytes_per_launch": d["bytes"], "ms_per_launch": round(k_ms, 4), "source_sha": sha,
            "timing": "mean over the launches of an eager replica of the timed step (same kernels and arguments, "
                      "right after the timed region) of a HIP event pair the library records on the launch stream "
                      "immediately around this kernel (pr_ktimer_arm); each launch behind a device-side lead spin "
                      "(host time excluded) and a 64 MB elementwise pass (clocks up)",
            "bytes_from": "algorithmic bytes of the call (SURVEY.md §8(d), bench.kernel_bytes), all attributed to "
                          "its dominant kernel",
            "dominant_from": dom_from}
    if prof and roof["kernel"] in prof.get("kernels", {}):
        avg_us = prof["kernels"][roof["kernel"]]["avg_us"]
        roof["rocprof"] = {"avg_us": avg_us, "achieved": round(d["bytes"] / (avg_us * 1e-6) / 1e9, 1),
                           "frac": round(d["bytes"] / (avg_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                           "source": f"profiles/rocprof_kernels.json ({prof.get('run', '')}), measured on these "
                                     f"native sources (source_sha {sha})"}
    if pmc and pmc.get(dom):  # PMC passes are taken on the headline workload
        # rocprofv3 cannot collect counters inside this process's timed run (the counter passes need
        # their own runs, tools/gpu.sh pmc), so the line carries the committed measurement of the
        # same workload and the same native sources (source_sha), labelled with its source
        tr = pmc[dom]
        roof["traffic"] = tr.get("bytes_per_launch")
        if roof["traffic"]:  # the bytes the kernel really moved, over the same duration
            t_us = roof.get("rocprof", {}).get("avg_us", 1e3 * k_ms)
            roof["frac_traffic"] = round(roof["traffic"] / (t_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
            roof["frac_traffic_time"] = "rocprofv3 average" if "rocprof" in roof else "live kernel events"
        roof["traffic_source"] = ("profiles/pmc_traffic.json: (2 FETCH_SIZE + WRITE_SIZE) KiB of this call's "
                                  f"kernels {tr.get('kernels')}, separate rocprofv3 --pmc passes of tools/kprof.py on "
                                  f"this workload, same source_sha ({pmc.get('_run', 'see profiles/')})")
        if tr.get("valu_issue_us"):  # the bound that applies: VALU issue
            roof["valu_issue_us"] = tr["valu_issue_us"]
            roof["valu_frac"] = round(tr["valu_issue_us"] / (1e3 * k_ms), 4)

    B, Hs, K = cfg["batch"], cfg["image_size"], cfg["K"]
    distinct = B * (world if shard == "frames" else 1)  # distinct frames per step
    value = args.steps * distinct / elapsed
    if args.config == "eval":
        meshes = "textured cube (TexturesUV) + RandomPhongShader, eval.py's renderer"
    elif B == 1:
        meshes = "sphere_642 (1280 faces)"
    else:
        meshes = f"{B} meshes alternating sphere_642 / cube2 ({wl.F} faces), one pose each"
    samples_txt = f"Sr={Sr} Sa={S}" if Sr != S else f"Sr=Sa={S}"
    if world == 1:
        par = "single GPU" + (f" (process group: one {backend} rank, gradient all-reduce between the forward/"
                              "backward and Adam graphs)" if dist_on else "")
    elif shard == "frames":
        par = (f"frame-parallel x{world}: each rank renders its own view (azimuth 120 + 360 r / {world}) of the "
               "shared pose; one RCCL all-reduce averages the gradients")
    else:
        par = (f"sample-parallel x{world}: the same frame on every rank, {S} global samples split "
               f"{[sample_shard(S, r, world)[1] for r in range(world)]}, shared Philox keys + global sample "
               "offsets; one RCCL all-reduce forms the full-S gradient estimate")
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "frames/s (fwd+bwd)", "n_gpus": world,
        "ranks": ranks, "backend": backend if dist_on else None,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True, "scaling": "strong" if shard == "samples" else "weak", "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (meshes from the reference data, random vertex colours, random target)",
        "config": {"workload": f"{args.config} pose-opt step: {meshes}, {Hs}x{Hs}, faces_per_pixel={K}, "
                               f"{samples_txt} Gaussian, sigma=1e-3 gamma=1e-2, blur=ln(1e4-1)*sigma, "
                               f"fwd + L2 loss ({args.loss}) + bwd + Adam step on the pose (lr 5e-2)",
                   "image_size": Hs, "faces_per_pixel": K, "nb_samples": S, "rast_samples": Sr, "batch": B,
                   "distinct_frames_per_step": distinct, "execution": mode, "parallelism": par,
                   "loss": ("eval.py:352-353's ((images[..., :3] - target) ** 2).mean() on the fused native "
                            "kernels pr_rgb_mse_fwd/_bwd" if args.loss == "native" else "torch ops"),
                   # where the eager autograd nodes run (host_layer.py): "c++" torch::autograd
                   # Functions over the C ABI, or the Python Functions
                   "host_layer": pa.host_layer.layer(),
                   # eval.py:4 sets CUDA_LAUNCH_BLOCKING=1; the HIP runtime honours HIP_LAUNCH_BLOCKING only
                   # (tools/launch_blocking_check.py), so eval.py itself runs launches asynchronously here
                   "launch_blocking": {k: os.environ[k] for k in ("HIP_LAUNCH_BLOCKING", "CUDA_LAUNCH_BLOCKING")
                                       if k in os.environ}},
        "ms_forward": round(ms_fwd, 4), "ms_backward": round(ms_bwd, 4), "fwd_bwd_split_from": split_from,
        "fwd_frames_per_s": round(distinct * 1e3 / ms_fwd, 2), "kernels": kern, "roofline": roof,
    }
    # SURVEY §8(d) RNG term: the algorithmic Gaussian draws of the step (the forward's Sr*K rast
    # and Sa*(K+1) agg normals per pixel, regenerated once more by the backward) against the
    # generator's measured peak (tools/philox_bench.hip: Philox4x32-7 + Box-Muller, every lane busy).
    # The kernels skip saturated rast slots, sure-loser logits and padded slots, so the achieved
    # rate can exceed the peak: that is work never done, not a faster generator.
    normals = 2 * B * Hs * Hs * (Sr_local * K + S_local * (K + 1)) * world
    out["rng"] = {"normals_per_step": normals, "normals_per_s": round(normals * args.steps / elapsed, 1),
                  "peak_normals_per_s": RNG_PEAK_NORMALS_PER_S * world,
                  "frac": round(normals * args.steps / elapsed / (RNG_PEAK_NORMALS_PER_S * world), 4),
                  "peak_from": "tools/philox_bench.hip on one MI355X: 690 G Philox4x32-7 blocks/s (the streams' rounds) "
                               "x 4 normals"}
    if shard == "samples":
        # strong scaling: the rasterizer (and the tiny pose kernels) run in full on every rank, the
        # blend on this rank's sample shard; T(N) >= T_rep + T_shard(1) / N bounds the speed-up
        rep_ms = sum(kern[k].get("kernel_ms", kern[k]["ms"]) for k in ("rast_fwd", "rast_bwd") if k in kern)
        sh_ms = sum(kern[k].get("kernel_ms", kern[k]["ms"]) for k in ("blend_fwd", "blend_bwd") if k in kern)
        out["strong_scaling"] = {
            "replicated_ms_per_rank": round(rep_ms, 4), "sharded_ms_per_rank": round(sh_ms, 4),
            "speedup_bound_vs_1gpu": round((rep_ms + sh_ms * world) / rep_ms, 2) if rep_ms > 0 else None,
            "from": "this rank's kernel events (rast_fwd + rast_bwd replicated; blend_fwd + blend_bwd over "
                    f"{S_local} of {S} agg samples)"}
    if note:
        out["note"] = note
    if rank == 0 and world == 1 and not args.no_dense and args.config != "eval":
        # the blend kernels' fraction of HBM peak on dense fragments at this configuration's shape
        out["roofline_dense"] = dense_roofline(device, Hs, K, S, N=B, Sr=Sr)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and headline:
        threads, total, model = host_cpus()
        v, dt = cpu_baseline(args.cpu_frames, threads)
        out["cpu_baseline"] = {"value": round(v, 4), "unit": "frames/s (fwd+bwd)", "cores": threads,
                               "kind": "port", "cpu_model": model, "machine_logical_cpus": total,
                               "sample": f"{args.cpu_frames} frames of the same workload ({dt:.1f} s) on all "
                                         f"{threads} CPUs this process may use (affinity / cgroup quota): "
                                         "C/OpenMP rasterizer oracle + torch-CPU blend oracle fwd+bwd + "
                                         "rasterizer bwd"}
        out["speedup_vs_cpu"] = round(value / v, 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
