"""Benchmark of the perturbed-renderer hot path (BASELINE.json configs[1]).

One step = one pose-optimisation iteration of experiments/eval.py:343-376: rotate
the mesh (so3 exp map), MeshRasterizer (native K-nearest rasterizer, 256x256,
faces_per_pixel=50, blur = ln(1/1e-4 - 1)*sigma), RandomSimpleShader with
GaussianRast(nb_samples=8) + GaussianAgg(nb_samples=8) (fused native blend with
TexturesVertex sampling), L2 loss to a fixed synthetic target, backward through
blend -> rasterizer -> vertices -> pose, Adam step on the pose (lr 5e-2, eval.py:337).
With N ranks the Monte-Carlo sample
dimension is sharded (BASELINE north star): every rank renders the SAME frame and
pose with its own disjoint range of global sample indices (Philox offset rank*S),
and one RCCL all-reduce averages the gradient estimates, i.e. each step is one
pose update from an (N*8)-sample estimator.  Per-GPU work is fixed (one 8-sample
render per rank per step): weak scaling; `value` counts renders over all ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Prints ONE JSON line on rank 0.  `value` = frames/s over all ranks (forward +
backward per frame); `roofline` is the dominant native kernel's algorithmic HBM
bytes / its mean HIP-event duration inside the timed region; `cpu_baseline` times
the CPU oracle (test-infrastructure restatement of the reference + PyTorch3D
rasterizer) on a bounded sample of the same workload, on rank 0 at N=1.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import pertrenderer_amd as pa  # noqa: E402
from pertrenderer_amd.renderer import (FoVPerspectiveCameras, MeshRasterizer, MeshRenderer, Meshes,  # noqa: E402
                                       RasterizationSettings, TexturesVertex, load_obj, look_at_view_transform)
from pertrenderer_amd.renderer.transforms import Rotate, so3_exponential_map  # noqa: E402
from pertrenderer_amd.parallel import average_gradients  # noqa: E402
from pertrenderer_amd.timing import KernelTimer  # noqa: E402

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
# configurations (16 meshes alternating sphere_642 / cube2, each with its own pose)
CONFIGS = {
    "cfg2": dict(batch=1, image_size=256, K=50, samples=8),
    "cfg3": dict(batch=16, image_size=256, K=100, samples=16),
    "cfg4": dict(batch=16, image_size=512, K=150, samples=64),
}


class Workload:
    def __init__(self, device, image_size=256, K=50, samples=8, sigma=1e-3, gamma=1e-2, dist_cam=2.7, seed=0,
                 batch=1):
        self.device = device
        g = torch.Generator().manual_seed(seed)
        vl, fl, cl = [], [], []
        for i in range(batch):
            verts, faces = load_mesh(device, "sphere_642.obj" if i % 2 == 0 else "cube2.obj")
            vl.append(verts)
            fl.append(faces)
            cl.append(torch.rand((verts.shape[0], 3), generator=g).to(device))
        self.base = Meshes(vl, fl, TexturesVertex(cl))
        faces = torch.cat(fl)
        R, T = look_at_view_transform(dist_cam, 30.0, 120.0, device=device)
        self.cameras = FoVPerspectiveCameras(R=R, T=T, device=device, fov=60.0)
        self.settings = RasterizationSettings(image_size=image_size,
                                              blur_radius=math.log(1.0 / 1e-4 - 1.0) * sigma,
                                              faces_per_pixel=K, max_faces_per_bin=50000,
                                              perspective_correct=False)
        self.rast = pa.GaussianRast(nb_samples=samples, sigma=sigma)
        self.agg = pa.GaussianAgg(nb_samples=samples, gamma=gamma, alpha=1.0)
        self.renderer = MeshRenderer(
            rasterizer=MeshRasterizer(cameras=self.cameras, raster_settings=self.settings),
            shader=pa.RandomSimpleShader(device=device, cameras=self.cameras, smoothrast=self.rast,
                                         smoothagg=self.agg,
                                         blend_params=pa.random_rasterizer.BlendParams(sigma, gamma, (0.0, 0.0, 0.0))))
        self.log_rot = (0.3 * torch.randn((batch, 3), generator=g)).to(device).requires_grad_(True)
        self.target = torch.rand((batch, image_size, image_size, 3), generator=g).to(device)
        self.K, self.S, self.H, self.batch = K, samples, image_size, batch
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
        images = self.renderer(mesh, cameras=self.cameras)
        return ((images[..., :3] - self.target) ** 2).mean()

    def zero_grad(self):
        for p in self.params():
            p.grad = None


def allreduce_grads(params, world):
    """The single gradient reduction of the data-parallel step: one flattened RCCL
    all-reduce of every gradient, averaged over ranks (pertrenderer_amd.parallel)."""
    average_gradients(params)


def kernel_bytes(name, P, K, S, F):
    """Algorithmic HBM bytes per launch (int64 pix_to_face)."""
    slots = P * K
    return {
        "blend_fwd": slots * (8 + 4 + 4 + 12) + P * 16 + P * S,           # p2f,dists,zbuf,colors | image, winners
        "blend_bwd": slots * (8 + 4 + 4 + 12 + 4 + 4 + 12) + P * 16 + P * S,  # + d dists,d zbuf,d colors | d image
        "rast_fwd": slots * (8 + 4 + 12 + 4) + F * 36,                   # p2f,zbuf,bary,dists | face verts
        "rast_bwd": slots * (8 + 4 + 12 + 4) + F * 36 * 2,               # p2f + 3 upstream grads | verts, grads
    }.get(name)


def dense_roofline(device, P_side=256, K=50, S=8, iters=20):
    """Blend kernels on dense synthetic fragments (every slot valid) — the bandwidth microbench."""
    g = torch.Generator().manual_seed(0)
    N, H, W = 1, P_side, P_side
    p2f = torch.randint(0, 5000, (N, H, W, K), generator=g).to(device)
    dists = ((torch.rand((N, H, W, K), generator=g) - 0.5) * 6e-3).to(device).requires_grad_(True)
    zbuf = (5.0 + 2.0 * torch.rand((N, H, W, K), generator=g)).sort(-1).values.to(device).requires_grad_(True)
    colors = torch.rand((N, H, W, K, 3), generator=g).to(device).requires_grad_(True)
    sig, gam, alp = (torch.tensor(v, device=device, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
    gimg = torch.randn((N, H, W, 4), device=device)
    with KernelTimer(lead_cycles=LEAD_CYCLES) as kt:
        for it in range(iters + 3):
            if it == 3:
                torch.cuda.synchronize()
                kt.reset()
            img = pa.perturbed_blend(colors, p2f, dists, zbuf, sig, gam, alp, S, S, background=(0, 0, 0))
            img.backward(gimg)
        torch.cuda.synchronize()
    out = {}
    for name, (n, ms) in kt.summary().items():
        b = kernel_bytes(name, N * H * W, K, S, 0)
        out[name] = {"achieved": round(b / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "ms": round(ms, 4),
                     "bytes": b, "launches": n}
    return out


def cpu_baseline(frames, threads):
    """CPU oracle of one step of the same workload (rasterizer in C/OpenMP, blend in torch-CPU)."""
    from oracle import blend_oracle as bo
    from oracle import rast_ref
    torch.set_num_threads(threads)
    dev = torch.device("cpu")
    wl = WorkloadCPU()
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


def build_step(wl, world, mode, device):
    """Returns step() for eager or HIP-graph mode.  A step is one full pose-optimisation
    iteration of eval.py:343-376: forward, loss, backward, (N>1: the gradient all-reduce),
    Adam step on the pose (lr 5e-2, eval.py:320,337).  In graph mode forward+backward
    (incl. the Philox key advance) and the Adam step are captured HIP graphs (one graph at
    N=1); sigma/gamma/alpha live on the device so no host synchronisation remains."""
    if mode == "eager":
        wl.opt = torch.optim.Adam([wl.log_rot], lr=5e-2)

        def step():
            wl.forward().backward()
            if world > 1:
                allreduce_grads(wl.params(), world)
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
            wl.forward().backward()
            wl.opt.step()
            wl.zero_grad()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    # thread_local: CUDA calls of other threads (the RCCL watchdog at N>1) must not void the capture
    with torch.cuda.graph(graph, capture_error_mode="thread_local"):
        ds.advance()
        wl.forward().backward()
        if world == 1:
            wl.opt.step()
    wl.graph = graph
    if world == 1:
        return graph.replay
    opt_graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(opt_graph, capture_error_mode="thread_local"):
        wl.opt.step()
    wl.opt_graph = opt_graph

    def step():
        graph.replay()
        allreduce_grads(wl.params(), world)
        opt_graph.replay()
    return step


# device-side spin before each timed launch's start event (~80 us at the 2.4 GHz shader
# clock): the host submits the launch while the GPU spins, so the event pair brackets the
# call's kernels only, not the eager pass's Python time (timing.KernelTimer)
LEAD_CYCLES = 200_000


def instrumented_pass(wl, steps):
    """Eager replica of the timed step.  (1) HIP events around every native launch (on its
    stream, each behind a device-side lead spin): per-call kernel durations.  (2) Without
    the spins, events around forward / backward: the fwd/bwd split.  (ROCm cannot record
    events inside a captured graph.)"""
    seed = getattr(wl, "seed", None)
    grads = [p.grad for p in wl.params()]

    def one():
        if seed is not None:
            seed.advance()
        loss = wl.forward()
        loss.backward()
        for p in wl.params():
            p.grad = None

    torch.cuda.synchronize()
    with KernelTimer(lead_cycles=LEAD_CYCLES) as kt:
        for _ in range(steps):
            one()
        torch.cuda.synchronize()
    fb = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for i in range(steps):
        if seed is not None:
            seed.advance()
        fb[i][0].record()
        loss = wl.forward()
        fb[i][1].record()
        loss.backward()
        fb[i][2].record()
        for p in wl.params():
            p.grad = None
    torch.cuda.synchronize()
    for p, g in zip(wl.params(), grads):
        p.grad = g
    ms_fwd = float(np.mean([a.elapsed_time(b) for a, b, _ in fb]))
    ms_bwd = float(np.mean([b.elapsed_time(c) for _, b, c in fb]))
    return kt.summary("median"), ms_fwd, ms_bwd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--mode", choices=["graph", "eager"], default="graph")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="cfg2",
                    help="BASELINE.json configuration (cfg2 = the metric's headline workload)")
    ap.add_argument("--image-size", type=int, default=None)
    ap.add_argument("--faces-per-pixel", type=int, default=None)
    ap.add_argument("--samples", type=int, default=None, help="Monte-Carlo samples per rank")
    ap.add_argument("--batch", type=int, default=None, help="meshes per rank")
    ap.add_argument("--cpu-frames", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dense", action="store_true")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    for key, val in (("image_size", args.image_size), ("K", args.faces_per_pixel), ("samples", args.samples),
                     ("batch", args.batch)):
        if val is not None:
            cfg[key] = val
    headline = cfg == CONFIGS["cfg2"]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # PR_BENCH_BACKEND=gloo rehearses the N>1 path with several ranks on fewer GPUs
    # (rank -> GPU local % device_count); the measured configuration is nccl (RCCL)
    backend = os.environ.get("PR_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    torch.manual_seed(1234)  # same Philox keys on every rank ...
    pa.noise.set_sample_shard(rank)  # ... disjoint global sample ranges
    pa.native_library()

    mk_wl = lambda: Workload(device, cfg["image_size"], cfg["K"], cfg["samples"], seed=0,  # same frame on all ranks
                             batch=cfg["batch"])
    wl = mk_wl()
    P = cfg["batch"] * cfg["image_size"] * cfg["image_size"]
    mode, note = args.mode, None
    try:
        step = build_step(wl, world, mode, device)
    except Exception as e:  # graph capture unavailable: measure eagerly and say so
        note = f"graph capture failed ({type(e).__name__}: {e}); eager fallback"
        pa.noise.use_device_seed(None)
        wl = mk_wl()
        mode = "eager"
        step = build_step(wl, world, mode, device)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ksum, ms_fwd, ms_bwd = instrumented_pass(wl, min(args.steps, 20))
    kern = {}
    for name, (n, ms) in ksum.items():
        bts = kernel_bytes(name, P, wl.K, wl.S, wl.F)
        kern[name] = {"launches": n, "ms": round(ms, 4), "bytes": bts,
                      "GBps": round(bts / (ms * 1e-3) / 1e9, 1)}
    dom = max(kern, key=lambda k: kern[k]["ms"] * kern[k]["launches"])
    d = kern[dom]
    roof = {"kernel": dom, "bound": "hbm", "achieved": d["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(d["GBps"] / HBM_PEAK_GBS, 4), "traffic": None,
            "bytes_per_launch": d["bytes"], "ms_per_launch": d["ms"],
            "timing": "median of HIP events around each launch on its stream (each behind a device-side "
                      "lead spin, so host time is excluded), eager replica of the timed step right after "
                      "the timed region (same kernels and arguments)"}
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if headline and os.path.exists(pmc):  # PMC passes are taken on the headline workload
        tr = json.load(open(pmc)).get(dom)
        if tr:
            roof["traffic"] = tr.get("bytes_per_launch")
            if tr.get("valu_issue_us"):  # the bound that applies: VALU issue
                roof["valu_issue_us"] = tr["valu_issue_us"]
                roof["valu_frac"] = round(tr["valu_issue_us"] / (1e3 * d["ms"]), 4)

    B, Hs, K, S = cfg["batch"], cfg["image_size"], cfg["K"], cfg["samples"]
    frames = args.steps * world * B
    value = frames / elapsed
    meshes = ("sphere_642 (1280 faces)" if B == 1 else
              f"{B} meshes alternating sphere_642 / cube2 ({wl.F} faces), one pose each")
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "frames/s (fwd+bwd)", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (meshes from the reference data, random vertex colours, random target)",
        "config": {"workload": f"{args.config} pose-opt step: {meshes}, {Hs}x{Hs}, faces_per_pixel={K}, "
                               f"Sr=Sa={S} Gaussian, sigma=1e-3 gamma=1e-2, blur=ln(1e4-1)*sigma, "
                               "fwd + L2 loss + bwd + Adam step on the pose (lr 5e-2)",
                   "image_size": Hs, "faces_per_pixel": K, "nb_samples": S, "batch": B,
                   "frames_per_rank_per_step": B, "execution": mode,
                   "parallelism": f"sample-parallel x{world} (same frames, Philox sample shard per rank, "
                                  f"one RCCL gradient all-reduce per step)"},
        "ms_forward": round(ms_fwd, 4), "ms_backward": round(ms_bwd, 4),
        "fwd_bwd_split_from": "eager instrumented replica (HIP events around forward / loss.backward())",
        "fwd_frames_per_s": round(world * B * 1e3 / ms_fwd, 2), "kernels": kern, "roofline": roof,
    }
    if note:
        out["note"] = note
    if rank == 0 and not args.no_dense and headline:
        out["roofline_dense"] = dense_roofline(device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and headline:
        threads = int(os.environ.get("OMP_NUM_THREADS", str(min(16, os.cpu_count() or 1))))
        os.environ.setdefault("OMP_NUM_THREADS", str(threads))
        v, dt = cpu_baseline(args.cpu_frames, threads)
        out["cpu_baseline"] = {"value": round(v, 4), "unit": "frames/s (fwd+bwd)", "cores": threads,
                               "kind": "port",
                               "sample": f"{args.cpu_frames} frames of the same workload ({dt:.1f} s): C/OpenMP "
                                         "rasterizer oracle + torch-CPU blend oracle fwd+bwd + rasterizer bwd"}
        out["speedup_vs_cpu"] = round(value / v, 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
