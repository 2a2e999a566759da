"""Host time of the eager bench step's forward, stage by stage (no synchronisation inside the
timed loop), plus a cProfile of the forward's Python.  Diagnostic for the eager row.

    python tools/eager_host_breakdown.py [iterations]
"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import pertrenderer_amd as pa  # noqa: E402
from pertrenderer_amd.renderer import Rotate, so3_exponential_map  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda:0")
    wl = bench.Workload(dev)
    r = wl.renderer
    acc = {}

    def stage(name, t0):
        t = time.perf_counter()
        acc[name] = acc.get(name, 0.0) + (t - t0)
        return t

    def fwd(timed):
        t = time.perf_counter()
        R = so3_exponential_map(wl.log_rot)
        t = stage("so3", t) if timed else t
        vp = wl.base.verts_padded()
        v = Rotate(R).transform_points(vp)
        t = stage("rotate", t) if timed else t
        mesh = wl.base.update_padded(v)
        t = stage("update_padded", t) if timed else t
        img = r(mesh, cameras=wl.cameras)
        t = stage("renderer", t) if timed else t
        loss = ((img[..., :3] - wl.target) ** 2).mean()
        t = stage("loss", t) if timed else t
        return loss

    for _ in range(30):
        fwd(False).backward()
    torch.cuda.synchronize()
    for _ in range(n):
        fwd(True).backward()
        wl.zero_grad()
    torch.cuda.synchronize()
    print("forward host us/step:", {k: round(1e6 * v / n, 1) for k, v in acc.items()},
          "total", round(1e6 * sum(acc.values()) / n, 1), flush=True)
    # the renderer's parts
    acc.clear()
    mesh = wl.base.update_padded(Rotate(so3_exponential_map(wl.log_rot)).transform_points(wl.base.verts_padded()))
    for _ in range(n):
        t = time.perf_counter()
        frag = r.rasterizer(mesh, cameras=wl.cameras)
        t = stage("rasterizer", t)
        img = r.shader(frag, mesh, cameras=wl.cameras)
        t = stage("shader", t)
        del img, frag
    torch.cuda.synchronize()
    print("renderer parts us/call:", {k: round(1e6 * v / n, 1) for k, v in acc.items()}, flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        fwd(False).backward()
        wl.zero_grad()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
