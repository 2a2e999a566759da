"""Host-side profile of the eager bench step (eval.py's execution mode): cProfile over N
steps, top functions by own time and by cumulative time.

    python tools/eager_host_prof.py [steps]
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


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda:0")
    pa.native_library()
    wl = bench.Workload(dev)
    step = bench.build_step(wl, 1, "eager", dev, None)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    print(f"eager: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(40)
    st.sort_stats("cumulative").print_stats("pertrenderer_amd|bench", 60)
    # host time per stage with the GPU drained before each stage (no waiting inside a stage)
    import collections
    acc = collections.defaultdict(float)
    from pertrenderer_amd.renderer.transforms import Rotate, so3_exponential_map
    for _ in range(steps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        R = so3_exponential_map(wl.log_rot)
        mesh = wl.base.update_padded(Rotate(R).transform_points(wl.base.verts_padded()))
        t1 = time.perf_counter(); acc["pose"] += t1 - t
        frag = wl.renderer.rasterizer(mesh, cameras=wl.cameras)
        t2 = time.perf_counter(); acc["rasterizer"] += t2 - t1
        img = wl.renderer.shader(frag, mesh, cameras=wl.cameras)
        t3 = time.perf_counter(); acc["shader"] += t3 - t2
        loss = ((img[..., :3] - wl.target) ** 2).mean()
        t4 = time.perf_counter(); acc["loss"] += t4 - t3
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        loss.backward()
        t5 = time.perf_counter(); acc["backward (incl. its waits)"] += t5 - t4
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        wl.opt.step()
        wl.zero_grad()
        t6 = time.perf_counter(); acc["adam + zero_grad"] += t6 - t5
    for k, v in acc.items():
        print(f"{k:30s} {v / steps * 1e6:8.1f} us host")


if __name__ == "__main__":
    main()
