"""torch.profiler view of the eager bench step (eval.py's execution mode): host time per op and
autograd node, CPU side only.

    python tools/eager_torch_prof.py [steps]
"""
import os
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
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        print(f"eager: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms/step", flush=True)
    # host time per phase (no synchronisation inside a step: the backward's includes the wait of
    # the smoothing scalars' gradient copy for the blend kernels)
    ph = [0.0, 0.0, 0.0]
    for _ in range(steps):
        t0 = time.perf_counter()
        loss = wl.forward()
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        wl.opt.step()
        wl.zero_grad()
        t3 = time.perf_counter()
        ph[0] += t1 - t0
        ph[1] += t2 - t1
        ph[2] += t3 - t2
    torch.cuda.synchronize()
    print("host ms/step: forward %.3f  backward %.3f  adam+zero %.3f" % tuple(1e3 * v / steps for v in ph), flush=True)
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=45))


if __name__ == "__main__":
    main()
