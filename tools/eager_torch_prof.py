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
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=45))


if __name__ == "__main__":
    main()
