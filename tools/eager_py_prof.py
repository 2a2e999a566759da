"""Python-level profile of the eager bench step with the autograd engine's device threads off
(torch.autograd.set_multithreading_enabled(False): backward nodes run on this thread, so cProfile
sees them): own time per function, ours and torch's.

    python tools/eager_py_prof.py [steps]
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
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    dev = torch.device("cuda:0")
    pa.native_library()
    wl = bench.Workload(dev)
    step = bench.build_step(wl, 1, "eager", dev, None)
    with torch.autograd.set_multithreading_enabled(False):
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        print(f"eager (single-threaded autograd): {(time.perf_counter() - t0) / steps * 1e3:.3f} ms/step")
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(40)


if __name__ == "__main__":
    main()
