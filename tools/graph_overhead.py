"""Where the graph step's time goes besides the four native kernels:
* host enqueue rate of the bench step's graph replay (no sync) vs its GPU rate;
* per-node cost of a graph of trivial dependent kernels (1-element adds).

    python tools/graph_overhead.py
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import pertrenderer_amd as pa  # noqa: E402


def rate(fn, n, sync_each=False):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    return th / n * 1e6, (time.perf_counter() - t0) / n * 1e6


def main():
    dev = torch.device("cuda:0")
    pa.native_library()
    wl = bench.Workload(dev)
    step = bench.build_step(wl, 1, "graph", dev)
    for _ in range(20):
        step()
    host, total = rate(step, 200)
    print(f"bench step graph: host enqueue {host:.1f} us/step, total {total:.1f} us/step")
    for nodes in (1, 8, 25, 50):
        x = torch.zeros(1, device=dev)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                for _ in range(nodes):
                    x.add_(1.0)
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            for _ in range(nodes):
                x.add_(1.0)
        for _ in range(10):
            g.replay()
        host, total = rate(g.replay, 200)
        print(f"trivial graph, {nodes:3d} nodes: host {host:.1f} us/replay, total {total:.1f} us/replay, "
              f"{total / nodes:.2f} us/node")


if __name__ == "__main__":
    main()
