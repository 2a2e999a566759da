"""Kernel-profiling driver: the bench workload's forward+backward, eagerly, a few
times (for rocprofv3 --pmc passes; one process, no graph, no CPU baseline).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d out -- python tools/kprof.py
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import pertrenderer_amd as pa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--dense", action="store_true", help="dense synthetic fragments (blend only)")
    ap.add_argument("--config", choices=sorted(bench.CONFIGS), default="cfg2")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    pa.native_library()
    if args.dense:
        bench.dense_roofline(dev, iters=args.iters)
    else:
        c = bench.CONFIGS[args.config]
        wl = bench.Workload(dev, c["image_size"], c["K"], c["samples"], batch=c["batch"])
        for _ in range(args.iters):
            wl.forward().backward()
            wl.zero_grad()
    torch.cuda.synchronize()
    print("kprof done")


if __name__ == "__main__":
    main()
