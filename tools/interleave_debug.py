"""Where interleaved and consecutive blend blocks differ on the 128^2 bench frame (debug aid)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import test_gpu_interleave as t  # noqa: E402

dev = torch.device("cuda:0")
for vr in (True, False):
    run = t._bench_frame(dev, vr)
    a = t._with("1", run)
    b = t._with("0", run)
    c = t._with("1", run)
    names = ("image", "d dists", "d zbuf", "d bary", "d vc", "d sigma", "d gamma", "d alpha")
    for x, y, z, n in zip(a, b, c, names):
        d = (x - y).abs()
        nd = int((x != y).sum())
        print(f"vr={vr} {n}: ndiff {nd} max {float(d.max()):.3e} scale {float(y.abs().max()):.3e} "
              f"il-vs-il ndiff {int((x != z).sum())}")
        if nd and x.dim() >= 4:
            idx = (x != y).nonzero()[:8].tolist()
            print("   first", idx, [(float(x[tuple(i)]), float(y[tuple(i)])) for i in idx[:4]])
