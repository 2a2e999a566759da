"""Fragment statistics of a bench frame (what the blend kernels' Monte-Carlo work scales with):
valid slots per pixel, Gaussian-unsaturated slots (|dist/sigma| <= 5.8: the forward's rast MC
queue), covered pixels.  python tools/frag_stats.py --config cfg4"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pertrenderer_amd.renderer.rasterizer import valid_counts  # noqa: E402
from pertrenderer_amd.renderer.transforms import Rotate, so3_exponential_map  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", choices=sorted(bench.CONFIGS), default="cfg2")
cfg = bench.CONFIGS[ap.parse_args().config]
wl = bench.Workload(torch.device("cuda:0"), cfg["image_size"], cfg["K"], cfg["samples"], batch=cfg["batch"])
with torch.no_grad():
    R = so3_exponential_map(wl.log_rot)
    mesh = wl.base.update_padded(Rotate(R).transform_points(wl.base.verts_padded()))
    frag = wl.renderer.rasterizer(mesh, cameras=wl.cameras)
p2f, d = frag.pix_to_face, frag.dists
valid = p2f >= 0
cnt = valid.sum(-1)
c = valid_counts(p2f)
unsat = valid & (d.abs() <= 5.8 * 1e-3)
P = cnt.numel()
cov = (cnt > 0).sum().item()
print(f"{cfg}: pixels {P}, covered {cov} ({cov / P:.3f}), counts attached {c is not None}")
print(f"valid slots/pixel: mean {cnt.float().mean():.2f}, over covered {cnt.sum().item() / max(cov, 1):.2f}, "
      f"max {cnt.max().item()}, p99 {cnt.float().flatten().quantile(0.99).item() if P < 2**24 else float('nan'):.0f}")
print(f"unsaturated slots: total {unsat.sum().item()}, /pixel {unsat.sum().item() / P:.3f}, "
      f"/covered {unsat.sum().item() / max(cov, 1):.3f}, pixels with any {unsat.any(-1).sum().item()}")
hist = torch.bincount(cnt.flatten().clamp(max=40), minlength=41).tolist()
print("count histogram (0..40+):", hist)
