"""Rasterizer forward time with and without coarse bins (PR_RAST_BINS semantics through
RasterizationSettings.bin_size): sphere_642 (1280 faces) and its 3x subdivision (81 920 faces)
at 256^2 / 512^2, K = 50, cfg 2's blur.  Mean of 20 launches between HIP events (no grad).

    python tools/rast_bins_bench.py OUT.json
"""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import meshgen  # noqa: E402
from pertrenderer_amd.renderer import (FoVPerspectiveCameras, MeshRasterizer, Meshes,  # noqa: E402
                                       RasterizationSettings, look_at_view_transform)


def main():
    dev = torch.device("cuda:0")
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=dev)
    cams = FoVPerspectiveCameras(R=R, T=T, device=dev)
    blur = math.log(1.0 / 1e-4 - 1.0) * 1e-3
    out = []
    for levels in (0, 3):
        v, f = meshgen.fine_sphere(levels)
        mesh = Meshes([torch.tensor(v, device=dev)], [torch.tensor(f, device=dev)])
        for size in (256, 512):
            ref = None
            for bs in (0, None, 8, 16, 32):
                rs = RasterizationSettings(image_size=size, blur_radius=blur, faces_per_pixel=50, bin_size=bs,
                                           max_faces_per_bin=50000)
                r = MeshRasterizer(cameras=cams, raster_settings=rs)
                with torch.no_grad():
                    for _ in range(3):
                        frag = r(mesh)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(20):
                        r(mesh)
                    e1.record()
                    torch.cuda.synchronize()
                same = True
                if ref is None:
                    ref = frag.pix_to_face
                else:
                    same = bool(torch.equal(ref, frag.pix_to_face))
                row = dict(faces=int(f.shape[0]), image=size, bin_size=bs, ms=e0.elapsed_time(e1) / 20, same=same)
                print(row, flush=True)
                out.append(row)
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
