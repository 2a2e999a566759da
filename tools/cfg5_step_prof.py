"""Time one eval.py pose-optimisation iteration (cfg5 renderer: cube + TexturesUV +
RandomPhongShader, 256^2, K=50) at a given sample count, eager, for rocprofv3 --stats.

    python tools/cfg5_step_prof.py --samples 16 8 --iters 50 [--noise gaussian|softras]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pertrenderer_amd import pose_opt as po  # noqa: E402
from pertrenderer_amd.renderer.transforms import Rotate, so3_exponential_map  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, nargs=2, default=(16, 8), help="Sr Sa")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--image-size", type=int, default=256)
    ap.add_argument("--noise", default="gaussian")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(1)
    scene = po.Scene(dev, args.image_size)
    target, R_true = scene.target()
    log_rot0, (renderer,) = po.init_renderers(scene, R_true, noise_type=[args.noise])
    sh = renderer.shader
    sh.smoothrast.nb_samples, sh.smoothagg.nb_samples = args.samples
    log_rot = log_rot0.clone().requires_grad_(True)
    opt = torch.optim.Adam([log_rot], lr=5e-2)
    mesh = scene.meshes

    def it():
        R = so3_exponential_map(log_rot)
        m = mesh.update_padded(Rotate(R).transform_points(mesh.verts_padded()))
        img = renderer(m, cameras=scene.cameras[0], lights=scene.lights)
        loss = ((img[..., :3] - target[0]) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    for _ in range(5):
        it()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        it()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.iters
    print(json.dumps({"noise": args.noise, "Sr": args.samples[0], "Sa": args.samples[1],
                      "ms_per_iter_eager_nosync": round(1e3 * dt, 4)}), flush=True)


if __name__ == "__main__":
    main()
