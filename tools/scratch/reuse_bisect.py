"""Scratch: which call between problems breaks the reused graphs' loss records."""
import sys, os, torch, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pertrenderer_amd import pose_opt as po
variant = sys.argv[1]
dev = torch.device("cuda:0")
if "setdev" in variant:
    torch.cuda.set_device(dev)
torch.manual_seed(1)
scene = po.Scene(dev, 256)
probs = po.make_problems(scene, 3, ["softras", "gaussian"], 20.0)
sessions = {}
for i, p in enumerate(probs):
    target_rgb, R_true, log_rot_init = p
    _, rs = po.init_renderers(scene, R_true, noise_type=["softras"])
    if "sync" in variant:
        torch.cuda.synchronize()
    lr, info = po.optimize_pose_graph(scene, log_rot_init, rs[0], target_rgb, Niter=800,
                                      session=sessions.setdefault("softras", po.GraphSession()))
    if "sync" in variant:
        torch.cuda.synchronize()
    e = po.angle_deg(lr, R_true)
    if "init" in variant:
        e0 = po.angle_deg(log_rot_init, R_true)
    L = info["loss_values"]
    print(variant, i, "err", round(e, 3), "loss", [round(L[k], 7) for k in (0, 1, 2, 100, 101, 799)], flush=True)
