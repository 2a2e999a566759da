import sys, os, torch, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pertrenderer_amd import pose_opt as po
dev = torch.device("cuda:0")
torch.manual_seed(0)
scene = po.Scene(dev, 256)
NT = ["softras", "gaussian"]
probs = po.make_problems(scene, 3, NT, 20.0)
for use in (False, True):
    torch.manual_seed(1)
    sessions = {} if use else None
    for i, p in enumerate(probs):
        target_rgb, R_true, log_rot_init = p
        _, rs = po.init_renderers(scene, R_true, noise_type=NT)
        for nt, r in zip(NT, rs):
            ses = None if sessions is None else sessions.setdefault(nt, po.GraphSession())
            lr, info = po.optimize_pose_graph(scene, log_rot_init, r, target_rgb, Niter=800, session=ses)
            L = info["loss_values"]
            print("ses" if use else "new", i, nt, "err", round(po.angle_deg(lr, R_true), 3),
                  "loss", [round(L[k], 6) for k in (0, 1, 2, 50, 100, 101, 150, 799)], flush=True)
