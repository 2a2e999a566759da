"""Scratch: problem-1 loss trace of the cfg5 graph driver with and without GraphSession reuse
(softras only, fresh process per mode), to find where the two runs part."""
import sys, os, json, torch, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pertrenderer_amd import pose_opt as po
mode = sys.argv[1]  # "new" | "ses" | "ses_warm"
nts = sys.argv[2].split(",") if len(sys.argv) > 2 else ["softras"]
dev = torch.device("cuda:0")
torch.manual_seed(1)
scene = po.Scene(dev, 256)
probs = po.make_problems(scene, 3, ["softras", "gaussian"], 20.0)
sessions = {} if mode.startswith("ses") else None
out = {}
for i, p in enumerate(probs):
    target_rgb, R_true, log_rot_init = p
    _, rs = po.init_renderers(scene, R_true, noise_type=nts)
    for nt, r in zip(nts, rs):
        ses = None if sessions is None else sessions.setdefault(nt, po.GraphSession())
        if mode == "ses_warm" and i == 0:
            ses = None
        lr, info = po.optimize_pose_graph(scene, log_rot_init, r, target_rgb, Niter=800, session=ses)
        L = np.asarray(info["loss_values"], dtype=np.float64)
        out[f"{i}_{nt}"] = L
        print(mode, i, nt, "err", round(po.angle_deg(lr, R_true), 4), "nb", info["nb_samples"], flush=True)
np.savez(f"gpurun_out/reuse/trace_{mode}_{'_'.join(nts)}.npz", **out)
