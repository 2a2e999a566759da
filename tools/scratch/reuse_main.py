"""Scratch: pose_opt.main with the loss traces of every optimize_pose_graph call saved."""
import sys, os, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pertrenderer_amd import pose_opt as po
tag, argv = sys.argv[1], sys.argv[2:]
orig = po.optimize_pose_graph
traces = []
def wrapped(*a, **k):
    r = orig(*a, **k)
    traces.append(np.asarray(r[1]["loss_values"], dtype=np.float64))
    return r
po.optimize_pose_graph = wrapped
rc = po.main(argv)
np.save(f"gpurun_out/reuse/main_{tag}.npy", np.stack(traces))
sys.exit(rc)
