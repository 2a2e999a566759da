"""Where a cfg 5 problem's time goes in graph mode: graph (re)captures against replays.

    python tools/cfg5_capture_cost.py [problems] [--sessions]

Wraps pose_opt._CapturedIteration (construction = warm-up pass + capture) and its replay with
device synchronisations, runs compare_pose_opt's problems through optimize_pose_graph and prints
the per-problem totals and the schedule states each capture was for."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pertrenderer_amd import pose_opt as po  # noqa: E402


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    n = int(args[0]) if args else 3
    dev = torch.device("cuda:0")
    torch.manual_seed(1)
    scene = po.Scene(dev, 256)
    acc = {"capture": 0.0, "replay": 0.0, "captures": 0, "replays": 0}
    Cap = po._CapturedIteration
    init0, replay0 = Cap.__init__, Cap.replay

    def init(self, *a, **k):
        torch.cuda.synchronize()
        t = time.perf_counter()
        init0(self, *a, **k)
        torch.cuda.synchronize()
        acc["capture"] += time.perf_counter() - t
        acc["captures"] += 1

    def replay(self, m):
        torch.cuda.synchronize()
        t = time.perf_counter()
        replay0(self, m)
        torch.cuda.synchronize()
        acc["replay"] += time.perf_counter() - t
        acc["replays"] += m

    Cap.__init__, Cap.replay = init, replay
    sessions = {} if "--sessions" in sys.argv else None
    for noise_type in ("gaussian", "softras"):
        for p in range(n):
            target, R_true = scene.target()
            log_rot0, (renderer,) = po.init_renderers(scene, R_true, noise_type=[noise_type])
            for k in acc:
                acc[k] = 0 if isinstance(acc[k], int) else 0.0
            t = time.perf_counter()
            ses = None if sessions is None else sessions.setdefault(noise_type, po.GraphSession())
            po.optimize_pose_graph(scene, log_rot0, renderer, target, Niter=800, session=ses)
            torch.cuda.synchronize()
            tot = time.perf_counter() - t
            print(f"{noise_type} problem {p}: {tot:.3f} s; captures {acc['captures']} in {acc['capture']:.3f} s, "
                  f"replays {acc['replays']} in {acc['replay']:.3f} s ({1e3 * acc['replay'] / max(acc['replays'], 1):.3f} "
                  f"ms each), other {tot - acc['capture'] - acc['replay']:.3f} s; final S "
                  f"{(ses.renderer if ses is not None else renderer).shader.get_nb_samples()}",
                  flush=True)


if __name__ == "__main__":
    main()
