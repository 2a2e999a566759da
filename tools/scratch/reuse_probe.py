"""Scratch: pose_opt.main --graph-reuse with the session state printed around the first replays
of each problem (softras only)."""
import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pertrenderer_amd import pose_opt as po
orig_bind, orig_replay = po.GraphSession.bind, po._CapturedIteration.replay
cnt = {"p": -1, "r": 0}
def bind(self, *a, **k):
    r = orig_bind(self, *a, **k)
    cnt["p"] += 1; cnt["r"] = 0
    st = self.st
    print("BIND", cnt["p"], "log_rot", self.log_rot.data_ptr(), self.log_rot.tolist(), "grad", self.log_rot.grad.tolist(),
          "target", self.target.data_ptr(), float(self.target.sum()), "it", int(st["it"]),
          "opt", {k: (v.data_ptr(), v.tolist()) for k, v in self.opt.state[self.log_rot].items()},
          "lr", float(self.opt.param_groups[0]["lr"]), "blur", float(self.blur),
          "leaves", [(float(l), float(l.grad)) for l in self.renderer.shader.get_smoothing() if torch.is_tensor(l)],
          "nb", po._nb(self.renderer.shader), flush=True)
    return r
def replay(self, n):
    if cnt["r"] < 3:
        for _ in range(2):
            self.graph.replay()
            it = int(self.st["it"])
            print("  REPLAY post", self.post, "it", it, "loss", float(self.st["losses"][it - 1]),
                  "log_rot", self.log_rot.data_ptr(), self.log_rot.tolist(), "grad", self.log_rot.grad.tolist(),
                  "step", self.opt.state[self.log_rot]["step"].tolist(), flush=True)
        n -= 2
    cnt["r"] += 1
    return orig_replay(self, n)
po.GraphSession.bind, po._CapturedIteration.replay = bind, replay
sys.exit(po.main(sys.argv[1:]))
