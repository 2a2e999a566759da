"""Per-kernel cost of a chain of dependent tiny kernels on one stream: eager launches and a
captured HIP graph replay (torch add_ on a 1-element tensor, n kernels), microseconds per kernel.
Diagnostic for the step's small-kernel floor (25 kernels per cfg-2 step)."""
import json

import torch

dev = torch.device("cuda:0")
x = torch.zeros(1, device=dev)
big = torch.zeros(256 * 256 * 3, device=dev)
out = {}
for name, t in (("1 elem", x), ("196608 elem", big)):
    for n in (10, 50):
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                for _ in range(n):
                    t.add_(1.0)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(n):
                t.add_(1.0)
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 50
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        out[f"graph {name} x{n}"] = round(e0.elapsed_time(e1) * 1e3 / (reps * n), 3)
        e0.record()
        for _ in range(reps):
            for _ in range(n):
                t.add_(1.0)
        e1.record()
        torch.cuda.synchronize()
        out[f"eager {name} x{n}"] = round(e0.elapsed_time(e1) * 1e3 / (reps * n), 3)
print(json.dumps(out, indent=1))
