"""Host cost of one launch in the current launch mode: mean wall time of N tiny dependent kernel
launches (torch.cuda._sleep of a few cycles) with a synchronise at the end.  Under
HIP_LAUNCH_BLOCKING=1 every launch waits for its kernel, so this is the per-op round trip eval.py's
launch-blocking mode pays; HSA_ENABLE_INTERRUPT=0 makes those waits poll instead of sleeping on an
interrupt.

    HIP_LAUNCH_BLOCKING=1 [HSA_ENABLE_INTERRUPT=0] python tools/launch_blocking_cost.py
"""
import json
import os
import time

import torch

n = 2000
x = torch.zeros(1024, device="cuda")
for _ in range(200):
    x.add_(1.0)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    x.add_(1.0)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / n
print(json.dumps({"env": {k: os.environ.get(k) for k in ("HIP_LAUNCH_BLOCKING", "HSA_ENABLE_INTERRUPT")},
                  "us_per_launch": round(dt * 1e6, 2)}))
