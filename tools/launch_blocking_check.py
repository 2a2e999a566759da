"""Does this process run kernel launches host-synchronously (CUDA_LAUNCH_BLOCKING /
HIP_LAUNCH_BLOCKING honoured)?  Times the host side of launching a ~2 ms device spin.

    CUDA_LAUNCH_BLOCKING=1 python tools/launch_blocking_check.py
    python tools/launch_blocking_check.py --eval-order   # eval.py's own order (eval.py:4, :22, :26):
        # set CUDA_LAUNCH_BLOCKING=1 in-process, import torch, import the pytorch3d shim, then launch
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EVAL_ORDER = "--eval-order" in sys.argv
if EVAL_ORDER:
    os.environ["CUDA_LAUNCH_BLOCKING"] = "1"  # eval.py:4

import torch  # noqa: E402

if EVAL_ORDER:
    sys.path.insert(0, ROOT)
    import pytorch3d.loss  # noqa: E402,F401  (eval.py:26: the shim's first import)

torch.cuda.init()
x = torch.zeros(1, device="cuda")
torch.cuda._sleep(1000)
torch.cuda.synchronize()
t0 = time.perf_counter()
torch.cuda._sleep(5_000_000)  # ~2 ms of spinning on the device
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
env = {k: os.environ.get(k) for k in ("CUDA_LAUNCH_BLOCKING", "HIP_LAUNCH_BLOCKING", "AMD_SERIALIZE_KERNEL")}
blocking = (t1 - t0) > 0.5 * (t2 - t0)
print(f"{'eval-order ' if EVAL_ORDER else ''}{env}: launch returned after {(t1 - t0) * 1e3:.3f} ms, kernel done after "
      f"{(t2 - t0) * 1e3:.3f} ms -> {'blocking' if blocking else 'asynchronous'}")
if EVAL_ORDER and not blocking:
    sys.exit(1)
