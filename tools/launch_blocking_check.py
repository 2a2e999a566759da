"""Does this process run kernel launches host-synchronously (CUDA_LAUNCH_BLOCKING /
HIP_LAUNCH_BLOCKING honoured)?  Times the host side of launching a ~2 ms device spin.

    CUDA_LAUNCH_BLOCKING=1 python tools/launch_blocking_check.py
"""
import os
import time

import torch

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
print(f"{env}: launch returned after {(t1 - t0) * 1e3:.3f} ms, kernel done after {(t2 - t0) * 1e3:.3f} ms -> "
      f"{'blocking' if (t1 - t0) > 0.5 * (t2 - t0) else 'asynchronous'}")
