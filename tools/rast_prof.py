"""Per-tile timeline + phase cycles of rast_fwd on the bench frame.  Needs the
-DPR_RAST_PROFILE variant:
    python -m pertrenderer_amd.build_native --out pertrenderer_amd/libpertrender_prof.so -D PR_RAST_PROFILE
    PR_NATIVE_LIB=pertrenderer_amd/libpertrender_prof.so python tools/rast_prof.py OUT.npy
Records (int64 x16 per tile): x y z list t0 t1 hw_id cull key sort suf test out SL (t in 100 MHz ticks)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pertrenderer_amd import _native as nat  # noqa: E402

name = os.environ.get("PR_PROF_CONFIG", "cfg2")
cfg = bench.CONFIGS[name]
wl = bench.Workload(torch.device("cuda:0"), cfg["image_size"], cfg["K"], cfg["samples"], batch=cfg["batch"],
                    rast_samples=cfg.get("rast_samples"), eval_scene=name == "eval")
for _ in range(3):  # warm: the last forward's records are kept
    wl.forward().backward()
    torch.cuda.synchronize()
lib = nat.load()
buf = np.zeros((1 << 16) * 16, dtype=np.int64)
assert lib.pr_rast_prof_dump(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(buf.nbytes)) == 0
rec = buf.reshape(-1, 16)
rec = rec[rec[:, 5] != 0]
np.save(sys.argv[1] if len(sys.argv) > 1 else "rast_prof.npy", rec)
print("rast_prof done", len(rec), flush=True)
