"""Per-phase s_memtime cycle counts of rast_fwd / rast_bwd on the bench frame (heavy
tiles only).  Needs the -DPR_RAST_PROFILE variant:
    python -m pertrenderer_amd.build_native --out pertrenderer_amd/libpertrender_prof.so -D PR_RAST_PROFILE
    PR_NATIVE_LIB=pertrenderer_amd/libpertrender_prof.so python tools/rast_prof.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

wl = bench.Workload(torch.device("cuda:0"))
wl.forward().backward()
torch.cuda.synchronize()
print("rast_prof done", flush=True)
