"""Resident workgroups per CU of the blend kernels at each BASELINE config (HIP occupancy
calculator, via the library's pr_diag_blend_occupancy), with the block counts they must cover.

    python tools/blend_occupancy.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pertrenderer_amd import _native as nat  # noqa: E402

lib = nat.load()
fn = lib.pr_diag_blend_occupancy
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
for name, cfg in sorted(bench.CONFIGS.items()):
    P = cfg["batch"] * cfg["image_size"] ** 2
    for cm in (1, 2):
        out = (ctypes.c_int * 8)()
        rc = fn(cfg["K"], cfg["samples"], P, cm, out)
        print(f"{name} cm={cm} P={P}: rc {rc}  per-CU blocks fwd {out[0]} (multi {out[1]}) lds {out[4]}  "
              f"bwd {out[2]} (multi {out[3]}) lds {out[6]}")
