"""Per-block timeline + phase cycles of the bench frame's blend kernels.  Needs the
-DPR_BLEND_PROFILE variant:
    python -m pertrenderer_amd.build_native --out pertrenderer_amd/libpertrender_prof.so -D PR_BLEND_PROFILE
    PR_NATIVE_LIB=pertrenderer_amd/libpertrender_prof.so python tools/blend_prof.py
Forward phases: setup / slots / MC rast / pixel / MC argmax / output.  Backward: setup / B1 / B2 /
B5 / B6 / B7 / B8 / reduction.  Phases are summed over a block's passes."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pertrenderer_amd import _native as nat  # noqa: E402

import argparse  # noqa: E402
ap = argparse.ArgumentParser()
ap.add_argument("--config", choices=sorted(bench.CONFIGS), default="cfg2")
ap.add_argument("--dense", action="store_true", help="the dense-fragment microbench (bench.dense_roofline's blend)")
args = ap.parse_args()
cfg = bench.CONFIGS[args.config]
# blocks past the first 65536 are not recorded (a cfg4 frame has 524288: images 0-1 only)
if args.dense:
    bench.dense_roofline(torch.device("cuda:0"), cfg["image_size"], cfg["K"], cfg["samples"], iters=2,
                         Sr=cfg.get("rast_samples"))
else:
    wl = bench.Workload(torch.device("cuda:0"), cfg["image_size"], cfg["K"], cfg["samples"], batch=cfg["batch"])
    for _ in range(3):
        wl.forward().backward()
        torch.cuda.synchronize()
lib = nat.load()
NB = 1 << 16
REC = 12
buf = np.zeros(2 * NB * REC, dtype=np.int64)
assert lib.pr_blend_prof_dump(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(buf.nbytes)) == 0
rec = buf.reshape(2, NB, REC)
for w, name, ph in ((0, "blend_fwd", ["setup", "slots", "rast", "pixel", "argmax", "out"]),
                    (1, "blend_bwd", ["setup", "B1", "B2", "B5", "B6", "B7", "B8", "red"])):
    r = rec[w][rec[w][:, REC - 1] == 1]
    t0 = r[:, 0].min()
    st, en = (r[:, 0] - t0) / 100.0, (r[:, 1] - t0) / 100.0
    print(f"{name}: blocks {len(r)} span {en.max():.1f} us, last start {st.max():.1f}, dur mean {(en - st).mean():.1f} "
          f"max {(en - st).max():.1f}")
    pm = (r[:, 2:2 + len(ph)].mean(0) / 2400).round(2)
    px = (r[:, 2:2 + len(ph)].max(0) / 2400).round(2)
    print("  phase us mean", dict(zip(ph, pm.tolist())), "\n  phase us max ", dict(zip(ph, px.tolist())))
    hist = np.histogram(st, bins=8)[0]
    print("  start histogram", hist.tolist())
    dur = en - st
    for q in (50, 90, 99):
        print(f"  duration p{q} {np.percentile(dur, q):.1f} us")
    for i in np.argsort(-dur)[:5]:  # the longest blocks: start, duration, phases
        print(f"  long block start {st[i]:.1f} dur {dur[i]:.1f} phases",
              dict(zip(ph, (r[i, 2:2 + len(ph)] / 2400).round(2).tolist())))
