"""Summarise tools/rast_prof.py per-tile records: kernel span, start/end spread, phase cycles.

    python tools/rast_timeline.py gpurun_out/rprof_*.npy
"""
import sys

import numpy as np

for path in sys.argv[1:]:
    r = np.load(path)
    t0 = r[:, 4].min()
    st = (r[:, 4] - t0) / 100.0  # s_memrealtime: 100 MHz -> us
    en = (r[:, 5] - t0) / 100.0
    dur = en - st
    print(f"{path}: tiles {len(r)}  span {en.max():.1f} us  last start {st.max():.1f}  dur mean {dur.mean():.1f} "
          f"max {dur.max():.1f}  (CUs seen: {len(np.unique(r[:, 6] & 0xf00007f00))})")
    nl = r[:, 3]
    for lo, hi in [(0, 1), (1, 20), (20, 40), (40, 60), (60, 80), (80, 1000)]:
        m = (nl >= lo) & (nl < hi)
        if m.any():
            ph = (r[m, 7:13].mean(0) / 2.4 / 1000).round(2)  # ~2.4 GHz shader clock -> us
            print(f"  list [{lo:3d},{hi:4d}): {m.sum():5d} tiles  dur {dur[m].mean():6.1f} (max {dur[m].max():6.1f})  "
                  f"start {st[m].mean():6.1f} (max {st[m].max():6.1f})  cull/key/sort/suf/test/out us {ph.tolist()}")
    for i in np.argsort(-en)[:4]:
        print(f"  late tile {r[i,0]},{r[i,1]} list {r[i,3]} start {st[i]:.1f} end {en[i]:.1f}")
    # insert statistics (rec[14] = appends, rec[15] = (inserts << 32) | wave-groups with an insert)
    app, ins, wins = r[:, 14], r[:, 15] >> 32, r[:, 15] & 0xffffffff
    for lo, hi in [(20, 40), (40, 60), (60, 80), (80, 1000)]:
        m = (nl >= lo) & (nl < hi)
        if m.any():
            print(f"  list [{lo:3d},{hi:4d}): appends {app[m].mean():7.1f}  inserts {ins[m].mean():6.1f}  "
                  f"groups with an insert {wins[m].mean():5.1f}")
    # per-SIMD load: heavy tiles (list >= 20) per SIMD and the SIMD's last end
    simd = r[:, 6] & 0xf00007f30  # XCC id (bits 32-35) | SE, SH, CU, SIMD of HW_ID
    heavy = nl >= 20
    ids, inv = np.unique(simd, return_inverse=True)
    nh = np.bincount(inv, weights=heavy.astype(float))
    last = np.zeros(len(ids))
    np.maximum.at(last, inv, en)
    print(f"  SIMDs {len(ids)}: heavy tiles per SIMD histogram {np.bincount(nh.astype(int)).tolist()}")
    for k in range(int(nh.max()) + 1):
        sel = nh == k
        if sel.any():
            print(f"    {k} heavy: {sel.sum():4d} SIMDs, last end mean {last[sel].mean():5.1f} max {last[sel].max():5.1f} us")
