"""Kernel list of one graph replay (between two seed_advance kernels) from a
rocprofv3 kernel trace:  python tools/replay.py gpurun_out/<dir>"""
import collections
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "*kernel_trace.csv"))[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "seed_advance" in r["Kernel_Name"]]
i0, i1 = idx[len(idx) // 2], idx[len(idx) // 2 + 1]
seq = rows[i0:i1]
span = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seq:
    n = r["Kernel_Name"].replace("void ", "").replace("at::native::", "").replace("(anonymous namespace)::", "")
    n = n.split("(")[0][:80]
    agg[n][0] += 1
    agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print(f"replay: {len(seq)} kernels, span {span:.1f} us")
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{c:4d} {t:8.2f} us  {n}")
