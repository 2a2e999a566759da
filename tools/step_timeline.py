"""One graph step's kernel timeline from a rocprofv3 kernel trace (between two launches of the
step's first kernel: so3_exp_fwd since the seed advance moved into project_prep).

    python tools/step_timeline.py gpurun_out/prof_TAG/prof_kernel_trace.csv [step_index] [first_kernel]
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
first = sys.argv[3] if len(sys.argv) > 3 else "so3_exp_fwd"
idx = [i for i, x in enumerate(rows) if first in x["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(idx) // 2
i0, i1 = idx[k], idx[k + 1]
t0 = int(rows[i0]["Start_Timestamp"])
busy = 0
for x in rows[i0:i1]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1000:8.1f} {(e - s) / 1000:7.1f}  {x['Kernel_Name'][:100]}")
span = (int(rows[i1]["Start_Timestamp"]) - t0) / 1000
print(f"step span {span:.1f} us, kernels {i1 - i0}, kernel-busy {busy / 1000:.1f} us")
