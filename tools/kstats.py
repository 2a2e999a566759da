"""Print the native kernels' rows of a rocprofv3 --stats kernel summary (µs)."""
import csv
import glob
import os
import sys

for f in glob.glob(os.path.join(sys.argv[1], "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("pr::", "")
        if any(s in n for s in ("blend", "rast", "interp", "project", "heaviside", "face_prep", "seed")):
            print(f"{n:45s} calls {int(r['Calls']):5d} avg {float(r['AverageNs']) / 1e3:9.2f} us  "
                  f"min {float(r['MinNs']) / 1e3:9.2f}  max {float(r['MaxNs']) / 1e3:9.2f}")
