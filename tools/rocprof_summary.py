"""rocprofv3 --kernel-trace --stats CSV -> profiles/rocprof_kernels.json (per-kernel average
duration, stamped with the native sources' sha): the committed basis bench.py's roofline
reports beside its live per-kernel event timing.

    python tools/rocprof_summary.py <kernel_stats.csv> <out.json> "<run description>"
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pertrenderer_amd.build_native import source_sha  # noqa: E402


def short(raw):
    """rocprof's demangled name -> the bare kernel name (blend_bwd_kernel, ...)."""
    n = raw.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("pr::", "")
    return n.split("<")[0]


def main(src, dst, run):
    kernels = {}
    for r in csv.DictReader(open(src)):
        name = short(r["Name"])
        if name in kernels:  # template variants of one kernel: keep the most called
            if int(r["Calls"]) <= kernels[name]["calls"]:
                continue
        kernels[name] = {"avg_us": round(float(r["AverageNs"]) / 1e3, 3), "calls": int(r["Calls"]),
                         "min_us": round(float(r["MinNs"]) / 1e3, 3), "max_us": round(float(r["MaxNs"]) / 1e3, 3),
                         "variant": r["Name"].replace("(anonymous namespace)::", "").split("(")[0]}
    json.dump({"source_sha": source_sha(), "run": run, "kernels": kernels}, open(dst, "w"), indent=1)
    for k in ("rast_fwd_kernel", "rast_bwd_kernel", "blend_fwd_kernel", "blend_bwd_kernel"):
        if k in kernels:
            print(k, kernels[k]["avg_us"], "us")


if __name__ == "__main__":
    main(*sys.argv[1:4])
