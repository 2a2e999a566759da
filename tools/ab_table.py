"""Per-kernel table of a same-lease A/B (tools/ab.sh): rocprofv3 average durations (us) of every
kernel in each side's runs, with the bench lines' frames/s.

    python tools/ab_table.py gpurun_out/ab_TAG [A-label B-label]
"""
import csv
import glob
import json
import os
import sys


def short(raw):
    n = raw.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("pr::", "")
    return n if len(n) < 60 else n[:57] + "..."


def main(d, la="A", lb="B"):
    rows = {}
    lines = {}
    for side in ("A", "B"):
        for f in sorted(glob.glob(os.path.join(d, f"{side}_prof_r*", "**", "*kernel_stats.csv"), recursive=True)):
            for r in csv.DictReader(open(f)):
                rows.setdefault(short(r["Name"]), {}).setdefault(side, []).append(float(r["AverageNs"]) / 1e3)
        lines[side] = [json.load(open(f))["value"] for f in sorted(glob.glob(os.path.join(d, f"{side}_r*.json")))]
    print(f"frames/s  {la}: {lines['A']}  {lb}: {lines['B']}")
    print(f"{'kernel':60s} {la:>16s} {lb:>16s}  delta")
    keyed = sorted(rows.items(), key=lambda kv: -max(sum(v) / len(v) for v in kv[1].values()))
    for k, v in keyed[:24]:
        a, b = v.get("A", []), v.get("B", [])
        ma = sum(a) / len(a) if a else float("nan")
        mb = sum(b) / len(b) if b else float("nan")
        fa = "/".join(f"{x:.1f}" for x in a)
        fb = "/".join(f"{x:.1f}" for x in b)
        print(f"{k:60s} {fa:>16s} {fb:>16s}  {mb - ma:+.1f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
