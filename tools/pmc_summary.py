"""Summarise rocprofv3 --pmc counter CSVs per native kernel (mean per dispatch).

    python tools/pmc_summary.py DIR... [--traffic-out profiles/pmc_traffic.json]

With --traffic-out, writes per-kernel HBM traffic per launch for bench.py's
`roofline.traffic`, corrected as /opt/skills/guides/MI355X_MICROARCH.md's
HBM/rocprofv3 section prescribes: FETCH_SIZE / WRITE_SIZE are KiB; on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads, so it is doubled."""
import collections
import csv
import glob
import json
import os
import sys

SHORT = {"blend_fwd_kernel": "blend_fwd", "blend_bwd_kernel": "blend_bwd", "rast_fwd_kernel": "rast_fwd",
         "rast_bwd_kernel": "rast_bwd", "interp_fwd_kernel": "interp_fwd", "interp_bwd_kernel": "interp_bwd",
         "rast_frag_kernel": "rast_frag"}


def kname(raw):
    return raw.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("pr::", "")


def load(dirs):
    data = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                data[kname(r["Kernel_Name"])][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
    out = {}
    for k, cs in data.items():
        out[k] = {}
        for c, vals in cs.items():
            per = collections.defaultdict(float)
            for did, v in vals:
                per[did] += v
            out[k][c] = sum(per.values()) / len(per)
    return out


def traffic(res):
    tr = {}
    for k, c in res.items():
        short = SHORT.get(k.split("<")[0])
        if short is None or "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        rd, wr = 2.0 * c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
        tr[short] = {"bytes_per_launch": int(rd + wr), "read_bytes": int(rd), "write_bytes": int(wr),
                     "kernel": k, "correction": "FETCH_SIZE x2 (gfx950 wide-read half count), KiB -> bytes"}
    return tr


if __name__ == "__main__":
    args = sys.argv[1:]
    out = None
    if "--traffic-out" in args:
        i = args.index("--traffic-out")
        out = args[i + 1]
        del args[i:i + 2]
    res = load(args)
    for k in sorted(res, key=lambda x: -res[x].get("SQ_WAVE_CYCLES", 0)):
        if any(s in k for s in ("blend", "rast", "interp", "project", "heaviside")):
            print(k, json.dumps({c: round(v) for c, v in sorted(res[k].items())}))
    if out:
        json.dump(traffic(res), open(out, "w"), indent=1)
        print("wrote", out)
