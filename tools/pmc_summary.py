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

# C-ABI call (bench.py's timed unit) -> the kernels it launches
CALLS = {"rast_fwd": ["face_prep_kernel", "project_prep_kernel", "rast_fwd_kernel", "rast_frag_kernel"],
         "rast_bwd": ["rast_bwd_kernel"],
         "blend_fwd": ["blend_fwd_kernel"],
         "blend_bwd": ["blend_bwd_kernel", "blend_finalize_kernel"],
         "interp_fwd": ["interp_fwd_kernel"], "interp_bwd": ["interp_bwd_kernel"]}


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
    """Per C-ABI call: summed HBM bytes per launch of its kernels."""
    tr = {}
    for call, kernels in CALLS.items():
        rd = wr = valu = 0.0
        found = []
        for k, c in res.items():
            if k.split("<")[0] in kernels and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                rd += 2.0 * c["FETCH_SIZE"] * 1024
                wr += c["WRITE_SIZE"] * 1024
                valu += c.get("SQ_INSTS_VALU", 0.0)
                found.append(k)
        if found:
            tr[call] = {"bytes_per_launch": int(rd + wr), "read_bytes": int(rd), "write_bytes": int(wr),
                        "kernels": found, "correction": "FETCH_SIZE x2 (gfx950 wide-read half count), KiB -> bytes",
                        # VALU issue time if the instructions were spread evenly: wave64 VALU
                        # op = 4 cycles on a SIMD, 1024 SIMDs, 2.4 GHz
                        "valu_insts_per_launch": int(valu),
                        "valu_issue_us": round(valu * 4 / (1024 * 2.4e3), 2)}
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
        if any(s in k for s in ("blend", "rast", "interp", "project", "heaviside", "shade")):
            print(k, json.dumps({c: round(v) for c, v in sorted(res[k].items())}))
    if out:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from pertrenderer_amd.build_native import source_sha
        tr = traffic(res)
        tr["source_sha"] = source_sha()  # bench.py uses the record only for the same native sources
        tr["_run"] = os.environ.get("PR_PROFILE_RUN", "tools/gpu.sh pmc")
        json.dump(tr, open(out, "w"), indent=1)
        print("wrote", out)
