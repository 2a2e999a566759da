"""Per-step kernel list of the bench step, each kernel attributed to the call that issued it
(VERDICT r4 item 4).

Runs bench.Workload's step eagerly through the same host layer and kernels as the captured graph
(device seed, device smoothing scalars, capturable fused Adam), under torch.profiler, with the
step's stages labelled (record_function) and the backward split by autograd node.  Prints one
line per device kernel of the last profiled step: stage / issuing op / kernel; and a count.

    python tools/step_kernels.py [--config cfg2] [--steps 3] [--json out.json]
"""
import argparse
import collections
import json
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile, record_function

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import pertrenderer_amd as pa  # noqa: E402
from pertrenderer_amd.renderer.transforms import Rotate, so3_exponential_map  # noqa: E402


def step(wl, ds):
    if ds is not None:
        with record_function("## seed advance"):
            ds.advance()
    with record_function("## pose (so3 exp, rotate)"):
        R = so3_exponential_map(wl.log_rot)
        mesh = wl.base.update_padded(Rotate(R).transform_points(wl.base.verts_padded()))
    kw = {"lights": wl.lights} if wl.lights is not None else {}
    with record_function("## renderer (rasterizer + shader)"):
        images = wl.renderer(mesh, cameras=wl.cameras, **kw)
    with record_function("## loss (caller)"):
        if wl.loss_kind == "native":  # bench's default: eval.py's loss on pose_opt.rgb_mse
            from pertrenderer_amd.pose_opt import rgb_mse
            loss = rgb_mse(images, wl.target)
        else:
            loss = ((images[..., :3] - wl.target) ** 2).mean()
    with record_function("## backward"):
        loss.backward(wl.one)
    with record_function("## adam (caller)"):
        wl.opt.step()
    wl.zero_grad()


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2", choices=sorted(bench.CONFIGS))
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--json", default=None)
    ap.add_argument("--loss", choices=["native", "torch"], default="native", help="bench.py --loss")
    ap.add_argument("--mode", choices=["graph", "eager"], default="graph",
                    help="graph: the captured step's configuration (device seed and smoothing scalars, "
                         "capturable Adam), run eagerly; eager: bench --mode eager / eval.py's (CPU smoothing "
                         "leaves, host Philox keys)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    pa.native_library()
    c = bench.CONFIGS[args.config]
    wl = bench.Workload(dev, c["image_size"], c["K"], c["samples"], batch=c["batch"],
                        rast_samples=c.get("rast_samples"), eval_scene=args.config == "eval", loss=args.loss)
    if args.mode == "graph":
        ds = pa.noise.DeviceSeed(dev)
        pa.noise.use_device_seed(ds)
        wl.device_scalars()
        wl.opt = torch.optim.Adam([wl.log_rot], lr=5e-2, capturable=True, fused=True)
    else:
        ds = None
        wl.opt = torch.optim.Adam([wl.log_rot], lr=5e-2, fused=True)
    for _ in range(3):
        step(wl, ds)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for i in range(args.steps):
            with record_function(f"#step {i}"):
                step(wl, ds)
        torch.cuda.synchronize()
    # the chrome trace links each kernel to its launch call (runtime event, "correlation"): a
    # launch's enclosing labelled ranges give the stage and, in the backward, the autograd node
    import tempfile
    tr = os.path.join(tempfile.mkdtemp(), "trace.json")
    prof.export_chrome_trace(tr)
    ev = json.load(open(tr))["traceEvents"]
    X = [e for e in ev if e.get("ph") == "X"]
    steps = sorted((e for e in X if e.get("name", "").startswith("#step ")), key=lambda e: e["ts"])
    last = steps[-1]
    t0, t1 = last["ts"], last["ts"] + last["dur"]
    ranges = [e for e in X if e.get("cat") in ("user_annotation", "cpu_op", "python_function")
              and t0 <= e["ts"] <= t1]
    launches = {e["args"]["correlation"]: e for e in X if e.get("cat") == "cuda_runtime"
                and "correlation" in e.get("args", {}) and t0 <= e["ts"] <= t1}
    kern = [e for e in X if e.get("cat") in ("kernel", "gpu_memcpy", "gpu_memset")
            and e.get("args", {}).get("correlation") in launches]
    out = []
    for k in sorted(kern, key=lambda e: e["ts"]):
        la = launches[k["args"]["correlation"]]
        encl = sorted((r for r in ranges if r["ts"] <= la["ts"] and la["ts"] + la.get("dur", 0) <= r["ts"] + r["dur"]),
                      key=lambda r: -r["ts"])
        stage = next((r["name"] for r in encl if r["name"].startswith("## ")), "?")
        node = next((r["name"].replace("autograd::engine::evaluate_function: ", "") for r in encl
                     if r["name"].startswith("autograd::engine::evaluate_function")), "")
        op = next((r["name"] for r in encl if r.get("cat") == "cpu_op" and not r["name"].startswith("autograd::")), "")
        out.append(dict(stage=stage, node=node, op=op or la["name"], kernel=short(k["name"]),
                        us=round(k.get("dur", 0), 2)))
    for o in out:
        print(f"{o['stage']:34s} {o['node'][:28]:28s} {o['op'][:30]:30s} {o['us']:7.2f} {o['kernel']}")
    cnt = collections.Counter(o["stage"] for o in out)
    print(f"kernels per step: {len(out)}", dict(cnt))
    if args.json:
        json.dump({"config": args.config, "mode": args.mode, "kernels_per_step": len(out), "by_stage": dict(cnt), "kernels": out},
                  open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
