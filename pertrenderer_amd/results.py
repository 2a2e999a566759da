"""eval.py's result formats: writers that produce the same files as
experiments/eval.py, readers, and a comparison of two runs' pose-error tables.

Files and formats follow the reference:
* `compare_runtime` (eval.py:566-573): `runtimes.txt`, `memory.txt` -- one `json.dump`
  each, {noise_type: [mean per setting]}.
* `compare_pose_opt` (eval.py:644-661): `angle_error.txt`, `angle_error_final.txt`,
  `angle_error_init.txt`, `angle_std.txt`, `solved_percentage.txt`, `params.txt`,
  `exp_setup.txt` -- one `json.dump` each.
* `optimize_pose` (eval.py:394-405): `optimization_details/<date>/loss_values.npy`,
  `gradient_values.npy` (`np.save` of the per-iteration lists) and the training-image grid
  `grid_cube.png` (`image_grid`, eval.py:787-821: rows x cols axes, RGB clipped to [0, 1]
  or the alpha channel, axes off, tight bbox).
Results live in `<cwd>/../experiments/results/<exp_id>` as in eval.py:396-397 / :566-567.

`compare_pose_results` puts a GPU run beside a CPU run of the same seeds: per noise type
and setting, the mean angle error difference and the solved-fraction difference at each
threshold.  (The reference has no such tool: its tables are read back with pandas, eval.py:662-665.)
"""
import json
from datetime import datetime
from pathlib import Path

import numpy as np

RUNTIME_FILES = {"mean_runtimes": "runtimes.txt", "mean_memory": "memory.txt"}
POSE_FILES = {
    "mean_errors": "angle_error.txt",
    "final_errors": "angle_error_final.txt",
    "init_errors": "angle_error_init.txt",
    "var_errors": "angle_std.txt",
    "mean_solved": "solved_percentage.txt",
    "params": "params.txt",
    "exp_setup": "exp_setup.txt",
}
DETAIL_DIR = "optimization_details"
DATE_FORMAT = "%Y-%m-%d-%H:%M:%S"  # eval.py:398


def _plain(x):
    """json.dump hook for numpy / torch scalars and arrays (eval.py's tables hold python
    floats; a caller passing numpy values gets the same text)."""
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    if isinstance(x, np.ndarray):
        return x.tolist()
    if isinstance(x, np.generic):
        return x.item()
    raise TypeError(f"not JSON serialisable: {type(x).__name__}")


def results_dir(exp_id, cwd=None):
    """`Path().cwd().parent / 'experiments/results/<exp_id>'` (eval.py:396-397, :566-567)."""
    base = Path(cwd) if cwd is not None else Path().cwd()
    return base.parent / ("experiments/results/" + str(exp_id))


def _dump(path, obj):
    with open(path, "w") as f:
        json.dump(obj, f, default=_plain)


def write_runtime_results(path_res, mean_runtimes, mean_memory):
    """eval.py:568-573."""
    path_res = Path(path_res)
    path_res.mkdir(parents=True, exist_ok=True)
    _dump(path_res / RUNTIME_FILES["mean_runtimes"], mean_runtimes)
    _dump(path_res / RUNTIME_FILES["mean_memory"], mean_memory)


def write_pose_results(path_res, mean_errors, final_errors, init_errors, var_errors, mean_solved, params,
                       exp_setup):
    """eval.py:646-661 (same file per table, same order)."""
    path_res = Path(path_res)
    path_res.mkdir(parents=True, exist_ok=True)
    tables = dict(mean_errors=mean_errors, final_errors=final_errors, init_errors=init_errors,
                  var_errors=var_errors, mean_solved=mean_solved, params=params, exp_setup=exp_setup)
    for key, name in POSE_FILES.items():
        _dump(path_res / name, tables[key])


def image_grid(images, title, rows=None, cols=None, fill=True, show_axes=False, rgb=True):
    """eval.py:787-821: a rows x cols grid of (H, W, 4) images saved as
    `<title>/grid_cube.png` (eval.py resolves `cwd/'results'/title`; an absolute `title`,
    as optimize_pose passes, is used as is).  Returns the file path."""
    if (rows is None) != (cols is None):
        raise ValueError("Specify either both rows and cols or neither.")
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    if rows is None:
        rows, cols = len(images), 1
    gridspec_kw = {"wspace": 0.0, "hspace": 0.0} if fill else {}
    fig, axarr = plt.subplots(rows, cols, gridspec_kw=gridspec_kw, figsize=(15, 9), squeeze=False)
    fig.subplots_adjust(left=0, bottom=0, right=1, top=1)
    for ax, im in zip(axarr.ravel(), images):
        if rgb:
            im = np.array(im, copy=True)
            im[..., :3] = np.clip(im[..., :3], 0.0, 1.0)
            ax.imshow(im[..., :3])
        else:
            ax.imshow(im[..., 3])
        if not show_axes:
            ax.set_axis_off()
    out = Path().cwd() / "results" / title
    out.mkdir(parents=True, exist_ok=True)
    fig.savefig(out / "grid_cube.png", bbox_inches="tight")
    plt.close(fig)
    return out / "grid_cube.png"


def write_optimization_details(path_fig, loss_values, gradient_values, images=None, datenow=None):
    """eval.py:398-405: `optimization_details/<date>/{loss_values,gradient_values}.npy` and
    the grid of training images (rows=4, cols=1+len//4).  Returns the detail directory."""
    datenow = datenow or datetime.now().strftime(DATE_FORMAT)
    d = Path(path_fig) / DETAIL_DIR / datenow
    d.mkdir(parents=True, exist_ok=True)
    np.save(d / "loss_values.npy", loss_values)
    np.save(d / "gradient_values.npy", gradient_values)
    if images is not None and len(images):
        images = images.detach().cpu().numpy() if hasattr(images, "detach") else np.asarray(images)
        image_grid(images, rows=4, cols=1 + images.shape[0] // 4, rgb=True, title=d.resolve())
    return d


def read_results(path_res):
    """Every eval.py table present in `path_res` -> {key: parsed JSON}."""
    path_res = Path(path_res)
    out = {}
    for key, name in {**RUNTIME_FILES, **POSE_FILES}.items():
        f = path_res / name
        if f.exists():
            with open(f) as fh:
                out[key] = json.load(fh)
    return out


def read_optimization_details(detail_dir):
    d = Path(detail_dir)
    return {name: np.load(d / f"{name}.npy") for name in ("loss_values", "gradient_values")
            if (d / f"{name}.npy").exists()}


def compare_pose_results(a, b):
    """Two runs' pose tables (dicts from read_results, e.g. GPU vs CPU of the same seeds)
    -> {noise_type: {"mean_error_diff": [...], "max_abs_mean_error_diff": x,
    "solved_diff": {thresh: [...]}, "max_abs_solved_diff": y}} over the noise types and
    settings both hold."""
    rep = {}
    ea, eb = a.get("mean_errors", {}), b.get("mean_errors", {})
    sa, sb = a.get("mean_solved", {}), b.get("mean_solved", {})
    for nt in sorted(set(ea) & set(eb)):
        n = min(len(ea[nt]), len(eb[nt]))
        de = [float(eb[nt][i]) - float(ea[nt][i]) for i in range(n)]
        r = {"mean_error_diff": de, "max_abs_mean_error_diff": max((abs(x) for x in de), default=0.0)}
        sd = {}
        for th in sorted(set(sa.get(nt, {})) & set(sb.get(nt, {})), key=float):
            m = min(len(sa[nt][th]), len(sb[nt][th]))
            sd[th] = [float(sb[nt][th][i]) - float(sa[nt][th][i]) for i in range(m)]
        r["solved_diff"] = sd
        r["max_abs_solved_diff"] = max((abs(x) for v in sd.values() for x in v), default=0.0)
        rep[nt] = r
    return rep


def main(argv=None):
    """python -m pertrenderer_amd.results RUN_A RUN_B: print the pose-table comparison."""
    import argparse
    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("run_a")
    ap.add_argument("run_b")
    args = ap.parse_args(argv)
    rep = compare_pose_results(read_results(args.run_a), read_results(args.run_b))
    print(json.dumps(rep, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
