"""BASELINE cfg5 driver (pertrenderer_amd/pose_opt.py, mirroring eval.py:320-409, 576-690) at
reduced size: the pose optimisation converges towards the true pose for both of eval.py's
default renderers ("softras", "gaussian"), eagerly and as captured graphs, and the result
tables have the reference's json layout.  The full run (100 problems x 800 iterations at 256^2)
is profiles/r2_cfg5.json."""
import json

import numpy as np
import pytest
import torch

from pertrenderer_amd import pose_opt
from pertrenderer_amd.results import compare_pose_results

pytestmark = pytest.mark.gpu
NOISE = ("softras", "gaussian")


@pytest.fixture(scope="module")
def problems(device):
    torch.manual_seed(0)
    scene = pose_opt.Scene(device, 128)
    return scene, pose_opt.make_problems(scene, 3, NOISE, 20.0)


@pytest.mark.parametrize("mode", ["graph", "eager"])
def test_pose_optimisation_converges(problems, mode):
    scene, probs = problems
    torch.manual_seed(1)
    niter = 200 if mode == "graph" else 120
    per = [pose_opt.run_problem(scene, p, NOISE, 1e-3, 1e-2, 8, 20.0, niter, True, (1.1, 1.1), mode) for p in probs]
    for nt in NOISE:
        init = np.array([r[nt]["init_error"] for r in per])
        final = np.array([r[nt]["final_error"] for r in per])
        print(mode, nt, "init", init.round(2), "final", final.round(2))
        assert np.all(np.isfinite(final))
        assert np.allclose(init, 20.0, atol=1e-3)  # pert_init_intensity: a 20 degree rotation
        assert final.mean() < 0.6 * init.mean(), (nt, final)
        assert (final < init).sum() >= 2, (nt, final)
    tab = pose_opt.tables(per, NOISE, dict(niter=niter), dict(mode=mode))
    json.dumps(tab)  # eval.py writes these tables with json.dump
    assert set(tab["mean_solved"]["gaussian"]) == set(pose_opt.THRESHOLDS)


def test_graph_and_eager_runs_compare(problems):
    """results.compare_pose_results over two runs of the same problems: per-problem error
    differences are reported for every noise type."""
    scene, probs = problems
    runs = []
    for mode in ("graph", "eager"):
        torch.manual_seed(2)
        per = [pose_opt.run_problem(scene, p, NOISE, 1e-3, 1e-2, 8, 20.0, 60, False, (1.1, 1.1), mode)
               for p in probs[:2]]
        runs.append(pose_opt.tables(per, NOISE, dict(niter=60), dict(mode=mode)))
    cmp = compare_pose_results(runs[0], runs[1])
    assert set(NOISE) <= set(cmp)


@pytest.mark.parametrize("mode", ["eager", "graph"])
def test_compare_runtime_tables(tmp_path, device, mode):
    """eval.py compare_runtime (:506-574) mirror: per (lr, smoothing, MC) setting and problem, the
    wall time of a whole optimize_pose run and its peak device memory, written as runtimes.txt /
    memory.txt with the reference's {noise: [[per problem] per setting]} layout."""
    torch.manual_seed(2)
    scene = pose_opt.Scene(device, 64)
    rt, mem, params = pose_opt.compare_runtime(scene, 2, list(NOISE), [(1e-3, 1e-2)], [4, 8], niter=12,
                                               mode=mode, out=str(tmp_path))
    for table in (rt, mem):
        assert set(table) == set(NOISE)
        for nt in NOISE:
            assert len(table[nt]) == 2 and all(len(per) == 2 for per in table[nt])
            assert all(v > 0 for per in table[nt] for v in per)
    assert params["MC"] == [4, 8] and params["lr-smoothing-MC"] == [(5e-2, 1e-3, 1e-2, 4), (5e-2, 1e-3, 1e-2, 8)]
    on_disk = json.load(open(tmp_path / "runtimes.txt")), json.load(open(tmp_path / "memory.txt"))
    assert on_disk[0] == rt and on_disk[1] == mem


def test_cfg5_full_size_graph_runs(device):
    """BASELINE cfg 5 at its size: eval.py's pose benchmark (compare_pose_opt's problems,
    optimize_pose with the adaptive schedule, eval.py:320-409, 576-690) at 256 x 256 for the full
    800 iterations, graph mode, both default renderers, 2 problems: every run improves on its
    20-degree start and the tables have the reference's layout (the 100-problem run is
    profiles/r2_cfg5.json)."""
    torch.manual_seed(0)
    scene = pose_opt.Scene(device, 256)
    probs = pose_opt.make_problems(scene, 2, NOISE, 20.0)
    torch.manual_seed(1)
    per = [pose_opt.run_problem(scene, p, NOISE, 1e-3, 1e-2, 8, 20.0, 800, True, (1.1, 1.1), "graph")
           for p in probs]
    for nt in NOISE:
        init = np.array([r[nt]["init_error"] for r in per])
        final = np.array([r[nt]["final_error"] for r in per])
        print("cfg5", nt, "init", init.round(2), "final", final.round(3),
              "S", [r[nt]["final_nb_samples"] for r in per], "s", [round(r[nt]["seconds"], 2) for r in per])
        assert np.allclose(init, 20.0, atol=1e-3)
        assert np.all(np.isfinite(final)) and np.all(final < init), (nt, final)
        assert all(r[nt]["iterations"] == 800 for r in per)
    tab = pose_opt.tables(per, NOISE, dict(niter=800), dict(mode="graph"))
    json.dumps(tab)
    assert set(tab["mean_solved"]["gaussian"]) == set(pose_opt.THRESHOLDS)
    assert set(tab["mean_errors"]) == set(NOISE)


def test_graph_session_replays_captured_iterations(device, monkeypatch):
    """compare_pose_opt's driver keeps one GraphSession per noise type: the second problem resets
    the session's tensors to its own start and replays the iterations the first one captured (no
    capture at a sample count already seen), and still optimises its pose."""
    torch.manual_seed(3)
    scene = pose_opt.Scene(device, 64)
    probs = pose_opt.make_problems(scene, 2, ["gaussian"], 20.0)
    count = []
    init0 = pose_opt._CapturedIteration.__init__

    def counting(self, *a, **k):
        count.append(1)
        init0(self, *a, **k)

    monkeypatch.setattr(pose_opt._CapturedIteration, "__init__", counting)
    sessions = {}
    per = []
    for p in probs:
        before = len(count)
        per.append((pose_opt.run_problem(scene, p, ["gaussian"], 1e-3, 1e-2, 8, 20.0, 300, True, (1.1, 1.1), "graph",
                                         sessions=sessions), len(count) - before))
    (r1, c1), (r2, c2) = per
    assert c1 >= 2 and c2 < c1, (c1, c2)
    for r in (r1, r2):
        assert np.isfinite(r["gaussian"]["final_error"]) and r["gaussian"]["final_error"] < r["gaussian"]["init_error"]


@pytest.mark.parametrize("noise_type", ["softras", "gaussian"])
def test_kept_graphs_record_each_problems_losses(device, noise_type):
    """A kept (GraphSession) graph replayed for a later problem -- after the eager work between
    compare_pose_opt's problems (init_renderers' bmm, angle_deg) and host synchronisations -- records
    that problem's own losses, gradient norms, best pose and smoothing EMA: the same as a fresh capture
    of it (softras: the first iterations to 1e-4, the best pose within 0.5 deg; gaussian, whose noise
    keys differ between the two drivers: the same statistics).  (With torch's one-pass frame mean in
    the captured step, the reused graphs recorded the first problem's last loss at every iteration:
    pose_opt._CapturedIteration._forward)"""
    torch.manual_seed(1)
    scene = pose_opt.Scene(device, 256)  # a whole 256^2 frame: torch's mean reduces it across workgroups
    probs = pose_opt.make_problems(scene, 2, ["softras", "gaussian"], 20.0)
    res = {}
    for use in (False, True):
        kept = pose_opt.GraphSession() if use else None
        for i, (target_rgb, R_true, log_rot_init) in enumerate(probs):
            _, rs = pose_opt.init_renderers(scene, R_true, noise_type=[noise_type])
            torch.cuda.synchronize()
            ses = kept if use else pose_opt.GraphSession()
            best, info = pose_opt.optimize_pose_graph(scene, log_rot_init, rs[0], target_rgb, Niter=800, session=ses)
            torch.cuda.synchronize()
            res[(use, i)] = dict(loss=np.asarray(info["loss_values"]), gnorm=np.asarray(info["gradient_values"]),
                                 angle=pose_opt.angle_deg(best, R_true), v=ses.st["v"].detach().cpu().numpy().copy(),
                                 best_loss=float(ses.st["best_loss"]), nb=info["nb_samples"])
    fresh, kept = res[(False, 1)], res[(True, 1)]
    for r in (fresh, kept):  # a live trace whose best is its own minimum
        assert len(np.unique(r["loss"][:100].round(9))) > 10, r["loss"][:5]
        assert len(np.unique(r["gnorm"][:100].round(9))) > 10, r["gnorm"][:5]
        assert r["best_loss"] <= r["loss"].min() * (1 + 1e-6)
    assert kept["nb"] == fresh["nb"]
    if noise_type == "softras":
        np.testing.assert_allclose(kept["loss"][:20], fresh["loss"][:20], rtol=1e-4)
        # gradient norms: the backward's float-atomic sums differ run to run (~1e-4 relative on the
        # small norms); a stale replay would differ by O(1)
        np.testing.assert_allclose(kept["gnorm"][:20], fresh["gnorm"][:20], rtol=1e-3)
        assert abs(kept["loss"][:100].mean() - fresh["loss"][:100].mean()) < 1e-3 * fresh["loss"][:100].mean()
        assert abs(kept["angle"] - fresh["angle"]) < 0.5, (kept["angle"], fresh["angle"])
        np.testing.assert_allclose(kept["v"], fresh["v"], rtol=2e-2, atol=1e-9)
    else:
        assert abs(kept["loss"][:100].mean() - fresh["loss"][:100].mean()) < 0.1 * fresh["loss"][:100].mean()
        assert abs(kept["gnorm"][:100].mean() - fresh["gnorm"][:100].mean()) < 0.25 * fresh["gnorm"][:100].mean()
        assert abs(kept["angle"] - fresh["angle"]) < 10.0, (kept["angle"], fresh["angle"])


def test_captured_step_has_no_torch_cross_workgroup_reduction(device, tmp_path):
    """the kept-graph hazard (a torch one-pass cross-workgroup reduction in a kept graph
    goes stale after eager BLAS between replays) is avoided by construction: the captured pose
    iteration of both eval.py renderers launches no at::native::reduce_kernel (its loss is
    pr_rgb_mse_*, its bookkeeping pr_pose_step).  The iteration's body is run eagerly under the
    profiler (the graph records the same launches)."""
    import json
    from torch.profiler import ProfilerActivity, profile
    torch.manual_seed(1)
    scene = pose_opt.Scene(device, 128)
    target_rgb, R_true, log_rot_init = pose_opt.make_problems(scene, 1, ["softras", "gaussian"], 20.0)[0]
    for noise_type in ("softras", "gaussian"):
        _, rs = pose_opt.init_renderers(scene, R_true, noise_type=[noise_type])
        ses = pose_opt.GraphSession()
        ses.bind(scene, log_rot_init, rs[0], target_rgb, 5e-2, 800)
        it = ses.step(True)
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            it._body()
            torch.cuda.synchronize()
        tr = str(tmp_path / f"{noise_type}.json")
        prof.export_chrome_trace(tr)
        names = [e.get("name", "") for e in json.load(open(tr))["traceEvents"]
                 if e.get("ph") == "X" and e.get("cat") == "kernel"]
        assert any("rast_fwd" in n for n in names) and any("pose_step" in n for n in names), names
        assert not any("reduce_kernel" in n for n in names), [n for n in names if "reduce_kernel" in n]
        from pertrenderer_amd import noise
        noise.use_device_seed(None)


@pytest.mark.parametrize("shape,tshape", [((1, 256, 256, 4), (256, 256, 3)), ((2, 33, 17, 4), (2, 33, 17, 3)),
                                          ((3, 8, 8, 3), (8, 8, 3))])
def test_native_rgb_loss_matches_torch(device, shape, tshape):
    """The captured step's loss (pose_opt._RgbMse, pr_rgb_mse_fwd / _bwd) against eval.py:352-353's
    torch expression: value and image gradient at 1e-6 relative (fp32 summation order only)."""
    torch.manual_seed(5)
    img = torch.rand(shape, device=device, requires_grad=True)
    t = torch.rand(tshape, device=device)
    ref = ((img[..., :3] - t) ** 2).mean()
    (gref,) = torch.autograd.grad(ref * 3.0, img)
    out = pose_opt._RgbMse.apply(img, t)
    (g,) = torch.autograd.grad(out * 3.0, img)
    assert abs(float(out) - float(ref)) <= 1e-6 * abs(float(ref))
    torch.testing.assert_close(g, gref, rtol=1e-6, atol=1e-9)
    if shape[-1] > 3:
        assert float(g[..., 3:].abs().max()) == 0.0


def test_rgb_mse_target_gradient_not_dropped(device):
    """pose_opt.rgb_mse with a target that requires grad: both gradients match eval.py's torch
    expression (the native nodes differentiate the images only, so such a call takes torch's)."""
    torch.manual_seed(6)
    img = torch.rand((2, 9, 7, 4), device=device, requires_grad=True)
    t = torch.rand((9, 7, 3), device=device, requires_grad=True)
    gi, gt = torch.autograd.grad(pose_opt.rgb_mse(img, t), (img, t))
    ri, rt = torch.autograd.grad(((img[..., :3] - t) ** 2).mean(), (img, t))
    torch.testing.assert_close(gi, ri)
    torch.testing.assert_close(gt, rt)
    assert float(gt.abs().max()) > 0


def test_pose_step_kernel_bookkeeping(device):
    """pr_pose_step (the captured step's bookkeeping) against eval.py:356-358, 372-385 restated in
    torch: records, best-loss pose, the grad-norm guard, the smoothing gradients' running sum and
    (post) EMA, the counter."""
    from pertrenderer_amd import _native as nat
    f32 = dict(dtype=torch.float32, device=device)
    st = dict(it=torch.tensor(4, dtype=torch.int64, device=device), losses=torch.zeros(8, **f32),
              gnorms=torch.zeros(8, **f32), best_loss=torch.tensor(0.5, **f32), best=torch.zeros(1, 3, **f32),
              v=torch.tensor([0.1, -0.2, 0.3], **f32), acc=torch.tensor([1.0, 2.0, 3.0], **f32))
    seed = torch.tensor([12345], dtype=torch.int64, device=device)

    def run(loss, log_rot, grad, leaf, post):
        a = nat.PRPoseStepArgs()
        a.loss, a.log_rot, a.grad, a.it = nat.ptr(loss), nat.ptr(log_rot), nat.ptr(grad), nat.ptr(st["it"])
        a.losses, a.gnorms, a.best_loss, a.best = (nat.ptr(st[k]) for k in ("losses", "gnorms", "best_loss", "best"))
        a.v, a.acc, a.seed = nat.ptr(st["v"]), nat.ptr(st["acc"]), nat.ptr(seed)
        for i in range(3):
            a.leaf_grad[i] = nat.ptr(leaf[i])
        a.niter, a.n, a.post = 8, 3, int(post)
        nat.call("pr_pose_step", "pose_step", loss, a)
        torch.cuda.synchronize()

    log_rot = torch.tensor([[0.1, 0.2, 0.3]], **f32)
    grad = torch.tensor([[3.0, 4.0, 0.0]], **f32)
    leaf = [torch.tensor(x, **f32) for x in (0.5, -1.0, 2.0)]
    run(torch.tensor(0.25, **f32), log_rot, grad, leaf, post=False)  # better loss, small grad, pre-phase
    assert int(st["it"]) == 5 and float(st["losses"][4]) == 0.25 and float(st["gnorms"][4]) == 5.0
    assert float(st["best_loss"]) == 0.25 and torch.equal(st["best"], log_rot)
    assert torch.equal(grad, torch.tensor([[3.0, 4.0, 0.0]], **f32))
    assert torch.equal(st["acc"], torch.tensor([1.5, 1.0, 5.0], **f32))
    assert torch.equal(st["v"], torch.tensor([0.1, -0.2, 0.3], **f32))
    big = torch.tensor([[3000.0, 0.0, 0.0]], **f32)
    run(torch.tensor(0.75, **f32), log_rot * 2, big, leaf, post=True)  # worse loss, guard, post-phase EMA
    assert int(st["it"]) == 6 and float(st["losses"][5]) == 0.75 and float(st["gnorms"][5]) == 3000.0
    assert float(st["best_loss"]) == 0.25 and torch.equal(st["best"], log_rot)
    assert 0.0 < float(big.norm()) < 1e-3  # eval.py:375-379: 1e-5 * normal draws
    acc = torch.tensor([1.5, 1.0, 5.0], **f32) + torch.stack(leaf)
    ema = torch.tensor([0.1, -0.2, 0.3], **f32) * 0.9 + 0.1 * acc
    torch.testing.assert_close(st["v"], ema, rtol=0, atol=0)
    assert float(st["acc"].abs().max()) == 0.0


def test_pose_step_adam_matches_torch_adam(device):
    """pr_pose_step's Adam update against torch.optim.Adam (fused, capturable, tensor lr) over a few
    steps on the same gradients: parameters and state at 1e-6."""
    from pertrenderer_amd import _native as nat
    f32 = dict(dtype=torch.float32, device=device)
    torch.manual_seed(7)
    ref = torch.randn(1, 3, **f32).requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=torch.tensor(5e-2, **f32), capturable=True, fused=True)
    mine = ref.detach().clone()
    m, s2, step = torch.zeros(1, 3, **f32), torch.zeros(1, 3, **f32), torch.zeros((), **f32)
    lr = torch.tensor(5e-2, **f32)
    st = dict(it=torch.zeros((), dtype=torch.int64, device=device), losses=torch.zeros(8, **f32),
              gnorms=torch.zeros(8, **f32), best_loss=torch.tensor(float("inf"), **f32), best=torch.zeros(1, 3, **f32))
    for k in range(5):
        g = torch.randn(1, 3, **f32)
        ref.grad = g.clone()
        opt.step()
        gm = g.clone()
        a = nat.PRPoseStepArgs()
        loss = torch.tensor(1.0, **f32)
        a.loss, a.log_rot, a.grad, a.it = nat.ptr(loss), nat.ptr(mine), nat.ptr(gm), nat.ptr(st["it"])
        a.losses, a.gnorms, a.best_loss, a.best = (nat.ptr(st[q]) for q in ("losses", "gnorms", "best_loss", "best"))
        a.exp_avg, a.exp_avg_sq, a.step, a.lr, a.adam = nat.ptr(m), nat.ptr(s2), nat.ptr(step), nat.ptr(lr), 1
        a.niter, a.n, a.post = 8, 3, 0
        nat.call("pr_pose_step", "pose_step", loss, a)
    torch.cuda.synchronize()
    ost = opt.state[ref]
    torch.testing.assert_close(mine, ref.detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(m, ost["exp_avg"], rtol=1e-6, atol=1e-8)
    torch.testing.assert_close(s2, ost["exp_avg_sq"], rtol=1e-6, atol=1e-10)
    assert float(step) == float(ost["step"]) == 5.0
