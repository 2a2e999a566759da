"""Deterministic-order mode (SURVEY.md §5 "race detection"; torch.use_deterministic_algorithms).

The fast backward passes scatter into per-face / per-vertex sums with float atomics, whose order
varies run to run.  With torch's deterministic switch on, the library forms those sums by a stable
sort of the contributions and in-order sums (PR_DETERMINISTIC, pr_detsum.hip):
  * pr_rast_bwd sums each face's slot gradients in slot order with the oracle's slot arithmetic:
    bit for bit the C oracle (PyTorch3D's CPU backward order) on every configuration;
  * pr_shade_bwd's vertex / light / camera / texture-map gradients are in-order sums;
  * the projection backward and the vertex normals gather per vertex over the topology's corner
    index in every mode (no atomics).
Checked: bitwise oracle equality, bitwise run-to-run equality of whole pose-optimisation runs in
graph mode, and agreement of the deterministic and fast paths at the 1e-5 bar."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, assert_close
from oracle import rast_ref
from pertrenderer_amd.renderer import Meshes, load_obj
from pertrenderer_amd.renderer.rasterizer import _rasterize

pytestmark = pytest.mark.gpu


@pytest.fixture
def deterministic():
    old = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True)
    yield
    torch.use_deterministic_algorithms(old)


def _soup(F, seed, zmin=0.5, spread=1.2, size=0.4):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-spread, spread, (F, 1, 2))
    xy = c + rng.uniform(-size, size, (F, 3, 2))
    z = rng.uniform(zmin, 5.0, (F, 3, 1))
    fv = np.concatenate([xy, z], -1).astype(np.float32)
    fv[: F // 10, :, 2] -= 6.0
    return fv


def _rast_grad(fv, first, nf, H, K, blur, persp, clip, seed, device):
    fvt = torch.tensor(fv, device=device, requires_grad=True)
    p2f, zbuf, bary, dists = _rasterize(fvt, torch.tensor(first, device=device), torch.tensor(nf, device=device),
                                        H, H, K, blur, persp, clip, False)
    g = np.random.default_rng(seed)
    gz = g.standard_normal(zbuf.shape).astype(np.float32)
    gb = g.standard_normal(bary.shape).astype(np.float32)
    gd = g.standard_normal(dists.shape).astype(np.float32)
    T = lambda a: torch.tensor(a, device=device)
    (got,) = torch.autograd.grad((zbuf * T(gz)).sum() + (bary * T(gb)).sum() + (dists * T(gd)).sum(), fvt)
    return got.cpu().numpy(), p2f.cpu().numpy(), gz, gb, gd


@pytest.mark.parametrize("persp,clip", [(False, False), (False, True), (True, True)])
@pytest.mark.parametrize("F,H,K,size", [(120, 32, 10, 0.4), (400, 16, 50, 0.5), (900, 20, 120, 0.9)])
def test_rasterizer_backward_is_oracle_bitwise(F, H, K, size, persp, clip, device, deterministic):
    """Two meshes; the dense cases hold tiles with > 1024 valid slots and > 128 faces (the fast
    path's global-atomic overflow), so every fast-path branch has a deterministic twin here."""
    fv = np.concatenate([_soup(F, 11, spread=0.6, size=size), _soup(F // 2, 12, spread=0.6, size=size)])
    first, nf = np.array([0, F]), np.array([F, F // 2])
    got, p2f, gz, gb, gd = _rast_grad(fv, first, nf, H, K, 2e-2, persp, clip, 4, device)
    assert (p2f >= 0).sum() > 100
    ref = rast_ref.rast_bwd(fv, p2f, gz, gb, gd, persp, clip)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("persp,clip", [(False, False), (False, True), (True, True)])
def test_fast_rasterizer_backward_matches_deterministic(persp, clip, device):
    """The default (tile-reduced, float atomics) backward against the deterministic one at the 1e-5
    bar: they differ only in the order of each face's sum."""
    fv = _soup(400, 3, spread=0.6, size=0.5)
    args = (fv, np.array([0]), np.array([400]), 24, 50, 2e-2, persp, clip, 7, device)
    fast = _rast_grad(*args)[0]
    torch.use_deterministic_algorithms(True)
    try:
        det = _rast_grad(*args)[0]
    finally:
        torch.use_deterministic_algorithms(False)
    assert_close(fast, det, name="d face_verts")


def _eval_frame_grads(device, seed=5, size=96):
    """eval.py's renderer (RandomPhongShader, TexturesUV cube, Philox noise) on one frame: d log_rot,
    d verts, d light location and d texture map."""
    from pertrenderer_amd import pose_opt
    from pertrenderer_amd.renderer import Rotate, so3_exponential_map
    torch.manual_seed(0)
    scene = pose_opt.Scene(device, size)
    target, R_true = scene.target()
    _, (renderer,) = pose_opt.init_renderers(scene, R_true, sigma=1e-3, gamma=1e-2, nb_samples=8,
                                             noise_type=("gaussian",))
    log_rot = pose_opt.so3_log_map(R_true @ so3_exponential_map(torch.tensor([[0.2, -0.15, 0.1]], device=device)))
    log_rot = log_rot.detach().requires_grad_(True)
    tex = scene.meshes.textures
    maps = tex._maps[0].detach().clone().requires_grad_(True)
    tex._maps = [maps]
    light = scene.lights.location.detach().clone().requires_grad_(True)
    scene.lights.location = light
    torch.manual_seed(seed)
    verts = Rotate(so3_exponential_map(log_rot)).transform_points(scene.meshes.verts_padded())
    verts.retain_grad()
    img = renderer(scene.meshes.update_padded(verts), cameras=scene.cameras[0], lights=scene.lights)
    ((img[..., :3] - target[0]) ** 2).mean().backward()
    torch.cuda.synchronize()
    return [t.detach().clone() for t in (img, log_rot.grad, verts.grad, light.grad, maps.grad)]


def test_eval_frame_gradients_bitwise_reproducible(device, deterministic):
    a = _eval_frame_grads(device)
    b = _eval_frame_grads(device)
    for name, x, y in zip(("image", "d log_rot", "d verts", "d light", "d maps"), a, b):
        assert x is not None and torch.equal(x, y), name
    assert float(a[1].abs().sum()) > 0 and float(a[4].abs().sum()) > 0


def test_eval_frame_fast_matches_deterministic(device):
    fast = _eval_frame_grads(device)
    torch.use_deterministic_algorithms(True)
    try:
        det = _eval_frame_grads(device)
    finally:
        torch.use_deterministic_algorithms(False)
    assert torch.equal(fast[0], det[0])  # the forward has no atomics
    for name, x, y in zip(("d log_rot", "d verts", "d light", "d maps"), fast[1:], det[1:]):
        assert_close(x, y, name=name)


def test_graph_mode_pose_run_bitwise_reproducible(device, deterministic):
    """eval.py's optimize_pose as captured graphs (pose_opt.optimize_pose_graph, Philox noise,
    adaptive schedule) run twice from the same seed: identical losses and pose, bit for bit."""
    from pertrenderer_amd import pose_opt
    torch.manual_seed(0)
    scene = pose_opt.Scene(device, 64)
    (problem,) = pose_opt.make_problems(scene, 1, ("gaussian",), 20.0)
    runs = []
    for _ in range(2):
        target_rgb, R_true, log_rot_init = problem
        torch.manual_seed(3)
        _, (renderer,) = pose_opt.init_renderers(scene, R_true, sigma=1e-3, gamma=1e-2, nb_samples=8,
                                                 noise_type=("gaussian",))
        best, info = pose_opt.optimize_pose_graph(scene, log_rot_init, renderer, target_rgb, Niter=160)
        runs.append((best.cpu(), info["loss_values"], info["gradient_values"]))
    assert torch.equal(runs[0][0], runs[1][0])
    assert runs[0][1] == runs[1][1] and runs[0][2] == runs[1][2]


def test_projection_gather_matches_atomic_scatter(device):
    """pr_project_bwd over the corner index (every mode) against its float-atomic form."""
    from pertrenderer_amd.renderer import FoVPerspectiveCameras, look_at_view_transform
    from pertrenderer_amd.renderer.project import project_faces
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    mesh = Meshes([verts.to(device)], [faces.verts_idx.to(device)])
    R, T = look_at_view_transform(2.7, 30.0, 120.0, device=device)
    cams = FoVPerspectiveCameras(R=R, T=T, device=device)
    out = []
    for csr in (mesh.corner_csr(), None):
        v = mesh.verts_packed().detach().clone().requires_grad_(True)
        fv = project_faces(v, mesh.faces_packed(), mesh.mesh_to_faces_packed_first_idx(), mesh.num_faces_per_mesh(),
                           cams.world_to_view_matrix(), cams.projection_matrix(), csr=csr)
        g = torch.randn(fv.shape, generator=torch.Generator().manual_seed(1)).to(device)
        out.append(torch.autograd.grad((fv * g).sum(), v)[0])
    assert_close(out[0], out[1], name="d verts")


def test_normals_gather_matches_atomic_scatter(device):
    """Vertex normals over the corner index (PyTorch3D's accumulation order) against the one-thread-
    per-face atomic form: forward and backward."""
    from pertrenderer_amd.renderer.mesh import _VertNormalsFn
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", "sphere_642.obj"))
    mesh = Meshes([(verts * torch.tensor([1.0, 0.7, 1.3])).to(device)], [faces.verts_idx.to(device)])
    out = []
    for csr in (mesh.corner_csr("normals"), (None, None)):
        v = mesh.verts_packed().detach().clone().requires_grad_(True)
        n = _VertNormalsFn.apply(v, mesh.faces_packed(), *csr)
        g = torch.randn(n.shape, generator=torch.Generator().manual_seed(2)).to(device)
        out.append((n.detach(), torch.autograd.grad((n * g).sum(), v)[0]))
    assert_close(out[0][0], out[1][0], name="normals")
    assert_close(out[0][1], out[1][1], name="d verts")


@pytest.fixture
def small_batches():
    """PR_DET_BATCH: the deterministic scatters run in batches of this many entries (default 2^24,
    which bounds their workspace at cfg 4's 629 M slots); small batches drive the batched path on
    small frames."""
    old = os.environ.get("PR_DET_BATCH")
    os.environ["PR_DET_BATCH"] = "1000"
    yield
    if old is None:
        os.environ.pop("PR_DET_BATCH", None)
    else:
        os.environ["PR_DET_BATCH"] = old


@pytest.mark.parametrize("persp,clip", [(False, True), (True, True)])
def test_batched_rasterizer_backward_is_oracle_bitwise(persp, clip, device, deterministic, small_batches):
    """Batches of 1000 slots whose face sums continue each face's chain (detsum_reduce_chain): still
    bit for bit the oracle's single serial loop."""
    fv = np.concatenate([_soup(400, 11, spread=0.6, size=0.5), _soup(200, 12, spread=0.6, size=0.5)])
    first, nf = np.array([0, 400]), np.array([400, 200])
    got, p2f, gz, gb, gd = _rast_grad(fv, first, nf, 20, 50, 2e-2, persp, clip, 4, device)
    assert p2f.size > 10 * 1000 and (p2f >= 0).sum() > 1000
    np.testing.assert_array_equal(got, rast_ref.rast_bwd(fv, p2f, gz, gb, gd, persp, clip))


def test_batched_eval_frame_reproducible_and_close(device, deterministic, small_batches):
    """Shading's deterministic scatters in batches (each batch's ordered sums added to the previous
    ones): bitwise reproducible, and the unbatched deterministic path's values at the 1e-5 bar."""
    a = _eval_frame_grads(device, size=48)
    b = _eval_frame_grads(device, size=48)
    for name, x, y in zip(("image", "d log_rot", "d verts", "d light", "d maps"), a, b):
        assert torch.equal(x, y), name
    os.environ["PR_DET_BATCH"] = str(1 << 24)
    c = _eval_frame_grads(device, size=48)
    for name, x, y in zip(("d log_rot", "d verts", "d light", "d maps"), a[1:], c[1:]):
        assert_close(x, y, name=name)


def test_deterministic_workspace_is_bounded():
    """The workspace of the deterministic rasterizer backward at cfg 4 (16 x 512^2 x K 150: 629 M
    slots) is one batch's, not the frame's (~55 GB unbatched)."""
    from pertrenderer_amd import _native as nat
    a = nat.PRRastArgs()
    a.N, a.H, a.W, a.K, a.F = 16, 512, 512, 150, 20000
    a.flags = nat.PR_DETERMINISTIC
    assert nat.load().pr_rast_bwd_workspace_size(nat.C.byref(a)) < 3 * 2**30
