"""Parity of the bench's headline frame (BASELINE cfg 2) at its full size.

bench.Workload's exact frame -- sphere_642, 256x256, faces_per_pixel=50, GaussianRast +
GaussianAgg with Sr = Sa = 8, sigma 1e-3, gamma 1e-2, blur = ln(1e4 - 1) sigma, RandomSimpleShader
with fused TexturesVertex sampling, L2 loss to the bench's target -- rendered on the GPU with the
reference's own noise draws (set_noise_source("torch"): torch.randn (Sr,N,H,W,K) then
(Sa,N,H,W,K+1) on the CPU generator, smoothrast.py:21 then smoothagg.py:21) and by the CPU
oracle composition (oracle/pipeline_ref.py: C rasterizer oracle, torch interpolation, blend
oracle) fed the same draws.  Compared (random_rasterizer.py:34-56, eval.py:343-370):
  * fragments: bit for bit;
  * image, loss, d dists, d zbuf, d bary: conftest.assert_close (1e-5 relative);
  * d verts and d log_rot: 1e-5 relative, with torch.use_deterministic_algorithms (the
    rasterizer backward then sums each face's slot gradients in the oracle's slot order).
The oracle side's projection and rotation run torch's CPU transforms; their outputs are pinned
to the GPU's values (straight-through), so both sides rasterize the same bits and the gradients
flow through torch's Jacobians on the CPU side.
"""
import math

import numpy as np
import pytest
import torch

import pertrenderer_amd as pa
from conftest import assert_close
from oracle import pipeline_ref
from pertrenderer_amd.renderer import Rotate, so3_exponential_map
from pertrenderer_amd.renderer.project import project_faces

pytestmark = pytest.mark.gpu


def _straight(cpu_value, gpu_value):
    """cpu_value's autograd graph with gpu_value's bits."""
    return cpu_value + (gpu_value.detach().cpu() - cpu_value).detach()


def headline_frame(device, deterministic=True, seed=3):
    import bench
    old_src, old_det = pa.noise.get_noise_source(), torch.are_deterministic_algorithms_enabled()
    pa.set_noise_source("torch")
    torch.use_deterministic_algorithms(deterministic)
    try:
        wl = bench.Workload(device, **{k: v for k, v in bench.CONFIGS["cfg2"].items() if k != "batch"})
        H, K, S = wl.H, wl.K, wl.S
        # ---- GPU: the bench's forward with the intermediate gradients kept
        log_rot = wl.log_rot.detach().clone().requires_grad_(True)
        R = so3_exponential_map(log_rot)
        verts = Rotate(R).transform_points(wl.base.verts_padded())
        verts.retain_grad()
        mesh = wl.base.update_padded(verts)
        frag = wl.renderer.rasterizer(mesh, cameras=wl.cameras)
        for t in (frag.dists, frag.zbuf, frag.bary_coords):
            t.retain_grad()
        torch.manual_seed(seed)
        img = wl.renderer.shader(frag, mesh, cameras=wl.cameras)
        loss = ((img[..., :3] - wl.target) ** 2).mean()
        loss.backward()
        torch.cuda.synchronize()
        fv_gpu = project_faces(verts.detach()[0], mesh.faces_packed(), mesh.mesh_to_faces_packed_first_idx(),
                               mesh.num_faces_per_mesh(), wl.cameras.world_to_view_matrix(),
                               wl.cameras.projection_matrix())
        gpu = dict(fv=fv_gpu, p2f=frag.pix_to_face, zbuf=frag.zbuf, bary=frag.bary_coords, dists=frag.dists, img=img,
                   loss=loss, g_dists=frag.dists.grad, g_zbuf=frag.zbuf.grad, g_bary=frag.bary_coords.grad,
                   g_verts=verts.grad[0], g_log_rot=log_rot.grad, g_sigma=wl.rast.sigma.grad,
                   g_gamma=wl.agg.gamma.grad, g_alpha=wl.agg.alpha.grad)
        # ---- CPU oracle composition, same draws
        cams = wl.cameras.to(torch.device("cpu"))
        lc = wl.log_rot.detach().cpu().clone().requires_grad_(True)
        vc = Rotate(so3_exponential_map(lc)).transform_points(wl.base.verts_padded().detach().cpu())
        vc = _straight(vc, verts)
        vc.retain_grad()
        view = cams.get_world_to_view_transform().transform_points(vc)
        ndc = cams.get_projection_transform().transform_points(view)
        screen = torch.cat([ndc[..., :2], view[..., 2:3]], -1)[0]
        faces = wl.base.faces_packed().cpu()
        fv = _straight(screen[faces], fv_gpu)
        blur = math.log(1.0 / 1e-4 - 1.0) * 1e-3
        p2f, zbuf, bary, dists = pipeline_ref.RastRef.apply(fv, H, H, K, blur, True)
        for t in (zbuf, bary, dists):
            t.retain_grad()
        colors = pipeline_ref._interp(p2f, bary, wl.base.textures.verts_features_packed().detach().cpu()[faces])
        torch.manual_seed(seed)
        noise_r = torch.randn((S, 1, H, H, K))
        noise_a = torch.randn((S, 1, H, H, K + 1))
        sig, gam, alp = (torch.tensor(v, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
        zn, zf = torch.ones((1, 1, 1, 1)), torch.full((1, 1, 1, 1), 100.0)
        imgc = pipeline_ref.BlendRef.apply(dists, zbuf, colors, sig, gam, alp, p2f, noise_r, noise_a,
                                           torch.zeros(3), zn, zf)
        lossc = ((imgc[..., :3] - wl.target.cpu()) ** 2).mean()
        lossc.backward()
        cpu = dict(p2f=p2f, zbuf=zbuf, bary=bary, dists=dists, img=imgc, loss=lossc, g_dists=dists.grad,
                   g_zbuf=zbuf.grad, g_bary=bary.grad, g_verts=vc.grad[0], g_log_rot=lc.grad, g_sigma=sig.grad,
                   g_gamma=gam.grad, g_alpha=alp.grad)
        return gpu, cpu
    finally:
        pa.set_noise_source(old_src)
        torch.use_deterministic_algorithms(old_det)


@pytest.fixture(scope="module")
def frame(device):
    return headline_frame(device)


def test_headline_fragments_bitwise(frame):
    gpu, cpu = frame
    for k in ("p2f", "zbuf", "bary", "dists"):
        np.testing.assert_array_equal(gpu[k].detach().cpu().numpy(), cpu[k].detach().numpy(), err_msg=k)
    assert int((cpu["p2f"] >= 0).sum()) > 500_000  # the frame is the real one (~1.1 M valid slots)


def test_headline_image_and_fragment_gradients(frame):
    gpu, cpu = frame
    for k in ("img", "g_dists", "g_zbuf", "g_bary"):
        assert_close(gpu[k], cpu[k], name=k)
    assert abs(float(gpu["loss"]) - float(cpu["loss"])) <= 1e-5 * abs(float(cpu["loss"]))
    for k in ("g_sigma", "g_gamma", "g_alpha"):
        assert_close(gpu[k].reshape(1), cpu[k].reshape(1), rtol=2e-5, name=k)


def test_headline_rasterizer_backward_is_oracle_bitwise(frame, device):
    """The frame's rasterizer backward alone, fed the GPU's own upstream gradients: with
    torch.use_deterministic_algorithms the native d face_verts are the C oracle's bits (exact slot
    arithmetic, per-face sums in slot order); the default (tile-reduced) path agrees at 1e-5."""
    from oracle import rast_ref
    from pertrenderer_amd.renderer.rasterizer import _rasterize
    gpu, _ = frame
    H, K, blur = 256, 50, math.log(1.0 / 1e-4 - 1.0) * 1e-3
    gz, gb, gd = gpu["g_zbuf"].detach(), gpu["g_bary"].detach(), gpu["g_dists"].detach()
    first, nf = torch.tensor([0], device=device), torch.tensor([gpu["fv"].shape[0]], device=device)
    ref = rast_ref.rast_bwd(gpu["fv"].detach().cpu().numpy(), gpu["p2f"].cpu().numpy(), gz.cpu().numpy(),
                            gb.cpu().numpy(), gd.cpu().numpy(), False, True)
    old = torch.are_deterministic_algorithms_enabled()
    try:
        for det in (True, False):
            torch.use_deterministic_algorithms(det)
            fv = gpu["fv"].detach().clone().requires_grad_(True)
            p2f, zbuf, bary, dists = _rasterize(fv, first, nf, H, H, K, blur, False, True, False)
            (g,) = torch.autograd.grad((zbuf * gz).sum() + (bary * gb).sum() + (dists * gd).sum(), fv)
            if det:
                np.testing.assert_array_equal(g.cpu().numpy(), ref)
            else:
                assert_close(g, ref, name="d face_verts (tile path)")
    finally:
        torch.use_deterministic_algorithms(old)


def test_headline_pose_gradients(frame):
    gpu, cpu = frame
    assert_close(gpu["g_verts"], cpu["g_verts"], name="d verts")
    assert_close(gpu["g_log_rot"], cpu["g_log_rot"], name="d log_rot")


if __name__ == "__main__":  # diagnostic: worst |a - e| / tol per quantity
    import sys
    sys.path.insert(0, ".")
    det = len(sys.argv) < 2 or sys.argv[1] != "nondet"
    gpu, cpu = headline_frame(torch.device("cuda:0"), deterministic=det)
    for k in cpu:
        a = np.asarray(gpu[k].detach().cpu(), np.float64).reshape(-1)
        e = np.asarray(cpu[k].detach(), np.float64).reshape(-1)
        scale = np.abs(e).max() if e.size else 0.0
        tol = 1e-5 * np.abs(e) + 1e-6 * scale + 1e-30
        r = np.abs(a - e) / tol
        print(f"{k:10s} n={a.size:9d} max|e|={scale:.3e} worst/tol={r.max():.3g} bad={int((r > 1).sum())} "
              f"maxrel={float((np.abs(a - e) / (np.abs(e) + 1e-30)).max()):.3g}", flush=True)
