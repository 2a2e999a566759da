"""K-nearest-face mesh rasterizer (PyTorch3D 0.4.0 ``MeshRasterizer`` /
``rasterize_meshes`` semantics) on the native gfx950 kernels pr_rast_fwd/bwd.

MeshRasterizer.forward(meshes_world): world -> view (R,T) -> NDC with view-space z
kept, then per pixel the K nearest faces (ascending z, ties by face index) within
``blur_radius`` (a squared-distance threshold).  Output ``Fragments`` as PyTorch3D:
pix_to_face (N,H,W,K) int64 packed face ids (-1 padded), zbuf, bary_coords
(N,H,W,K,3), dists (signed squared distance, negative inside).  Called by the
reference at experiments/eval.py:165-168 (RasterizationSettings at :135-141).
"""
import os
from typing import NamedTuple, Optional

import torch

from .. import _native as nat
from .. import host_layer
from .. import noise as noise_mod
from .. import timing as _timing
from .mesh import gather_faces
from .project import project_faces

F32 = torch.float32


class Fragments(NamedTuple):
    pix_to_face: torch.Tensor
    zbuf: torch.Tensor
    bary_coords: torch.Tensor
    dists: torch.Tensor


class RasterizationSettings:
    """Mutable settings object (eval.py:390 assigns blur_radius in place)."""

    def __init__(self, image_size=256, blur_radius=0.0, faces_per_pixel=1, bin_size=None,
                 max_faces_per_bin=None, perspective_correct=False, clip_barycentric_coords=None,
                 cull_backfaces=False):
        self.image_size = image_size
        self.blur_radius = blur_radius
        self.faces_per_pixel = faces_per_pixel
        self.bin_size = bin_size                  # coarse bins (0: every tile culls the whole mesh)
        self.max_faces_per_bin = max_faces_per_bin  # bin list capacity; an overflowing bin culls the mesh
        self.perspective_correct = perspective_correct
        self.clip_barycentric_coords = clip_barycentric_coords
        self.cull_backfaces = cull_backfaces


def _hw(image_size):
    if isinstance(image_size, (tuple, list)):
        return int(image_size[0]), int(image_size[1])
    return int(image_size), int(image_size)


def bin_params(bin_size, max_faces_per_bin, H, W, F, N=1):
    """(bin_size, max_faces_per_bin) for the native rasterizer.  An explicit bin_size > 0 bins
    with PyTorch3D 0.4.0's meaning (rasterize_meshes.py; the dependency is not vendored, restated)
    and max_faces_per_bin (None: max(10000, F / 5)) is the list capacity; an overflowing bin falls
    back to the whole mesh, so the fragments never depend on either knob.  bin_size None or 0 runs
    the tiles' whole-mesh cull: measured faster than bins on the cfg 2 frame (1280 faces) and on
    an 81 920-face sphere at 256^2 (tools/rast_bins_bench.py).
    PR_RAST_BINS=0 forces the naive path, PR_RAST_BINS=1 resolves None as PyTorch3D does (bins of
    8 / 16 / 32 / 64 pixels up to 64 / 256 / 512 / 1024-pixel images)."""
    env = os.environ.get("PR_RAST_BINS")
    if env == "0" or (bin_size is None and env != "1") or (bin_size is not None and bin_size <= 0):
        return 0, 0
    if bin_size is None:
        size = max(H, W)
        bin_size = 8 if size <= 64 else 16 if size <= 256 else 32 if size <= 512 else 64
    if max_faces_per_bin is None:
        max_faces_per_bin = int(max(10000, F / 5))
    return int(bin_size), int(min(max_faces_per_bin, 2**31 - 1))


def attach_valid_counts(pix_to_face, counts):
    """Remember the rasterizer's per-pixel valid-prefix counts on its pix_to_face tensor (the
    valid slots of a pixel are 0..count-1, PyTorch3D's -1 padding after them).  Native ops on
    these fragments then read no fragment data at padded slots.  Tied to the tensor's version:
    an in-place change of pix_to_face drops them."""
    pix_to_face._pr_valid_counts = (pix_to_face._version, counts)
    return pix_to_face


def valid_counts(pix_to_face):
    """The (N,H,W) int32 counts attached by the native rasterizer, or None."""
    e = getattr(pix_to_face, "_pr_valid_counts", None)
    return e[1] if e is not None and e[0] == pix_to_face._version else None


def _blur_arg(blur, device):
    """(by-value threshold, device threshold or None) for PRRastArgs: RasterizationSettings.blur_radius
    may be a one-element float32 tensor on the mesh's device (an extension of PyTorch3D's float),
    which the kernels read in place -- a captured graph then replays with the value the caller
    last wrote (pose_opt's graph mode, eval.py's adaptive blur)."""
    if torch.is_tensor(blur):
        if blur.device != device or blur.dtype != F32 or blur.numel() != 1:
            raise ValueError("a tensor blur_radius must be one float32 on the mesh's device")
        return 0.0, blur
    return float(blur), None


def _bwd_workspace(lib, a, device):
    """Deterministic mode (torch.use_deterministic_algorithms): PR_DETERMINISTIC and its sort
    workspace on the rasterizer backward's args; None otherwise."""
    if not nat.deterministic():
        return None
    a.flags = a.flags | nat.PR_DETERMINISTIC
    ws = nat.workspace(lib.pr_rast_bwd_workspace_size(a), device)
    a.workspace, a.workspace_bytes = nat.ptr(ws), ws.numel()
    return ws


class _RasterizeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, face_verts, first, nfaces, H, W, K, blur, persp, clip, cull, bins=(0, 0)):
        nat.require_device(face_verts, first, nfaces)
        lib = nat.load()
        fv = nat.dense(face_verts, F32)
        N = first.shape[0]
        dev = fv.device
        a = nat.PRRastArgs()
        a.face_verts, a.mesh_first_face, a.mesh_num_faces = nat.ptr(fv), nat.ptr(first), nat.ptr(nfaces)
        a.F, a.N, a.H, a.W, a.K = fv.shape[0], N, H, W, K
        a.blur_radius, a.perspective_correct = float(blur), int(persp)
        a.clip_barycentric_coords, a.cull_backfaces = int(clip), int(cull)
        a.bin_size, a.max_faces_per_bin = bins
        p2f = torch.empty((N, H, W, K), dtype=torch.int64, device=dev)
        zbuf = torch.empty((N, H, W, K), dtype=F32, device=dev)
        bary = torch.empty((N, H, W, K, 3), dtype=F32, device=dev)
        dists = torch.empty((N, H, W, K), dtype=F32, device=dev)
        counts = torch.empty((N, H, W), dtype=torch.int32, device=dev)
        a.pix_to_face, a.zbuf, a.bary, a.dists = nat.ptr(p2f), nat.ptr(zbuf), nat.ptr(bary), nat.ptr(dists)
        a.pix_count = nat.ptr(counts)
        ws = torch.empty(max(1, lib.pr_rast_fwd_workspace_size(a)), dtype=torch.uint8, device=dev)
        a.workspace, a.workspace_bytes = nat.ptr(ws), ws.numel()
        timing = _timing.active()
        if timing is not None:
            timing.start("rast_fwd")
        nat.call("pr_rast_fwd", "pr_rast_fwd", fv, a)
        if timing is not None:
            timing.stop("rast_fwd")
        ctx.save_for_backward(fv, first, nfaces, p2f, counts)
        ctx.cfg = (H, W, K, float(blur), int(persp), int(clip), int(cull))
        ctx.mark_non_differentiable(p2f, counts)
        ctx.set_materialize_grads(False)  # no zero-filled int64 grad for pix_to_face
        return p2f, zbuf, bary, dists, counts

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gp2f, gzbuf, gbary, gdists, gcounts):
        fv, first, nfaces, p2f, counts = ctx.saved_tensors
        H, W, K, blur, persp, clip, cull = ctx.cfg
        lib = nat.load()
        a = nat.PRRastArgs()
        a.face_verts, a.mesh_first_face, a.mesh_num_faces = nat.ptr(fv), nat.ptr(first), nat.ptr(nfaces)
        a.F, a.N, a.H, a.W, a.K = fv.shape[0], first.shape[0], H, W, K
        a.blur_radius, a.perspective_correct, a.clip_barycentric_coords, a.cull_backfaces = blur, persp, clip, cull
        a.pix_to_face, a.pix_count = nat.ptr(p2f), nat.ptr(counts)
        keep = []
        for name, g in (("grad_zbuf", gzbuf), ("grad_bary", gbary), ("grad_dists", gdists)):
            if g is not None:
                g = nat.dense(g, F32)
                keep.append(g)
                setattr(a, name, nat.ptr(g))
        gfv = torch.empty_like(fv)
        a.grad_face_verts = nat.ptr(gfv)
        ws = _bwd_workspace(lib, a, fv.device)
        timing = _timing.active()
        if timing is not None:
            timing.start("rast_bwd")
        nat.call("pr_rast_bwd", "pr_rast_bwd", fv, a)
        if timing is not None:
            timing.stop("rast_bwd")
        del ws
        return gfv, None, None, None, None, None, None, None, None, None, None


class _ProjectRasterizeFn(torch.autograd.Function):
    """MeshRasterizer.forward's fast path as one op: world verts -> (projection + face gather +
    rasterization) -> fragments (pr_project_rast_fwd: one face pass, then the rasterizer);
    backward: pr_rast_bwd then pr_project_bwd into d verts, their accumulators zeroed by the
    forward kernel (no memsets).  Same values as project_faces followed by _RasterizeFn."""

    @staticmethod
    def forward(ctx, verts, faces, first, nfaces, w2v, proj, H, W, K, blur, persp, clip, cull, bins=(0, 0),
                csr_start=None, csr_corners=None, seed_adv=None, seed_n=0):
        from .project import _per_mesh
        nat.require_device(verts, faces, first, nfaces, w2v, proj)
        lib = nat.load()
        v = nat.dense(verts, F32)
        f = nat.dense(faces, torch.int64)
        N, F, dev = first.shape[0], f.shape[0], v.device
        m1, m2 = _per_mesh(w2v, N, "world_to_view"), _per_mesh(proj, N, "projection")
        fv = torch.empty((F, 3, 3), dtype=F32, device=dev)
        need = ctx.needs_input_grad[0]
        gfv = torch.empty((F, 3, 3), dtype=F32, device=dev) if need else None
        gv = torch.empty_like(v) if need else None
        pa = nat.PRProjectArgs()
        pa.verts, pa.faces, pa.mesh_first_face, pa.mesh_num_faces = nat.ptr(v), nat.ptr(f), nat.ptr(first), nat.ptr(nfaces)
        pa.world_to_view, pa.proj = nat.ptr(m1), nat.ptr(m2)
        pa.V, pa.F, pa.N = v.shape[0], F, N
        pa.face_verts, pa.grad_verts = nat.ptr(fv), nat.ptr(gv)
        if seed_adv is not None and seed_n > 0:  # the caller's deferred noise-key advances (DeviceSeed)
            pa.seed_advance, pa.seed_advance_n = nat.ptr(seed_adv), int(seed_n)
        a = nat.PRRastArgs()
        a.face_verts, a.mesh_first_face, a.mesh_num_faces = nat.ptr(fv), nat.ptr(first), nat.ptr(nfaces)
        a.F, a.N, a.H, a.W, a.K = F, N, H, W, K
        blur_v, blur_dev = _blur_arg(blur, dev)
        a.blur_radius, a.blur_radius_dev, a.perspective_correct = blur_v, nat.ptr(blur_dev), int(persp)
        a.clip_barycentric_coords, a.cull_backfaces = int(clip), int(cull)
        a.bin_size, a.max_faces_per_bin = bins
        p2f = torch.empty((N, H, W, K), dtype=torch.int64, device=dev)
        zbuf = torch.empty((N, H, W, K), dtype=F32, device=dev)
        bary = torch.empty((N, H, W, K, 3), dtype=F32, device=dev)
        dists = torch.empty((N, H, W, K), dtype=F32, device=dev)
        counts = torch.empty((N, H, W), dtype=torch.int32, device=dev)
        a.pix_to_face, a.zbuf, a.bary, a.dists = nat.ptr(p2f), nat.ptr(zbuf), nat.ptr(bary), nat.ptr(dists)
        a.pix_count, a.grad_face_verts = nat.ptr(counts), nat.ptr(gfv)
        ws = torch.empty(max(1, lib.pr_rast_fwd_workspace_size(a)), dtype=torch.uint8, device=dev)
        a.workspace, a.workspace_bytes = nat.ptr(ws), ws.numel()
        timing = _timing.active()
        if timing is not None:
            timing.start("rast_fwd")
        nat.call("pr_project_rast_fwd", "pr_project_rast_fwd", fv, pa, a)
        if timing is not None:
            timing.stop("rast_fwd")
        ctx.save_for_backward(v, f, first, nfaces, m1, m2, fv, p2f, counts, gfv, gv)
        ctx.cfg = (H, W, K, blur_v, int(persp), int(clip), int(cull))
        ctx.csr = (csr_start, csr_corners)
        ctx.prezeroed = True
        ctx.mark_non_differentiable(p2f, counts)
        ctx.set_materialize_grads(False)
        return p2f, zbuf, bary, dists, counts

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gp2f, gzbuf, gbary, gdists, gcounts):
        v, f, first, nfaces, m1, m2, fv, p2f, counts, gfv, gv = ctx.saved_tensors
        if gfv is None:
            return (None,) * 18
        H, W, K, blur, persp, clip, cull = ctx.cfg
        # a second backward (retain_graph) finds the accumulators used: zero them again
        flags = nat.PR_GRAD_PREZEROED if ctx.prezeroed else 0
        ctx.prezeroed = False
        lib = nat.load()
        a = nat.PRRastArgs()
        a.face_verts, a.mesh_first_face, a.mesh_num_faces = nat.ptr(fv), nat.ptr(first), nat.ptr(nfaces)
        a.F, a.N, a.H, a.W, a.K = fv.shape[0], first.shape[0], H, W, K
        a.blur_radius, a.perspective_correct, a.clip_barycentric_coords, a.cull_backfaces = blur, persp, clip, cull
        a.pix_to_face, a.pix_count, a.flags = nat.ptr(p2f), nat.ptr(counts), flags
        keep = []
        for name, g in (("grad_zbuf", gzbuf), ("grad_bary", gbary), ("grad_dists", gdists)):
            if g is not None:
                g = nat.dense(g, F32)
                keep.append(g)
                setattr(a, name, nat.ptr(g))
        a.grad_face_verts = nat.ptr(gfv)
        ws = _bwd_workspace(lib, a, fv.device)
        timing = _timing.active()
        if timing is not None:
            timing.start("rast_bwd")
        nat.call("pr_rast_bwd", "pr_rast_bwd", fv, a)
        if timing is not None:
            timing.stop("rast_bwd")
        del ws
        pa = nat.PRProjectArgs()
        pa.verts, pa.faces, pa.mesh_first_face, pa.mesh_num_faces = nat.ptr(v), nat.ptr(f), nat.ptr(first), nat.ptr(nfaces)
        pa.world_to_view, pa.proj = nat.ptr(m1), nat.ptr(m2)
        pa.V, pa.F, pa.N = v.shape[0], f.shape[0], first.shape[0]
        pa.grad_face_verts, pa.grad_verts, pa.flags = nat.ptr(gfv), nat.ptr(gv), flags
        pa.vert_corner_start, pa.vert_corners = nat.ptr(ctx.csr[0]), nat.ptr(ctx.csr[1])
        nat.call("pr_project_bwd", "pr_project_bwd", gv, pa)
        return (gv,) + (None,) * 17


def rasterize_meshes(meshes, image_size=256, blur_radius=0.0, faces_per_pixel=8, bin_size=None,
                     max_faces_per_bin=None, perspective_correct=False, clip_barycentric_coords=False,
                     cull_backfaces=False):
    """PyTorch3D rasterize_meshes on meshes already in NDC (x,y) + view z."""
    verts = meshes.verts_packed()
    face_verts = gather_faces(verts, meshes.faces_packed())
    first = meshes.mesh_to_faces_packed_first_idx().to(verts.device)
    nfaces = meshes.num_faces_per_mesh().to(verts.device)
    H, W = _hw(image_size)
    bins = bin_params(bin_size, max_faces_per_bin, H, W, face_verts.shape[0], first.shape[0])
    return _rasterize(face_verts, first, nfaces, H, W, int(faces_per_pixel), float(blur_radius),
                      bool(perspective_correct), bool(clip_barycentric_coords), bool(cull_backfaces), bins)


def _rasterize(face_verts, first, nfaces, H, W, K, blur, persp, clip, cull, bins=(0, 0)):
    p2f, zbuf, bary, dists, counts = _RasterizeFn.apply(face_verts, first, nfaces, H, W, K, blur, persp, clip, cull,
                                                        bins)
    return attach_valid_counts(p2f, counts), zbuf, bary, dists


class MeshRasterizer(torch.nn.Module):
    def __init__(self, cameras=None, raster_settings=None):
        super().__init__()
        self.cameras = cameras
        self.raster_settings = raster_settings if raster_settings is not None else RasterizationSettings()

    def to(self, device):
        if self.cameras is not None:
            self.cameras = self.cameras.to(device)
        return self

    def transform(self, meshes_world, **kwargs):
        cameras = kwargs.get("cameras", self.cameras)
        if cameras is None:
            raise ValueError("Cameras must be specified either at initialization or in the forward pass "
                             "of MeshRasterizer")
        verts_world = meshes_world.verts_padded()
        verts_view = cameras.get_world_to_view_transform(**kwargs).transform_points(verts_world)
        verts_ndc = cameras.get_projection_transform(**kwargs).transform_points(verts_view)
        verts_ndc = torch.cat([verts_ndc[..., :2], verts_view[..., 2:3]], dim=-1)
        return meshes_world.update_padded(verts_ndc)

    def forward(self, meshes_world, **kwargs) -> Fragments:
        # (MeshRenderer's, for a shader that reads each pixel's valid prefix only: the padding of the
        # fragments is then left unwritten -- PR_RAST_VALID_ONLY; never set for a caller's own use)
        valid_only = bool(kwargs.pop("_pr_valid_only", False))
        rs = kwargs.get("raster_settings", self.raster_settings)
        clip = rs.clip_barycentric_coords
        if clip is None:  # (a device blur_radius is taken as > 0: reading it would synchronise)
            clip = True if torch.is_tensor(rs.blur_radius) else rs.blur_radius > 0.0
        cameras = kwargs.get("cameras", self.cameras)
        overrides = any(k in kwargs for k in ("R", "T", "znear", "zfar", "fov", "aspect_ratio", "degrees"))
        if (hasattr(cameras, "world_to_view_matrix") and not overrides and not cameras.matrices_need_grad()
                and meshes_world.verts_packed().is_cuda):
            # fused native projection + face gather (pr_project_*), then the rasterizer
            first = meshes_world.mesh_to_faces_packed_first_idx()
            nfaces = meshes_world.num_faces_per_mesh()
            H, W = _hw(rs.image_size)
            faces = meshes_world.faces_packed()
            bins = bin_params(rs.bin_size, rs.max_faces_per_bin, H, W, faces.shape[0], first.shape[0])
            ext = host_layer.get()
            verts = meshes_world.verts_packed()
            # the active DeviceSeed's deferred advance rides on this face pass (noise.DeviceSeed)
            seed_adv, seed_n = noise_mod.take_pending_advance(verts.device)
            try:
                if ext is not None:  # the C++ autograd layer (host_layer.py): same kernels and arguments
                    p2f, zbuf, bary, dists, counts = ext.project_rasterize(
                        verts, faces, first, nfaces, cameras.world_to_view_matrix(),
                        cameras.projection_matrix(), *meshes_world.corner_csr("gather"),
                        [H, W, int(rs.faces_per_pixel), int(bool(rs.perspective_correct)), int(bool(clip)),
                         int(bool(rs.cull_backfaces)), bins[0], bins[1], int(valid_only)],
                        *_blur_arg(rs.blur_radius, verts.device),
                        seed_adv, seed_n)
                else:
                    p2f, zbuf, bary, dists, counts = _ProjectRasterizeFn.apply(
                        verts, faces, first, nfaces,
                        cameras.world_to_view_matrix(), cameras.projection_matrix(), H, W, int(rs.faces_per_pixel),
                        rs.blur_radius, bool(rs.perspective_correct), bool(clip), bool(rs.cull_backfaces),
                        bins, *meshes_world.corner_csr("gather"), seed_adv, seed_n)
            except BaseException:
                noise_mod.give_back_advance(seed_n)
                raise
            return Fragments(pix_to_face=attach_valid_counts(p2f, counts), zbuf=zbuf, bary_coords=bary, dists=dists)
        meshes_screen = self.transform(meshes_world, **kwargs)
        blur = float(rs.blur_radius)  # (the torch-transform path takes the value: one host read)
        p2f, zbuf, bary, dists = rasterize_meshes(
            meshes_screen, image_size=rs.image_size, blur_radius=blur,
            faces_per_pixel=rs.faces_per_pixel, bin_size=rs.bin_size, max_faces_per_bin=rs.max_faces_per_bin,
            perspective_correct=rs.perspective_correct, clip_barycentric_coords=clip,
            cull_backfaces=rs.cull_backfaces)
        return Fragments(pix_to_face=p2f, zbuf=zbuf, bary_coords=bary, dists=dists)
