"""ctypes binding of libpertrender.so (the C ABI declared in include/pertrender.h).

The library is the product: every public op of this package calls into it and
raises if it is missing or the tensors are not on a ROCm device.  There is no
CPU fallback.
"""
import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# PR_NATIVE_LIB selects a diagnostic build (e.g. the -DPR_RAST_PROFILE variant)
LIB_PATH = os.environ.get("PR_NATIVE_LIB") or os.path.join(_HERE, "libpertrender.so")

PR_NOISE_PHILOX = 0
PR_NOISE_INJECTED = 1
PR_BLEND_RAST = 1
PR_BLEND_COLOR = 2
PR_BLEND_VERTEX = 4
PR_BLEND_RAST_CAUCHY = 8
PR_BLEND_AGG_CAUCHY = 16
PR_BLEND_AGG_UNIFORM = 256
PR_BLEND_WINNERS_IN = 512
PR_BLEND_LIVE_ONLY = 1024
PR_BLEND_PHONG = 2048  # forward: RandomPhongShader's shading on demand (PRBlendFwdArgs.shade)
PR_BLEND_COLOR_SPARSE = 4096  # backward of PR_BLEND_PHONG: colours valid at the slots it reads only
PR_BLEND_RAST_WOVR = 32
PR_BLEND_AGG_WOVR = 64
PR_BLEND_SOFT = 128
PR_GRAD_PREZEROED = 1
PR_BLEND_SYNC_BYTES = 1024
PR_DETERMINISTIC = 2
PR_RAST_VALID_ONLY = 8  # pr_rast_fwd: only the valid prefix of the fragments is written (needs pix_count)
PR_SHADE_LIVE_ONLY = 4  # pr_shade_*: padded slots' colours / d bary left unwritten (needs pix_count)

_vp = C.c_void_p


class PRBlendParams(C.Structure):
    _fields_ = [("N", C.c_int32), ("H", C.c_int32), ("W", C.c_int32), ("K", C.c_int32),
                ("Sr", C.c_int32), ("Sa", C.c_int32),
                ("sample_offset_r", C.c_int32), ("sample_offset_a", C.c_int32),
                ("sigma", C.c_float), ("gamma", C.c_float), ("alpha", C.c_float), ("eps", C.c_float),
                ("background", C.c_float * 3), ("noise_mode", C.c_int32),
                ("seed_r", C.c_uint64), ("seed_a", C.c_uint64),
                ("noise_r", _vp), ("noise_a", _vp), ("znear", _vp), ("zfar", _vp),
                ("flags", C.c_int32), ("scalars", _vp * 3), ("seeds", _vp)]


class PRBlendFwdArgs(C.Structure):
    _fields_ = [("p", PRBlendParams), ("pix_to_face", _vp), ("mask", _vp), ("dists", _vp),
                ("prob", _vp), ("zbuf", _vp), ("colors", _vp), ("image", _vp), ("weights", _vp),
                ("winners", _vp), ("rast_cache", _vp), ("bary", _vp), ("faces", _vp), ("vert_colors", _vp),
                ("pix_count", _vp), ("plan", _vp), ("sync", _vp), ("shade", _vp)]


class PRBlendBwdArgs(C.Structure):
    _fields_ = [("p", PRBlendParams), ("pix_to_face", _vp), ("mask", _vp), ("dists", _vp),
                ("prob", _vp), ("zbuf", _vp), ("colors", _vp), ("winners", _vp),
                ("grad_image", _vp), ("grad_weights", _vp), ("grad_dists", _vp), ("grad_prob", _vp),
                ("grad_zbuf", _vp), ("grad_colors", _vp), ("grad_scalars", _vp),
                ("workspace", _vp), ("workspace_bytes", C.c_size_t), ("rast_cache", _vp), ("bary", _vp),
                ("faces", _vp), ("vert_colors", _vp), ("grad_bary", _vp), ("grad_vert_colors", _vp),
                ("pix_count", _vp), ("plan", _vp), ("sync", _vp)]


class PRHeavisideArgs(C.Structure):
    _fields_ = [("N", C.c_int32), ("H", C.c_int32), ("W", C.c_int32), ("K", C.c_int32),
                ("Sr", C.c_int32), ("sample_offset_r", C.c_int32), ("noise_mode", C.c_int32),
                ("sigma", C.c_float), ("seed_r", C.c_uint64), ("noise_r", _vp), ("dists", _vp),
                ("prob", _vp), ("grad_prob", _vp), ("grad_dists", _vp), ("grad_sigma", _vp),
                ("workspace", _vp), ("workspace_bytes", C.c_size_t), ("sigma_dev", _vp), ("seeds", _vp),
                ("flags", C.c_int32)]


class PRRastArgs(C.Structure):
    _fields_ = [("face_verts", _vp), ("mesh_first_face", _vp), ("mesh_num_faces", _vp),
                ("F", C.c_int64), ("N", C.c_int32), ("H", C.c_int32), ("W", C.c_int32),
                ("K", C.c_int32), ("blur_radius", C.c_float), ("perspective_correct", C.c_int32),
                ("clip_barycentric_coords", C.c_int32), ("cull_backfaces", C.c_int32),
                ("pix_to_face", _vp), ("zbuf", _vp), ("bary", _vp), ("dists", _vp),
                ("grad_zbuf", _vp), ("grad_bary", _vp), ("grad_dists", _vp),
                ("grad_face_verts", _vp), ("workspace", _vp), ("workspace_bytes", C.c_size_t),
                ("pix_count", _vp), ("flags", C.c_int32), ("bin_size", C.c_int32),
                ("max_faces_per_bin", C.c_int32), ("blur_radius_dev", _vp)]


class PRInterpArgs(C.Structure):
    _fields_ = [("pix_to_face", _vp), ("bary", _vp), ("face_attr", _vp), ("PK", C.c_int64),
                ("F", C.c_int64), ("D", C.c_int32), ("out", _vp), ("grad_out", _vp),
                ("grad_bary", _vp), ("grad_face_attr", _vp), ("faces", _vp), ("V", C.c_int64)]


class PRProjectArgs(C.Structure):
    _fields_ = [("verts", _vp), ("faces", _vp), ("mesh_first_face", _vp), ("mesh_num_faces", _vp),
                ("world_to_view", _vp), ("proj", _vp), ("V", C.c_int64), ("F", C.c_int64), ("N", C.c_int32),
                ("face_verts", _vp), ("grad_face_verts", _vp), ("grad_verts", _vp), ("flags", C.c_int32),
                ("vert_corner_start", _vp), ("vert_corners", _vp), ("seed_advance", _vp),
                ("seed_advance_n", C.c_int32)]


class PRSO3Args(C.Structure):
    _fields_ = [("N", C.c_int32), ("eps", C.c_float), ("log_rot", _vp), ("R", _vp), ("grad_R", _vp),
                ("grad_log_rot", _vp)]


class PRRotateArgs(C.Structure):
    _fields_ = [("N", C.c_int32), ("P", C.c_int32), ("R_batched", C.c_int32), ("points", _vp), ("R", _vp),
                ("out", _vp), ("grad_out", _vp), ("grad_points", _vp), ("grad_R", _vp)]


class PRRgbMseArgs(C.Structure):
    _fields_ = [("P", C.c_int64), ("C", C.c_int32), ("HW", C.c_int32), ("target_batched", C.c_int32),
                ("image", _vp), ("target", _vp), ("loss", _vp), ("partials", _vp), ("grad_loss", _vp),
                ("grad_image", _vp)]


class PRPoseStepArgs(C.Structure):
    _fields_ = [("loss", _vp), ("log_rot", _vp), ("grad", _vp), ("it", _vp), ("losses", _vp), ("gnorms", _vp),
                ("best_loss", _vp), ("best", _vp), ("v", _vp), ("acc", _vp), ("leaf_grad", _vp * 3), ("seed", _vp),
                ("exp_avg", _vp), ("exp_avg_sq", _vp), ("step", _vp), ("lr", _vp),
                ("niter", C.c_int64), ("n", C.c_int32), ("post", C.c_int32), ("adam", C.c_int32)]


PR_TEX_GIVEN = 0
PR_TEX_UV = 1
PR_TEX_VERTEX = 2


class PRShadeArgs(C.Structure):
    _fields_ = [("N", C.c_int32), ("H", C.c_int32), ("W", C.c_int32), ("K", C.c_int32),
                ("pix_to_face", _vp), ("pix_count", _vp), ("bary", _vp), ("faces", _vp), ("verts", _vp),
                ("flags", C.c_int32), ("workspace", _vp), ("workspace_bytes", C.c_size_t), ("normals", _vp), ("V", C.c_int64), ("F", C.c_int64), ("texture", C.c_int32), ("texels", _vp),
                ("vert_colors", _vp), ("face_uvs", _vp), ("maps", _vp), ("Hm", C.c_int32), ("Wm", C.c_int32),
                ("directional", C.c_int32), ("light", _vp), ("ambient", _vp), ("diffuse_color", _vp),
                ("specular_color", _vp), ("mat_diffuse", _vp), ("mat_specular", _vp), ("shininess", _vp),
                ("camera", _vp), ("colors", _vp), ("grad_colors", _vp), ("grad_bary", _vp), ("grad_verts", _vp),
                ("grad_normals", _vp), ("grad_texels", _vp), ("grad_vert_colors", _vp), ("grad_maps", _vp),
                ("grad_light", _vp), ("grad_camera", _vp)]


class PRNormalsArgs(C.Structure):
    _fields_ = [("verts", _vp), ("faces", _vp), ("V", C.c_int64), ("F", C.c_int64), ("normals", _vp),
                ("raw", _vp), ("grad_normals", _vp), ("grad_raw", _vp), ("grad_verts", _vp),
                ("vert_corner_start", _vp), ("vert_corners", _vp)]


# every symbol include/pertrender.h declares, with its argument struct (None = no args)
EXPORTS = {
    "pr_abi_version": (C.c_int, []),
    "pr_last_error": (C.c_char_p, []),
    "pr_ktimer_arm": (C.c_int, [C.c_int32]),
    "pr_blend_plan_size": (C.c_size_t, [C.POINTER(PRBlendParams)]),
    "pr_ktimer_read": (C.c_int, [C.c_int32, C.POINTER(C.c_float), C.c_char_p, C.c_int32]),
    "pr_blend_fwd": (C.c_int, [C.POINTER(PRBlendFwdArgs), _vp]),
    "pr_blend_bwd_workspace_size": (C.c_size_t, [C.POINTER(PRBlendBwdArgs)]),
    "pr_blend_bwd": (C.c_int, [C.POINTER(PRBlendBwdArgs), _vp]),
    "pr_heaviside_fwd": (C.c_int, [C.POINTER(PRHeavisideArgs), _vp]),
    "pr_heaviside_bwd_workspace_size": (C.c_size_t, [C.POINTER(PRHeavisideArgs)]),
    "pr_heaviside_bwd": (C.c_int, [C.POINTER(PRHeavisideArgs), _vp]),
    "pr_rast_fwd_workspace_size": (C.c_size_t, [C.POINTER(PRRastArgs)]),
    "pr_rast_fwd": (C.c_int, [C.POINTER(PRRastArgs), _vp]),
    "pr_rast_bwd_workspace_size": (C.c_size_t, [C.POINTER(PRRastArgs)]),
    "pr_rast_bwd": (C.c_int, [C.POINTER(PRRastArgs), _vp]),
    "pr_interp_fwd": (C.c_int, [C.POINTER(PRInterpArgs), _vp]),
    "pr_interp_bwd": (C.c_int, [C.POINTER(PRInterpArgs), _vp]),
    "pr_seed_advance": (C.c_int, [_vp, C.c_int32, _vp]),
    "pr_project_fwd": (C.c_int, [C.POINTER(PRProjectArgs), _vp]),
    "pr_project_bwd": (C.c_int, [C.POINTER(PRProjectArgs), _vp]),
    "pr_project_rast_fwd": (C.c_int, [C.POINTER(PRProjectArgs), C.POINTER(PRRastArgs), _vp]),
    "pr_pose_step": (C.c_int, [C.POINTER(PRPoseStepArgs), _vp]),
    "pr_rgb_mse_workspace": (C.c_size_t, [C.c_int64]),
    "pr_rgb_mse_fwd": (C.c_int, [C.POINTER(PRRgbMseArgs), _vp]),
    "pr_rgb_mse_bwd": (C.c_int, [C.POINTER(PRRgbMseArgs), _vp]),
    "pr_so3_exp_fwd": (C.c_int, [C.POINTER(PRSO3Args), _vp]),
    "pr_so3_exp_bwd": (C.c_int, [C.POINTER(PRSO3Args), _vp]),
    "pr_rotate_fwd": (C.c_int, [C.POINTER(PRRotateArgs), _vp]),
    "pr_rotate_bwd": (C.c_int, [C.POINTER(PRRotateArgs), _vp]),
    "pr_philox": (C.c_int, [_vp, _vp, C.c_int64, _vp, _vp, _vp, C.c_int32, _vp]),
    "pr_shade_fwd": (C.c_int, [C.POINTER(PRShadeArgs), _vp]),
    "pr_shade_bwd_workspace_size": (C.c_size_t, [C.POINTER(PRShadeArgs)]),
    "pr_shade_bwd": (C.c_int, [C.POINTER(PRShadeArgs), _vp]),
    "pr_vert_normals_fwd": (C.c_int, [C.POINTER(PRNormalsArgs), _vp]),
    "pr_vert_normals_bwd": (C.c_int, [C.POINTER(PRNormalsArgs), _vp]),
}
ABI_VERSION = 20

_lib = None


class NativeError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load (once) and type the native library.  Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NativeError(
            f"libpertrender.so not found at {path}; build it with "
            "`python -m pertrenderer_amd.build_native` (hipcc, gfx950)")
    lib = C.CDLL(path)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.pr_abi_version() != ABI_VERSION:
        raise NativeError(f"libpertrender ABI {lib.pr_abi_version()} != {ABI_VERSION}")
    _lib = lib
    return lib


def check(code, what):
    if code != 0:
        msg = load().pr_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed ({code}): {msg}")


def ptr(t):
    """Device address of `t` (None for a missing optional buffer).  A plain int: ctypes takes it
    for c_void_p fields and arguments without a wrapper object per pointer."""
    return None if t is None else t.data_ptr()


def dense(t, dtype):
    """`t` detached as a contiguous `dtype` tensor: `t.detach().to(dtype).contiguous()`, without
    the two no-op dispatcher calls when it already is one (the eager step makes ~30 of these)."""
    if t.dtype is dtype and t.is_contiguous():
        return t.detach()
    return t.detach().to(dtype).contiguous()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(t):
    """The current torch stream of `t`'s device, as the hipStream_t handle (a plain int: ctypes
    passes it for the c_void_p argument)."""
    if _raw_stream is not None:
        return _raw_stream(t.device.index if t.device.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(t.device).cuda_stream


_get_device = getattr(torch._C, "_cuda_getDevice", None) or torch.cuda.current_device
_FNS = {}


def call(name, what, t, *args):
    """Run C-ABI entry `name`(*args, stream) on `t`'s device: the stream is that device's current
    torch stream, and when `t` lives on another device than the current one (in-process sample
    sharding over devices, multidevice.py) the call runs under a device guard, so every launch,
    memset and error query of the library addresses `t`'s device.  Raises NativeError on a
    non-zero status."""
    fn = _FNS.get(name)
    if fn is None:
        fn = _FNS[name] = getattr(load(), name)
    idx = t.device.index
    if idx is not None and idx != _get_device():
        with torch.cuda.device(idx):
            code = fn(*args, stream_of(t))
    else:
        code = fn(*args, stream_of(t))
    if code != 0:
        check(code, what)


def deterministic():
    """Deterministic-order backward passes (PR_DETERMINISTIC), switched with torch's own
    ``torch.use_deterministic_algorithms(True)``: the sums the fast kernels scatter with float
    atomics (rasterizer, shading) are formed by a stable sort and in-order sums instead, and the
    rasterizer backward then reproduces the CPU oracle's (PyTorch3D's CPU) accumulation bit for
    bit.  Gathers over the mesh topology (projection, vertex normals) are deterministic always."""
    return torch.are_deterministic_algorithms_enabled()


def workspace(nbytes, device):
    """A caller-owned scratch buffer for a native call (the library allocates nothing)."""
    return torch.empty(max(1, int(nbytes)), dtype=torch.uint8, device=device)


def require_device(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise NativeError(
                "pertrenderer_amd native ops run on ROCm devices only (got a "
                f"{t.device} tensor); there is no CPU fallback")
