"""The C++ autograd layer (csrc/pr_torch.cpp -> _pr_torch*.so) for the eager step.

The pose, rasterizer, fused-blend, smoothing-scalar-link, Phong-shading and vertex-normal nodes of an eager step
(experiments/eval.py:343-376) run as torch C++ autograd Functions that fill the C-ABI structs and
launch through the loaded libpertrender's entry points: no ctypes packing, no Python
``Function.apply`` per op.  Same kernels, same arguments, same results as
the Python autograd Functions, which remain the path when

* a :class:`~pertrenderer_amd.timing.KernelTimer` is active (bench.py's instrumented pass marks
  each native call from Python),
* ``PR_TORCH_EXT=0`` is set, or
* the module was not built (``python -m pertrenderer_amd.build_native`` builds both libraries;
  :func:`layer` then reports ``"python"``, and bench.py prints it in its line).
"""
import contextlib
import ctypes
import importlib.machinery
import importlib.util
import os

from . import _native as nat
from . import timing as _timing

_EXT = None
_STATE = None  # None: not tried; "c++" / "python"
_ERROR = None
_ENTRIES = ("pr_abi_version", "pr_last_error", "pr_so3_exp_fwd", "pr_so3_exp_bwd", "pr_rotate_fwd",
            "pr_rotate_bwd", "pr_project_rast_fwd", "pr_project_bwd", "pr_rast_fwd_workspace_size",
            "pr_rast_bwd_workspace_size", "pr_rast_bwd", "pr_blend_fwd", "pr_blend_plan_size",
            "pr_blend_bwd_workspace_size", "pr_blend_bwd", "pr_shade_fwd", "pr_shade_bwd_workspace_size", "pr_shade_bwd",
            "pr_vert_normals_fwd", "pr_vert_normals_bwd", "pr_rgb_mse_workspace", "pr_rgb_mse_fwd", "pr_rgb_mse_bwd")


def _path():
    import sysconfig
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "_pr_torch" + sysconfig.get_config_var("EXT_SUFFIX"))


def _load():
    global _EXT, _STATE, _ERROR
    _STATE = "python"
    if os.environ.get("PR_TORCH_EXT", "1") == "0":
        return
    path = _path()
    if not os.path.exists(path):
        _ERROR = f"{path} not built"
        return
    lib = nat.load()  # the library the ctypes path drives: one instance for both layers
    loader = importlib.machinery.ExtensionFileLoader("_pr_torch", path)
    spec = importlib.util.spec_from_file_location("_pr_torch", path, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    if mod.ABI_VERSION != nat.ABI_VERSION or mod.PARAMS_BYTES != ctypes.sizeof(nat.PRBlendParams):
        _ERROR = f"_pr_torch built for ABI {mod.ABI_VERSION}, package ABI {nat.ABI_VERSION}: rebuild"
        return
    mod.bind({n: ctypes.cast(getattr(lib, n), ctypes.c_void_p).value for n in _ENTRIES})
    _EXT, _STATE = mod, "c++"


_OFF = 0  # disabled() nesting depth


def get():
    """The extension module when this call should take the C++ layer, else None."""
    if _STATE is None:
        _load()
    if _EXT is None or _OFF or _timing.active() is not None:
        return None
    return _EXT


@contextlib.contextmanager
def disabled():
    """Route the eager nodes through the Python Functions inside the block (A/B tests, profiling)."""
    global _OFF
    _OFF += 1
    try:
        yield
    finally:
        _OFF -= 1


def layer():
    """"c++" when eager autograd nodes run in the C++ layer, "python" otherwise."""
    if _STATE is None:
        _load()
    return _STATE


def error():
    """Why the C++ layer is not in use (None when it is, or when it was switched off)."""
    if _STATE is None:
        _load()
    return _ERROR
