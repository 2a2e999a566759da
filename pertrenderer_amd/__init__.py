"""pertrenderer_amd — MI355X-native perturbed differentiable renderer.

Drop-in for quentinll/pertrenderer's ``randomras`` plugin surface (also importable
as ``randomras``).  The hot path — K-nearest-face rasterization, the Gaussian-
perturbed Heaviside over signed edge distances and the Monte-Carlo perturbed-
argmax colour aggregation, forward and backward — runs in hand-written HIP for
gfx950 (libpertrender.so, C ABI in include/pertrender.h).
"""
from .launch_mode import honour_cuda_launch_blocking as _honour

_honour()  # first thing: eval.py's CUDA_LAUNCH_BLOCKING=1 as HIP_LAUNCH_BLOCKING=1 (launch_mode.py)

from . import _native  # noqa: E402
from .blend import perturbed_aggregate, perturbed_blend, perturbed_blend_vertex, perturbed_heaviside, soft_blend
from .multidevice import activate_from_env as _activate_sample_devices
from .multidevice import sample_devices, set_sample_devices
from .noise import Noise, get_noise_source, set_noise_source
from .random_rasterizer import (RandomPhongShader, RandomSimpleShader, SimpleShader, SoftSimpleShader,
                                smooth_rgb_blend)
from .smoothagg import CauchyAgg, GaussianAgg, GaussianAgg_wovr, HardAgg, SoftAgg, UniformAgg
from .smoothrast import AffineRast, ArctanRast, GaussianRast, GaussianRast_wovr, HardRast, SoftRast

__version__ = "0.1.0"

# PR_SAMPLE_DEVICES (e.g. "all"): shard every native Monte-Carlo blend's samples over the listed
# devices from import on (multidevice.py), so eval.py runs unchanged on a multi-GPU node
_activate_sample_devices()


def native_library():
    """Load libpertrender.so (raises NativeError if it was not built)."""
    return _native.load()
