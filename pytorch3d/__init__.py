"""Import shim: the PyTorch3D 0.4.0 names that quentinll/pertrenderer's code imports
(randomras/random_rasterizer.py:8-26, experiments/eval.py:26-59), served by
pertrenderer_amd's gfx950 implementations, so that code runs unchanged with this
repository on PYTHONPATH.  Only those names exist; anything else raises ImportError."""
from pertrenderer_amd.launch_mode import honour_cuda_launch_blocking as _honour

_honour()  # eval.py:4's CUDA_LAUNCH_BLOCKING=1 -> HIP_LAUNCH_BLOCKING=1, before any GPU call

__version__ = "0.4.0+pertrenderer_amd"
