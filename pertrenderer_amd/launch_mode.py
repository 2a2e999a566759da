"""eval.py's launch-blocking request under HIP.

The reference sets ``CUDA_LAUNCH_BLOCKING=1`` before importing torch (experiments/eval.py:4) so that
its per-phase wall-clock timers (:349-355 forward, :368-370 backward, printed at :406-408) measure
work, not launches.  The HIP runtime ignores that variable; its equivalent is
``HIP_LAUNCH_BLOCKING=1`` (profiles/r3_launch_blocking.txt).  The HIP runtime reads its flags when
it initialises, so the mapping must happen before the first GPU call of the process: the
``pytorch3d`` shim and this package call :func:`honour_cuda_launch_blocking` first thing at import
(eval.py:26 imports the shim before touching the GPU).  Nothing is re-executed.
"""
import os
import sys
import warnings


def _truthy(v):
    return v is not None and v.strip() not in ("", "0")


def honour_cuda_launch_blocking(environ=None):
    """Map CUDA_LAUNCH_BLOCKING=1 to HIP_LAUNCH_BLOCKING=1 when the GPU runtime is not yet
    initialised.  Returns True when the mapping was made (or was already in place), False when
    it was not requested or came too late (a warning says so).  An explicit HIP_LAUNCH_BLOCKING
    setting is left alone."""
    env = os.environ if environ is None else environ
    if not _truthy(env.get("CUDA_LAUNCH_BLOCKING")):
        return False
    if "HIP_LAUNCH_BLOCKING" in env:
        return _truthy(env.get("HIP_LAUNCH_BLOCKING"))
    torch = sys.modules.get("torch")
    cuda = getattr(torch, "cuda", None) if torch is not None else None
    if cuda is not None and getattr(cuda, "is_initialized", lambda: False)():
        warnings.warn("CUDA_LAUNCH_BLOCKING=1 is set but the HIP runtime is already initialised: launches stay "
                      "asynchronous (set HIP_LAUNCH_BLOCKING=1 before the first GPU call)", RuntimeWarning)
        return False
    env["HIP_LAUNCH_BLOCKING"] = "1"
    return True
