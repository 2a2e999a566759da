"""pytorch3d.structures (shim; experiments/eval.py:57)."""
from pertrenderer_amd.renderer.mesh import Meshes  # noqa: F401
