"""pytorch3d.io (shim; experiments/eval.py:59)."""
from pertrenderer_amd.renderer.io import load_obj, load_objs_as_meshes  # noqa: F401
