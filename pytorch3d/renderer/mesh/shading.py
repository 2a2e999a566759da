"""pytorch3d.renderer.mesh.shading (shim; random_rasterizer.py:8)."""
from pertrenderer_amd.renderer.shading import phong_shading  # noqa: F401
