"""pytorch3d.renderer.mesh (shim)."""
from pertrenderer_amd.renderer import Textures, TexturesAtlas, TexturesUV, TexturesVertex  # noqa: F401
from pertrenderer_amd.renderer.rasterizer import Fragments, rasterize_meshes  # noqa: F401
