"""pytorch3d.renderer names used by the reference (shim, see pytorch3d/__init__.py)."""
from pertrenderer_amd.renderer import (BlendParams, DirectionalLights, FoVPerspectiveCameras,  # noqa: F401
                                       HardPhongShader, Materials, MeshRasterizer, MeshRenderer,
                                       OpenGLPerspectiveCameras, PointLights, RasterizationSettings,
                                       SoftPhongShader, SoftSilhouetteShader, Textures, TexturesAtlas, TexturesUV,
                                       TexturesVertex, hard_rgb_blend, interpolate_face_attributes,
                                       look_at_rotation, look_at_view_transform, rasterize_meshes,
                                       sigmoid_alpha_blend, softmax_rgb_blend)
from pertrenderer_amd.renderer.rasterizer import Fragments  # noqa: F401
