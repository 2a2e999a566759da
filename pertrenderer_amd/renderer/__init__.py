"""PyTorch3D-compatible renderer subset (cameras, meshes, rasterizer, textures) on
the native gfx950 kernels.  Only what the reference's hot path and its caller
(experiments/eval.py) touch."""
from .cameras import (FoVPerspectiveCameras, OpenGLPerspectiveCameras, camera_position_from_spherical_angles,
                      look_at_rotation, look_at_view_transform)
from .interp import interpolate_face_attributes
from .io import load_obj
from .mesh import Meshes, TexturesVertex
from .rasterizer import Fragments, MeshRasterizer, RasterizationSettings, rasterize_meshes
from .renderer import BlendParams, DirectionalLights, Materials, MeshRenderer, PointLights

__all__ = [
    "FoVPerspectiveCameras", "OpenGLPerspectiveCameras", "camera_position_from_spherical_angles",
    "look_at_rotation", "look_at_view_transform", "interpolate_face_attributes", "load_obj", "Meshes",
    "TexturesVertex", "Fragments", "MeshRasterizer", "RasterizationSettings", "rasterize_meshes",
    "BlendParams", "DirectionalLights", "Materials", "MeshRenderer", "PointLights",
]
