"""PyTorch3D-compatible renderer subset (cameras, meshes, rasterizer, textures) on
the native gfx950 kernels.  Only what the reference's hot path and its caller
(experiments/eval.py) touch."""
from .cameras import (FoVPerspectiveCameras, OpenGLPerspectiveCameras, camera_position_from_spherical_angles,
                      look_at_rotation, look_at_view_transform)
from .blending import hard_rgb_blend, sigmoid_alpha_blend, softmax_rgb_blend
from .interp import interpolate_face_attributes
from .io import load_obj, load_objs_as_meshes
from .loss import chamfer_distance, mesh_edge_loss, mesh_laplacian_smoothing, mesh_normal_consistency
from .mesh import Meshes, TexturesVertex
from .rasterizer import Fragments, MeshRasterizer, RasterizationSettings, rasterize_meshes
from .renderer import BlendParams, DirectionalLights, Materials, MeshRenderer, PointLights
from .shaders import HardPhongShader, SoftPhongShader, SoftSilhouetteShader
from .shading import phong_shading
from .textures import Textures, TexturesAtlas, TexturesUV
from .transforms import (Rotate, random_rotations, so3_exp_map, so3_exponential_map, so3_log_map,
                         so3_relative_angle)

__all__ = [
    "FoVPerspectiveCameras", "OpenGLPerspectiveCameras", "camera_position_from_spherical_angles",
    "look_at_rotation", "look_at_view_transform", "interpolate_face_attributes", "load_obj", "Meshes",
    "TexturesVertex", "Fragments", "MeshRasterizer", "RasterizationSettings", "rasterize_meshes",
    "BlendParams", "DirectionalLights", "Materials", "MeshRenderer", "PointLights", "hard_rgb_blend",
    "sigmoid_alpha_blend", "softmax_rgb_blend", "load_objs_as_meshes", "chamfer_distance", "mesh_edge_loss",
    "mesh_laplacian_smoothing", "mesh_normal_consistency", "HardPhongShader", "SoftPhongShader",
    "SoftSilhouetteShader", "phong_shading", "Textures", "TexturesAtlas", "TexturesUV", "Rotate",
    "random_rotations", "so3_exp_map", "so3_exponential_map", "so3_log_map", "so3_relative_angle",
]
