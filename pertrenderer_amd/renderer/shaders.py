"""PyTorch3D 0.4.0 shaders that experiments/eval.py constructs besides the perturbed ones:
HardPhongShader (target renders, eval.py:265-283, 762-780), SoftPhongShader and
SoftSilhouetteShader (imported, eval.py:40-41).  Texels come from the mesh's textures
(TexturesVertex: native interpolation; TexturesUV / TexturesAtlas: textures.py),
lighting from shading.phong_shading."""
import torch
import torch.nn as nn

from .blending import hard_rgb_blend, sigmoid_alpha_blend, softmax_rgb_blend
from .renderer import BlendParams, Materials, PointLights
from .shading import textured_phong_shading


class _ShaderBase(nn.Module):
    def __init__(self, device="cpu", cameras=None, lights=None, materials=None, blend_params=None):
        super().__init__()
        self.lights = lights if lights is not None else PointLights(device=device)
        self.materials = materials if materials is not None else Materials(device=device)
        self.cameras = cameras
        self.blend_params = blend_params if blend_params is not None else BlendParams()

    def to(self, device):
        self.cameras = None if self.cameras is None else self.cameras.to(device)
        self.materials = self.materials.to(device)
        self.lights = self.lights.to(device)
        return self

    def _shade(self, fragments, meshes, kwargs):
        cameras = kwargs.get("cameras", self.cameras)
        if cameras is None:
            raise ValueError(f"Cameras must be specified either at initialization or in the forward pass of "
                             f"{type(self).__name__}")
        lights = kwargs.get("lights", self.lights)
        materials = kwargs.get("materials", self.materials)
        return cameras, textured_phong_shading(meshes, fragments, lights, cameras, materials)


class HardPhongShader(_ShaderBase):
    """Phong-lit nearest face, background elsewhere (PyTorch3D HardPhongShader)."""

    def forward(self, fragments, meshes, **kwargs):
        _, colors = self._shade(fragments, meshes, kwargs)
        return hard_rgb_blend(colors, fragments, kwargs.get("blend_params", self.blend_params))


class SoftPhongShader(_ShaderBase):
    """Phong-lit SoftRas softmax blend (PyTorch3D SoftPhongShader)."""

    def forward(self, fragments, meshes, **kwargs):
        cameras, colors = self._shade(fragments, meshes, kwargs)
        znear = kwargs.get("znear", getattr(cameras, "znear", 1.0))
        zfar = kwargs.get("zfar", getattr(cameras, "zfar", 100.0))
        shape = lambda z: z[:, None, None, None] if torch.is_tensor(z) and z.dim() == 1 else z
        return softmax_rgb_blend(colors, fragments, kwargs.get("blend_params", self.blend_params),
                                 znear=shape(znear), zfar=shape(zfar))


class SoftSilhouetteShader(nn.Module):
    """Sigmoid silhouette (PyTorch3D SoftSilhouetteShader)."""

    def __init__(self, blend_params=None):
        super().__init__()
        self.blend_params = blend_params if blend_params is not None else BlendParams()

    def forward(self, fragments, meshes, **kwargs):
        colors = torch.ones_like(fragments.bary_coords)
        return sigmoid_alpha_blend(colors, fragments, kwargs.get("blend_params", self.blend_params))
