"""MeshRenderer, BlendParams, lights and materials (PyTorch3D 0.4.0 surface used by
experiments/eval.py:36-48 and random_rasterizer.py:9-26)."""
from typing import NamedTuple, Sequence

import torch

F32 = torch.float32


class BlendParams(NamedTuple):
    sigma: float = 1e-4
    gamma: float = 1e-4
    background_color: Sequence = (1.0, 1.0, 1.0)


def _vec(v, device):
    t = v.to(device=device, dtype=F32) if torch.is_tensor(v) else torch.tensor(v, dtype=F32, device=device)
    return t.reshape(-1, 3) if t.numel() % 3 == 0 else t


class PointLights:
    def __init__(self, ambient_color=((0.5, 0.5, 0.5),), diffuse_color=((0.3, 0.3, 0.3),),
                 specular_color=((0.2, 0.2, 0.2),), location=((0, 1, 0),), device="cpu"):
        self.device = torch.device(device)
        self.ambient_color = _vec(ambient_color, self.device)
        self.diffuse_color = _vec(diffuse_color, self.device)
        self.specular_color = _vec(specular_color, self.device)
        self.location = _vec(location, self.device)

    def to(self, device):
        self.device = torch.device(device)
        for k in ("ambient_color", "diffuse_color", "specular_color", "location"):
            setattr(self, k, getattr(self, k).to(self.device))
        return self

    def light_direction(self, points):
        loc = self.location.reshape((-1,) + (1,) * (points.dim() - 2) + (3,))
        return torch.nn.functional.normalize(loc - points, dim=-1, eps=1e-6)


class DirectionalLights(PointLights):
    def __init__(self, ambient_color=((0.5, 0.5, 0.5),), diffuse_color=((0.3, 0.3, 0.3),),
                 specular_color=((0.2, 0.2, 0.2),), direction=((0, 1, 0),), device="cpu"):
        super().__init__(ambient_color, diffuse_color, specular_color, direction, device)

    def light_direction(self, points):
        d = self.location.reshape((-1,) + (1,) * (points.dim() - 2) + (3,))
        return torch.nn.functional.normalize(d, dim=-1, eps=1e-6).expand_as(points)


class Materials:
    def __init__(self, ambient_color=((1, 1, 1),), diffuse_color=((1, 1, 1),), specular_color=((1, 1, 1),),
                 shininess=64, device="cpu"):
        self.device = torch.device(device)
        self.ambient_color = _vec(ambient_color, self.device)
        self.diffuse_color = _vec(diffuse_color, self.device)
        self.specular_color = _vec(specular_color, self.device)
        self.shininess = torch.tensor([float(shininess)], dtype=F32, device=self.device)

    def to(self, device):
        self.device = torch.device(device)
        for k in ("ambient_color", "diffuse_color", "specular_color", "shininess"):
            setattr(self, k, getattr(self, k).to(self.device))
        return self


class MeshRenderer(torch.nn.Module):
    """fragments = rasterizer(meshes); images = shader(fragments, meshes)."""

    def __init__(self, rasterizer, shader):
        super().__init__()
        self.rasterizer = rasterizer
        self.shader = shader

    def to(self, device):
        self.rasterizer.to(device)
        self.shader.to(device)
        return self

    def forward(self, meshes_world, **kwargs):
        from .. import blend
        # the perturbed shaders' smoothing-scalar gradient link, made before the rasterizer's nodes
        # so that the backward's one host synchronisation comes after the rasterizer's backward is
        # launched (blend.prelink)
        token = blend.prelink_shader(self.shader, meshes_world)
        try:
            # a shader that reads each pixel's valid prefix only (the native perturbed shaders, when
            # every one of their consumers does) takes fragments whose padding is left unwritten
            takes = getattr(self.shader, "takes_valid_only", None)
            if takes is not None and takes(meshes_world, **kwargs):
                kwargs = dict(kwargs, _pr_valid_only=True)
            fragments = self.rasterizer(meshes_world, **kwargs)
            return self.shader(fragments, meshes_world, **kwargs)
        finally:
            blend.drop_prelink(token)
