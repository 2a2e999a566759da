"""Shader plugins and the blend — the reference's ``randomras.random_rasterizer`` surface.

``smooth_rgb_blend`` has the signature and outputs of random_rasterizer.py:34-56.
When it is handed a (GaussianRast, GaussianAgg) pair it runs ONE fused native
kernel pair (pr_blend_fwd/bwd) instead of the two-call split; any other pair goes
through the two duck-typed methods ``smoothrast.rasterize`` / ``smoothagg.aggregate``
exactly as the reference composes them.

RandomSimpleShader / RandomPhongShader (random_rasterizer.py:60-191) are
``MeshRenderer`` shaders with the same constructor arguments, attributes and
smoothing mutators.  SimpleShader / SoftSimpleShader (random_rasterizer.py:194-214)
wrap the hard / softmax blends.
"""
import os

import torch
import torch.nn as nn

from . import blend as _blend
from . import multidevice as _multidevice
from . import noise as _noise
from . import variants as _variants
from .renderer.cameras import OpenGLPerspectiveCameras, look_at_view_transform
from .renderer.blending import hard_rgb_blend, sigmoid_alpha_blend, softmax_rgb_blend  # noqa: F401
from .renderer.mesh import TexturesVertex
from .renderer.renderer import BlendParams, Materials, PointLights
from .renderer.shading import phong_inputs, phong_shading, textured_phong_shading  # noqa: F401
from .smoothagg import GaussianAgg, SoftAgg, _PerturbedAgg
from .smoothrast import GaussianRast, SoftRast, _PerturbedRast


def _is_fusable(smoothrast, smoothagg, fragments):
    """A native Monte-Carlo (rast, agg) pair on the GPU: fused into one pr_blend launch."""
    return (isinstance(smoothrast, _PerturbedRast) and isinstance(smoothagg, _PerturbedAgg)
            and fragments.pix_to_face.is_cuda)


def _variant_kw(smoothrast, smoothagg):
    return dict(rast_kind=smoothrast.noise_kind, rast_vr=smoothrast.variance_reduction,
                agg_kind=smoothagg.noise_kind, agg_vr=smoothagg.variance_reduction)


_BG_CACHE = {}


def _background_tensor(bg, device):
    """blend_params.background_color as a device tensor, made once per (value, device): no host
    copy per render (and none inside a captured graph)."""
    if torch.is_tensor(bg):
        return bg.to(device)
    key = (tuple(float(v) for v in bg), str(device))
    t = _BG_CACHE.get(key)
    if t is None:
        t = _BG_CACHE[key] = torch.tensor(key[0], dtype=torch.float32, device=device)
    return t


def _bg_needs_grad(bg):
    """A background colour tensor that requires grad: the reference's colour mix differentiates it
    (random_rasterizer.py:39-43, 52); the native kernels take it as constants, so such calls take
    the composition below (native rasterize / aggregate, torch colour mix)."""
    return torch.is_tensor(bg) and bg.requires_grad and torch.is_grad_enabled()


def smooth_rgb_blend(colors, fragments, smoothrast, smoothagg, blend_params, znear=1.0, zfar=100, live_only=False):
    """(N,H,W,K,3) colours + Fragments -> (N,H,W,4) RGBA (random_rasterizer.py:34-56).  live_only (an
    extension, RandomPhongShader's): every consumer of the colours' and fragments' gradients reads the
    valid prefix only, so the native backward leaves the masked slots' zero rows unwritten."""
    N, H, W, K = fragments.pix_to_face.shape
    device = fragments.pix_to_face.device
    background = blend_params.background_color
    bg_grad = _bg_needs_grad(background)
    if _is_fusable(smoothrast, smoothagg, fragments) and not bg_grad:
        if _multidevice.sample_devices() is not None and _noise.get_noise_source() == "philox":
            # samples split over the devices of set_sample_devices (in-process RCCL collectives)
            zbuf, _ = _blend.plane_link(fragments.zbuf, znear, zfar, fragments.pix_to_face)
            return _multidevice.sharded_blend(
                colors, fragments.pix_to_face, fragments.dists, zbuf, smoothrast.sigma,
                smoothagg.gamma, smoothagg.alpha, smoothrast.nb_samples, smoothagg.nb_samples,
                eps=smoothagg.eps, background=background, znear=znear, zfar=zfar,
                fixed_noise=smoothagg.fixed_noise, **_variant_kw(smoothrast, smoothagg))
        return _blend.perturbed_blend(
            colors, fragments.pix_to_face, fragments.dists, fragments.zbuf, smoothrast.sigma,
            smoothagg.gamma, smoothagg.alpha, smoothrast.nb_samples, smoothagg.nb_samples,
            eps=smoothagg.eps, background=background, znear=znear, zfar=zfar,
            fixed_noise=smoothagg.fixed_noise, live_only=live_only, **_variant_kw(smoothrast, smoothagg))
    if type(smoothrast) is SoftRast and type(smoothagg) is SoftAgg and fragments.pix_to_face.is_cuda and not bg_grad:
        # eval.py's "softras" pair as one native kernel pair (PR_BLEND_SOFT)
        return _blend.soft_blend(colors, fragments.pix_to_face, fragments.dists, fragments.zbuf, smoothrast.sigma,
                                 smoothagg.gamma, smoothagg.alpha, eps=smoothagg.eps, background=background,
                                 znear=znear, zfar=zfar)
    background = _background_tensor(background, device)
    mask = fragments.pix_to_face >= 0
    prob_map = smoothrast.rasterize(fragments.dists) * mask
    alpha_chan = _variants.prod_last(1.0 - prob_map)  # torch.prod(., dim=-1), capture-safe backward
    weights = smoothagg.aggregate(fragments.zbuf, zfar, znear, prob_map, mask)
    rgb = (weights[..., :-1, None] * colors).sum(dim=-2) + weights[..., -1:] * background
    return torch.cat([rgb, (1.0 - alpha_chan)[..., None]], dim=-1)


# RandomSimpleShader fuses TexturesVertex sampling into the blend on the GPU (set
# False to sample texels first; results are bit-identical, see tests/test_gpu_fused_texture.py)
FUSE_VERTEX_TEXTURES = True
# RandomPhongShader fuses the Phong shading (TexturesUV / TexturesVertex) into the blend on the GPU
# (set False to shade every slot first: pr_shade_* then the texel blend; the image is bit-identical,
# gradients agree to float-atomic order, tests/test_gpu_phong_fused.py)
FUSE_PHONG = os.environ.get("PR_FUSE_PHONG", "1") != "0"


def _vertex_colors(meshes):
    """Packed (V,3) per-vertex colours when the mesh's texture is a 3-channel
    TexturesVertex on the GPU (the fused-sampling case), else None."""
    tex = getattr(meshes, "textures", None)
    if not FUSE_VERTEX_TEXTURES or not isinstance(tex, TexturesVertex):
        return None
    vc = tex.verts_features_packed()
    return vc if vc.is_cuda and vc.dim() == 2 and vc.shape[-1] == 3 else None


def _planes_from(cameras, kwargs):
    znear = kwargs.get("znear", getattr(cameras, "znear", 1.0))
    zfar = kwargs.get("zfar", getattr(cameras, "zfar", 100.0))
    shape = lambda z: z[:, None, None, None] if torch.is_tensor(z) and z.dim() == 1 else z
    return shape(znear), shape(zfar)


class _RandomShaderBase(nn.Module):
    def get_smoothing(self):
        return self.smoothrast.sigma, self.smoothagg.gamma, self.smoothagg.alpha

    def get_nb_samples(self):
        return self.smoothagg.nb_samples

    def update_smoothing(self, sigma=4e-4, gamma=4e-2, alpha=1.0):
        self.smoothrast.update_smoothing(sigma)
        self.smoothagg.update_smoothing(gamma, alpha)

    def update_nb_samples(self, nb_samples=16):
        self.smoothrast.update_nb_samples(nb_samples)
        self.smoothagg.update_nb_samples(nb_samples)


class RandomPhongShader(_RandomShaderBase):
    """Phong-lit texels blended with the perturbed operators (random_rasterizer.py:60-130)."""

    def __init__(self, device="cpu", cameras=None, lights=None, materials=None, smoothrast=SoftRast(),
                 smoothagg=SoftAgg(), blend_params=None):
        super().__init__()
        self.lights = lights if lights is not None else PointLights(device=device)
        self.materials = materials if materials is not None else Materials(device=device)
        self.cameras = cameras
        self.blend_params = blend_params if blend_params is not None else BlendParams()
        self.smoothrast = smoothrast
        self.smoothagg = smoothagg

    def to(self, device):
        self.cameras = self.cameras.to(device)
        self.materials = self.materials.to(device)
        self.lights = self.lights.to(device)
        return self

    def takes_valid_only(self, meshes, **kwargs):
        """True when forward() reads each pixel's valid prefix only (MeshRenderer then rasterizes
        without writing the padding): a native blend, and the native live-only shading of a
        TexturesUV (one map size, 3 channels) or 3-channel TexturesVertex mesh on the GPU."""
        from .renderer.shading import _native_ok_params
        from .renderer.textures import TexturesUV
        if not meshes.verts_packed().is_cuda:
            return False
        native_blend = ((isinstance(self.smoothrast, _PerturbedRast) and isinstance(self.smoothagg, _PerturbedAgg)
                         and _multidevice.sample_devices() is None)
                        or (type(self.smoothrast) is SoftRast and type(self.smoothagg) is SoftAgg))
        if not native_blend or kwargs.get("cameras", self.cameras) is None:
            return False
        if _bg_needs_grad(kwargs.get("blend_params", self.blend_params).background_color):
            return False  # the composition path reads every slot
        if not _native_ok_params(kwargs.get("lights", self.lights), kwargs.get("materials", self.materials)):
            return False
        tex = getattr(meshes, "textures", None)
        if isinstance(tex, TexturesUV):
            if not tex.fusable():
                return False
            maps = tex.maps_padded()
            return maps.shape[0] == len(meshes) and maps.shape[-1] == 3
        if isinstance(tex, TexturesVertex):
            vc = tex.verts_features_packed()
            return vc.dim() == 2 and vc.shape[-1] == 3
        return False

    def forward(self, fragments, meshes, **kwargs):
        cameras = kwargs.get("cameras", self.cameras)
        if cameras is None:
            raise ValueError("Cameras must be specified either at initialization or in the forward "
                             "pass of RandomPhongShader")
        lights = kwargs.get("lights", self.lights)
        materials = kwargs.get("materials", self.materials)
        blend_params = kwargs.get("blend_params", self.blend_params)
        # texels = meshes.sample_textures(fragments); colors = phong_shading(..., texels) -- one
        # native kernel pair for TexturesUV / TexturesVertex (renderer/shading.py)
        # the native blends read a pixel's valid prefix only (the rasterizer's counts): the shading
        # then leaves the padded slots' colours (and their d bary) unwritten -- but only when
        # MeshRenderer says the fragments' sole consumer is its own rasterizer backward
        # (_pr_valid_only, takes_valid_only).  A direct shader(fragments, mesh) call gets the
        # reference's zero rows in d dists / d zbuf / d bary (random_rasterizer.py:46-47).
        live_only = bool(kwargs.get("_pr_valid_only", False)) and not _bg_needs_grad(blend_params.background_color) and (
            (_is_fusable(self.smoothrast, self.smoothagg, fragments) and _multidevice.sample_devices() is None)
            or (type(self.smoothrast) is SoftRast and type(self.smoothagg) is SoftAgg
                and fragments.pix_to_face.is_cuda))
        znear, zfar = _planes_from(cameras, kwargs)
        sr, sa = self.smoothrast, self.smoothagg
        if (FUSE_PHONG and _is_fusable(sr, sa, fragments) and _multidevice.sample_devices() is None
                and not _bg_needs_grad(blend_params.background_color)):
            # the shading fused into the blend's forward (PR_BLEND_PHONG): a slot is shaded only where
            # it wins a sample (no shading pass over every slot); the backward's shading chain rule
            # runs for those slots only (pr_shade_bwd skips zero d colours)
            sh = phong_inputs(meshes, fragments, lights, cameras, materials)
            if sh is not None:
                return _blend.perturbed_blend_phong(
                    sh, fragments.pix_to_face, fragments.bary_coords, fragments.dists, fragments.zbuf, sr.sigma,
                    sa.gamma, sa.alpha, sr.nb_samples, sa.nb_samples, eps=sa.eps,
                    background=blend_params.background_color, znear=znear, zfar=zfar, fixed_noise=sa.fixed_noise,
                    live_only=live_only, **_variant_kw(sr, sa))
        colors = textured_phong_shading(meshes, fragments, lights, cameras, materials, live_only=live_only)
        # (the blend's live-only backward also needs a live-only consumer of d colours: only when
        # the native shading ran live-only -- it marks its output -- are d colours read per live slot)
        return smooth_rgb_blend(colors, fragments, self.smoothrast, self.smoothagg, blend_params,
                                znear=znear, zfar=zfar, live_only=getattr(colors, "_pr_live_only", False))


class RandomSimpleShader(_RandomShaderBase):
    """Unlit texels blended with the perturbed operators (random_rasterizer.py:132-191)."""

    def __init__(self, device="cpu", cameras=None, lights=None, materials=None, smoothrast=SoftRast(),
                 smoothagg=SoftAgg(), blend_params=None):
        super().__init__()
        self.lights = lights if lights is not None else PointLights(device=device)
        self.materials = materials if materials is not None else Materials(device=device)
        if cameras is not None:
            self.cameras = cameras
        else:
            R, T = look_at_view_transform(dist=2.7, elev=torch.zeros((1)), azim=torch.zeros((1)))
            self.cameras = OpenGLPerspectiveCameras(device=device, R=R, T=T)
        self.blend_params = blend_params if blend_params is not None else BlendParams()
        self.smoothrast = smoothrast
        self.smoothagg = smoothagg

    def to(self, device):
        self.cameras = None if self.cameras is None else self.cameras.to(device)
        self.materials = self.materials.to(device)
        self.lights = None if self.lights is None else self.lights.to(device)
        return self

    def takes_valid_only(self, meshes, **kwargs):
        """True when forward() reads each pixel's valid prefix only: the TexturesVertex sampling
        fused into the native blend on one device (its gradients go to the rasterizer backward)."""
        return (_vertex_colors(meshes) is not None and isinstance(self.smoothrast, _PerturbedRast)
                and isinstance(self.smoothagg, _PerturbedAgg) and _multidevice.sample_devices() is None
                and kwargs.get("cameras", self.cameras) is not None
                and not _bg_needs_grad(kwargs.get("blend_params", self.blend_params).background_color))

    def forward(self, fragments, meshes, **kwargs):
        cameras = kwargs.get("cameras", self.cameras)
        if cameras is None:
            raise ValueError("Cameras must be specified either at initialization or in the forward "
                             "pass of RandomSimpleShader")
        blend_params = kwargs.get("blend_params", self.blend_params)
        znear, zfar = _planes_from(cameras, kwargs)
        vc = _vertex_colors(meshes)
        if (vc is not None and _is_fusable(self.smoothrast, self.smoothagg, fragments)
                and not _bg_needs_grad(blend_params.background_color)):
            # TexturesVertex sampling fused into the blend (no (N,H,W,K,3) texel tensor)
            sr, sa = self.smoothrast, self.smoothagg
            if _multidevice.sample_devices() is not None and _noise.get_noise_source() == "philox":
                # samples split over the devices of set_sample_devices (in-process RCCL collectives)
                zbuf, _ = _blend.plane_link(fragments.zbuf, znear, zfar, fragments.pix_to_face)
                return _multidevice.sharded_blend(
                    fragments.bary_coords, fragments.pix_to_face, fragments.dists, zbuf, sr.sigma,
                    sa.gamma, sa.alpha, sr.nb_samples, sa.nb_samples, eps=sa.eps,
                    background=blend_params.background_color, znear=znear, zfar=zfar, fixed_noise=sa.fixed_noise,
                    vert_colors=vc, faces=meshes.faces_packed(), **_variant_kw(sr, sa))
            # live_only (MeshRenderer's handshake only): the fragments' gradients go to the
            # rasterizer's backward, which reads each pixel's valid prefix only, so the masked slots'
            # zero rows are not written.  A direct call gets them written (smoothagg.py:198).
            return _blend.perturbed_blend_vertex(
                vc, meshes.faces_packed(), fragments.pix_to_face, fragments.bary_coords, fragments.dists,
                fragments.zbuf, sr.sigma, sa.gamma, sa.alpha, sr.nb_samples, sa.nb_samples, eps=sa.eps,
                background=blend_params.background_color, znear=znear, zfar=zfar, fixed_noise=sa.fixed_noise,
                live_only=bool(kwargs.get("_pr_valid_only", False)), **_variant_kw(sr, sa))
        texels = meshes.sample_textures(fragments)
        return smooth_rgb_blend(texels, fragments, self.smoothrast, self.smoothagg, blend_params,
                                znear=znear, zfar=zfar)


class SimpleShader(nn.Module):
    def __init__(self, device="cpu", blend_params=None):
        super().__init__()
        self.blend_params = blend_params if blend_params is not None else BlendParams()

    def forward(self, fragments, meshes, **kwargs):
        blend_params = kwargs.get("blend_params", self.blend_params)
        return hard_rgb_blend(meshes.sample_textures(fragments), fragments, blend_params)


class SoftSimpleShader(nn.Module):
    def __init__(self, device="cpu", blend_params=None):
        super().__init__()
        self.blend_params = blend_params if blend_params is not None else BlendParams()

    def forward(self, fragments, meshes, **kwargs):
        blend_params = kwargs.get("blend_params", self.blend_params)
        return softmax_rgb_blend(meshes.sample_textures(fragments), fragments, blend_params)
