"""UV-mapped and per-face-atlas textures with PyTorch3D 0.4.0 semantics, plus the
deprecated ``Textures`` wrapper that experiments/eval.py:755 still calls.

These are colour producers for the shaders, not the
perturbed hot path: sampling is a torch gather / ``grid_sample`` on the device the
mesh lives on.  Parity with PyTorch3D is unpinned (PyTorch3D is neither vendored nor
installable here); the conventions below are PyTorch3D's documented ones.
"""
import torch
import torch.nn.functional as F

from .interp import interpolate_face_attributes
from .mesh import TexturesVertex


def _listify(x):
    if x is None:
        return None
    if torch.is_tensor(x):
        return [t for t in x]
    return list(x)


class TexturesUV:
    """maps (N,H,W,C) sampled at per-face-corner UVs (faces_uvs (N,F,3) into verts_uvs
    (N,T,2)).  UV (0,0) is the bottom-left of the map, so the map is flipped vertically
    before ``grid_sample``; ``align_corners`` / ``padding_mode`` as PyTorch3D's
    TexturesUV defaults (True, "border")."""

    def __init__(self, maps, faces_uvs, verts_uvs, padding_mode="border", align_corners=True):
        self._maps = _listify(maps)
        self._faces_uvs = _listify(faces_uvs)
        self._verts_uvs = _listify(verts_uvs)
        if not (len(self._maps) == len(self._faces_uvs) == len(self._verts_uvs)):
            raise ValueError("maps, faces_uvs and verts_uvs must have the same batch size")
        self.padding_mode, self.align_corners = padding_mode, align_corners

    def maps_padded(self):
        if len(self._maps) == 1:  # a view: no copy of the map per render (gradients flow through it)
            return self._maps[0].unsqueeze(0)
        return torch.stack(self._maps, 0)

    def faces_uvs_list(self):
        return self._faces_uvs

    def verts_uvs_list(self):
        return self._verts_uvs

    def faces_verts_uvs_packed(self):
        """(F,3,2) per-face-corner UVs.  Without gradients on the UVs the gather is kept on the
        object, keyed by the UV tensors' identities and versions (an in-place edit misses): a
        render per step then launches no gather / concatenation kernels for constant UVs.  The
        returned tensor is shared between calls: treat it as read-only."""
        srcs = self._verts_uvs + self._faces_uvs
        if any(t.requires_grad for t in srcs):
            return torch.cat([vu[fu] for vu, fu in zip(self._verts_uvs, self._faces_uvs)], 0)
        key = tuple((id(t), t._version) for t in srcs)
        hit = getattr(self, "_fvu_cache", None)
        if hit is None or hit[0] != key:
            out = torch.cat([vu[fu] for vu, fu in zip(self._verts_uvs, self._faces_uvs)], 0)
            self._fvu_cache = hit = (key, out, srcs)  # (srcs held: their ids are not reused)
        return hit[1]

    def fusable(self):
        """The native shading kernel samples these maps itself: bilinear, align_corners, border
        padding, one map size, UVs without gradient (the maps may require one)."""
        return (self.align_corners and self.padding_mode == "border"
                and len({tuple(m.shape) for m in self._maps}) == 1
                and not any(t.requires_grad for t in self._verts_uvs))

    def sample_textures(self, fragments, faces_packed=None, **kwargs):
        p2f, bary = fragments.pix_to_face, fragments.bary_coords
        uv = interpolate_face_attributes(p2f, bary, self.faces_verts_uvs_packed().to(bary.device))
        N, Ho, Wo, K = p2f.shape
        maps = self.maps_padded().to(bary.device)
        C = maps.shape[-1]
        # one (Ho, Wo*K) sampling grid per mesh: every (pixel, slot) is an independent bilinear
        # lookup, so the map is read in place instead of being replicated K times
        uv = uv.reshape(N, Ho, Wo * K, 2) * 2.0 - 1.0
        m = torch.flip(maps.permute(0, 3, 1, 2), [2])  # v = 0 is the bottom row of the image
        tex = F.grid_sample(m, uv, align_corners=self.align_corners, padding_mode=self.padding_mode)
        return tex.reshape(N, C, Ho, Wo, K).permute(0, 2, 3, 4, 1)

    def extend(self, N):
        rep = lambda lst: [t for t in lst for _ in range(N)]
        return TexturesUV(rep(self._maps), rep(self._faces_uvs), rep(self._verts_uvs), self.padding_mode,
                          self.align_corners)

    def clone(self):
        return TexturesUV([t.clone() for t in self._maps], [t.clone() for t in self._faces_uvs],
                          [t.clone() for t in self._verts_uvs], self.padding_mode, self.align_corners)

    def detach(self):
        return TexturesUV([t.detach() for t in self._maps], self._faces_uvs, self._verts_uvs, self.padding_mode,
                          self.align_corners)

    def to(self, device):
        return TexturesUV([t.to(device) for t in self._maps], [t.to(device) for t in self._faces_uvs],
                          [t.to(device) for t in self._verts_uvs], self.padding_mode, self.align_corners)


class TexturesAtlas:
    """Per-face R x R texel grids (N list of (F,R,R,C)).  A fragment's barycentric
    (w0, w1) picks texel (floor(w1 R), floor(w0 R)) of its face, reflected into the
    lower triangle of the grid when it falls above the diagonal (PyTorch3D's atlas
    lookup)."""

    def __init__(self, atlas):
        self._atlas = _listify(atlas)

    def atlas_packed(self):
        return torch.cat(self._atlas, 0)

    def sample_textures(self, fragments, faces_packed=None, **kwargs):
        p2f, bary = fragments.pix_to_face, fragments.bary_coords
        atlas = self.atlas_packed().to(bary.device)
        R = atlas.shape[1]
        w01 = bary[..., :2].clamp(0.0, 1.0)
        wxy = (w01 * R).to(torch.int64).clamp(max=R - 1)
        wx, wy = wxy.unbind(-1)
        below = (w01.sum(-1) * R - wxy.to(bary.dtype).sum(-1)) <= 1.0
        wx = torch.where(below, wx, R - 1 - wx)
        wy = torch.where(below, wy, R - 1 - wy)
        f = p2f.clamp(min=0)
        tex = atlas[f, wy, wx]
        return tex * (p2f >= 0)[..., None].to(tex.dtype)

    def extend(self, N):
        return TexturesAtlas([t for t in self._atlas for _ in range(N)])

    def clone(self):
        return TexturesAtlas([t.clone() for t in self._atlas])

    def detach(self):
        return TexturesAtlas([t.detach() for t in self._atlas])

    def to(self, device):
        return TexturesAtlas([t.to(device) for t in self._atlas])


def Textures(maps=None, faces_uvs=None, verts_uvs=None, verts_rgb=None):
    """PyTorch3D 0.4.0's deprecated ``Textures(...)`` wrapper: UV maps when ``maps`` is
    given, per-vertex colours when ``verts_rgb`` is."""
    if maps is not None:
        if faces_uvs is None or verts_uvs is None:
            raise ValueError("Textures(maps=...) needs faces_uvs and verts_uvs")
        return TexturesUV(maps, faces_uvs, verts_uvs)
    if verts_rgb is not None:
        return TexturesVertex(verts_rgb)
    raise ValueError("Textures: give maps (+ uvs) or verts_rgb")
