"""Phong shading of per-slot texels (PyTorch3D 0.4.0 phong_shading, used by RandomPhongShader at
random_rasterizer.py:103-110 and HardPhongShader for eval.py's targets).

On ROCm tensors the whole per-slot computation -- position / normal interpolation, the texel
lookup (TexturesUV bilinear map sampling, TexturesVertex interpolation, or given texels), the
point / directional light terms and the specular highlight -- runs as one native kernel pair
(pr_shade_fwd / pr_shade_bwd, csrc/pr_shade.hip) instead of ~60 elementwise torch kernels over
(N,H,W,K,3) tensors.  Gradients reach the barycentrics (-> rasterizer), the vertex positions and
normals, vertex colours / UV maps, the light position and the camera centre (eval.py's
check_differentiability flows).  ``phong_shading_reference`` is the torch composition of the same
formulas (PyTorch3D's op order); it serves inputs the kernel does not cover (gradients w.r.t. the
light / material colours) and is the tests' reference.
"""
import collections

import torch
import torch.nn.functional as Fn

from .. import _native as nat
from .. import host_layer
from .interp import interpolate_vertex_attributes
from .mesh import TexturesVertex

F32 = torch.float32


def _bc(t, like):
    """(N,C) / (N,) per-batch parameters broadcast against (N,H,W,K,...) tensors."""
    t = t.to(like.device)
    if t.dim() == 2:
        return t.reshape((t.shape[0],) + (1,) * (like.dim() - 2) + (t.shape[-1],))
    return t.reshape((t.shape[0],) + (1,) * (like.dim() - 2))


def _is_directional(lights):
    from .renderer import DirectionalLights
    return isinstance(lights, DirectionalLights)


# ------------------------------------------------------------ torch composition
def _diffuse(normals, color, direction):
    n = Fn.normalize(normals, p=2, dim=-1, eps=1e-6)
    d = Fn.normalize(direction, p=2, dim=-1, eps=1e-6)
    angle = Fn.relu(torch.sum(n * d, dim=-1))
    return _bc(color, normals) * angle[..., None]


def _specular(points, normals, direction, camera_position, color, shininess):
    n = Fn.normalize(normals, p=2, dim=-1, eps=1e-6)
    d = Fn.normalize(direction, p=2, dim=-1, eps=1e-6)
    cos_angle = torch.sum(n * d, dim=-1)
    mask = (cos_angle > 0).to(torch.float32)
    view = Fn.normalize(_bc(camera_position, points) - points, p=2, dim=-1, eps=1e-6)
    reflect = -d + 2 * (cos_angle[..., None] * n)
    alpha = Fn.relu(torch.sum(view * reflect, dim=-1)) * mask
    return _bc(color, points) * torch.pow(alpha, _bc(shininess, alpha))[..., None]


def phong_shading_reference(meshes, fragments, lights, cameras, materials, texels):
    """PyTorch3D phong_shading as torch ops: (ambient + diffuse) * texels + specular."""
    verts = meshes.verts_packed()
    faces = meshes.faces_packed()
    vnormals = meshes.verts_normals_packed()
    coords = interpolate_vertex_attributes(fragments.pix_to_face, fragments.bary_coords, verts, faces)
    normals = interpolate_vertex_attributes(fragments.pix_to_face, fragments.bary_coords, vnormals, faces)
    N = coords.shape[0]
    expand = lambda t: t.expand(N, -1) if t.shape[0] == 1 else t
    if _is_directional(lights):
        direction = _bc(expand(lights.location), coords).expand_as(coords)
    else:
        direction = _bc(expand(lights.location), coords) - coords
    diffuse = _diffuse(normals, expand(lights.diffuse_color), direction)
    specular = _specular(coords, normals, direction, expand(cameras.get_camera_center()),
                         expand(lights.specular_color), expand(materials.shininess.reshape(-1)))
    ambient = _bc(expand(materials.ambient_color * lights.ambient_color), coords)
    diffuse = _bc(expand(materials.diffuse_color), coords) * diffuse
    specular = _bc(expand(materials.specular_color), coords) * specular
    return (ambient + diffuse) * texels + specular


# ------------------------------------------------------------------ native path
class _ShadeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, bary, verts, normals, tex, light, camera, cfg):
        nat.require_device(bary, verts, normals, tex, light, camera)
        N, H, W, K = cfg["p2f"].shape
        keep = dict(bary=nat.dense(bary, F32), verts=nat.dense(verts, F32),
                    normals=nat.dense(normals, F32), tex=nat.dense(tex, F32),
                    light=nat.dense(light, F32), camera=nat.dense(camera, F32))
        colors = torch.empty((N, H, W, K, 3), dtype=F32, device=bary.device)
        a = _args(cfg, keep)
        a.colors = nat.ptr(colors)
        nat.call("pr_shade_fwd", "pr_shade_fwd", colors, a)
        ctx.save_for_backward(*keep.values())
        ctx.cfg = cfg
        return colors

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gcol):
        bary, verts, normals, tex, light, camera = ctx.saved_tensors
        keep = dict(bary=bary, verts=verts, normals=normals, tex=tex, light=light, camera=camera)
        cfg = ctx.cfg
        lib = nat.load()
        need = ctx.needs_input_grad
        g = nat.dense(gcol, F32)
        a = _args(cfg, keep)
        a.grad_colors = nat.ptr(g)
        out = [torch.empty_like(t) if need[i] else None
               for i, t in enumerate((bary, verts, normals, tex, light, camera))]
        gb, gv, gn, gt, gl, gc = out
        a.grad_bary, a.grad_verts, a.grad_normals = nat.ptr(gb), nat.ptr(gv), nat.ptr(gn)
        if cfg["mode"] == nat.PR_TEX_GIVEN:
            a.grad_texels = nat.ptr(gt)
        elif cfg["mode"] == nat.PR_TEX_VERTEX:
            a.grad_vert_colors = nat.ptr(gt)
        else:
            a.grad_maps = nat.ptr(gt)
        a.grad_light, a.grad_camera = nat.ptr(gl), nat.ptr(gc)
        ws = None
        if nat.deterministic():  # torch.use_deterministic_algorithms: in-order sums, no float atomics
            a.flags |= nat.PR_DETERMINISTIC
            ws = nat.workspace(lib.pr_shade_bwd_workspace_size(a), g.device)
            a.workspace, a.workspace_bytes = nat.ptr(ws), ws.numel()
        nat.call("pr_shade_bwd", "pr_shade_bwd", g, a)
        del ws
        return gb, gv, gn, gt, gl, gc, None


def _shade_bwd_args(a, mode, gcol, out):
    """Point the PRShadeArgs `a` at d colours `gcol` and the outputs out = [d bary, d verts,
    d normals, d texels / vertex colours / maps, d light, d camera] (None: not wanted)."""
    gb, gv, gn, gt, gl, gc = out
    a.grad_colors = nat.ptr(gcol)
    a.grad_bary, a.grad_verts, a.grad_normals = nat.ptr(gb), nat.ptr(gv), nat.ptr(gn)
    if mode == nat.PR_TEX_GIVEN:
        a.grad_texels = nat.ptr(gt)
    elif mode == nat.PR_TEX_VERTEX:
        a.grad_vert_colors = nat.ptr(gt)
    else:
        a.grad_maps = nat.ptr(gt)
    a.grad_light, a.grad_camera = nat.ptr(gl), nat.ptr(gc)
    return a


def _args(cfg, t):
    a = nat.PRShadeArgs()
    N, H, W, K = cfg["p2f"].shape
    a.N, a.H, a.W, a.K = N, H, W, K
    a.pix_to_face, a.pix_count, a.faces = nat.ptr(cfg["p2f"]), nat.ptr(cfg["counts"]), nat.ptr(cfg["faces"])
    a.bary, a.verts, a.normals = nat.ptr(t["bary"]), nat.ptr(t["verts"]), nat.ptr(t["normals"])
    a.V, a.F = t["verts"].shape[0], cfg["faces"].shape[0]
    a.texture = cfg["mode"]
    if cfg["mode"] == nat.PR_TEX_GIVEN:
        a.texels = nat.ptr(t["tex"])
    elif cfg["mode"] == nat.PR_TEX_VERTEX:
        a.vert_colors = nat.ptr(t["tex"])
    else:
        a.maps, a.face_uvs = nat.ptr(t["tex"]), nat.ptr(cfg["face_uvs"])
        a.Hm, a.Wm = t["tex"].shape[1], t["tex"].shape[2]
    a.directional = int(cfg["directional"])
    a.flags = nat.PR_SHADE_LIVE_ONLY if cfg.get("live_only") and cfg["counts"] is not None else 0
    a.light, a.camera = nat.ptr(t["light"]), nat.ptr(t["camera"])
    for k in ("ambient", "diffuse_color", "specular_color", "mat_diffuse", "mat_specular", "shininess"):
        setattr(a, k, nat.ptr(cfg[k]))
    return a


def _rows(t, N, device):
    """(1|N, C) or (1|N,) -> contiguous (N, C) / (N,) float32 rows on `device`."""
    t = t.to(device=device, dtype=F32)
    t = t.reshape(t.shape[0], -1) if t.dim() >= 1 else t.reshape(1, 1)
    if t.shape[0] == 1:
        t = t.expand(N, t.shape[1])
    return t


_ROW_CACHE = collections.OrderedDict()
_ROW_CACHE_MAX = 32


def _param_rows(lights, materials, N, dev):
    """The six per-batch material / light colour rows of the shading kernel, made once per
    (source tensors and their versions, N, device): an eager step then launches no product / copy
    kernels for constant materials.  The sources (no gradient: _native_ok) are held by the entry,
    so their ids are not reused while it lives; an in-place change bumps a version and misses."""
    srcs = (materials.ambient_color, lights.ambient_color, lights.diffuse_color, lights.specular_color,
            materials.diffuse_color, materials.specular_color, materials.shininess)
    key = tuple((id(t), t._version) if torch.is_tensor(t) else ("v", float(t)) for t in srcs) + (N, str(dev))
    hit = _ROW_CACHE.get(key)
    if hit is not None:
        _ROW_CACHE.move_to_end(key)
        return hit[0]
    rows = lambda x: _rows(x, N, dev).contiguous()
    out = dict(ambient=rows(materials.ambient_color * lights.ambient_color),
               diffuse_color=rows(lights.diffuse_color), specular_color=rows(lights.specular_color),
               mat_diffuse=rows(materials.diffuse_color), mat_specular=rows(materials.specular_color),
               shininess=rows(materials.shininess.reshape(-1, 1)).reshape(N).contiguous())
    _ROW_CACHE[key] = (out, srcs)
    while len(_ROW_CACHE) > _ROW_CACHE_MAX:
        _ROW_CACHE.popitem(last=False)
    return out


def _native_ok_params(lights, materials):
    fixed = [lights.ambient_color, lights.diffuse_color, lights.specular_color, materials.ambient_color,
             materials.diffuse_color, materials.specular_color, materials.shininess]
    return not any(torch.is_tensor(x) and x.requires_grad for x in fixed)


def _native_ok(fragments, lights, materials):
    return fragments.pix_to_face.is_cuda and _native_ok_params(lights, materials)


def _shade_native(meshes, fragments, lights, cameras, materials, mode, tex, face_uvs=None, live_only=False):
    from .rasterizer import valid_counts
    p2f = fragments.pix_to_face
    N = p2f.shape[0]
    dev = p2f.device
    counts = valid_counts(p2f)
    if counts is not None and (counts.device != dev or tuple(counts.shape) != tuple(p2f.shape[:3])):
        counts = None
    verts = meshes.verts_packed()
    faces = meshes.faces_packed().to(torch.int64).contiguous()
    # live_only: the caller reads the valid prefix of the colours only (RandomPhongShader's native
    # blend with the counts), so the padded slots' colours and d bary are left unwritten
    live_only = bool(live_only) and counts is not None and mode != nat.PR_TEX_GIVEN
    cfg = dict(p2f=nat.dense(p2f, torch.int64), counts=counts, faces=faces, mode=mode, live_only=live_only,
               face_uvs=face_uvs, directional=_is_directional(lights), **_param_rows(lights, materials, N, dev))
    light = _rows(lights.location, N, dev)
    camera = _rows(cameras.get_camera_center(), N, dev)
    ext = host_layer.get()
    if ext is not None:  # the C++ autograd layer (host_layer.py): same kernel, same arguments
        out = ext.shade(fragments.bary_coords, verts, meshes.verts_normals_packed(), tex, light, camera, cfg["p2f"],
                        counts, faces, face_uvs,
                        [cfg[k] for k in ("ambient", "diffuse_color", "specular_color", "mat_diffuse", "mat_specular",
                                          "shininess")], int(mode), bool(cfg["directional"]), live_only)
    else:
        out = _ShadeFn.apply(fragments.bary_coords, verts, meshes.verts_normals_packed(), tex, light, camera, cfg)
    if live_only:
        out._pr_live_only = True  # padded colours unwritten; d colours read per live slot only
    return out


def phong_inputs(meshes, fragments, lights, cameras, materials):
    """The native shading's inputs for a TexturesUV (maps of one size, 3 channels) or 3-channel
    TexturesVertex mesh on the GPU with constant lights / materials -- what pr_shade_* and the blend's
    fused Phong colour mode (PR_BLEND_PHONG) take -- or None when the texture or parameters are
    outside the native path."""
    from .rasterizer import valid_counts
    from .textures import TexturesUV
    if not _native_ok(fragments, lights, materials):
        return None
    tex = getattr(meshes, "textures", None)
    p2f = fragments.pix_to_face
    N = p2f.shape[0]
    dev = p2f.device
    if isinstance(tex, TexturesUV) and tex.fusable():
        maps = tex.maps_padded().to(dev)
        if maps.shape[0] != N or maps.shape[-1] != 3:
            return None
        mode, texture = nat.PR_TEX_UV, maps
        face_uvs = tex.faces_verts_uvs_packed().to(device=dev, dtype=F32).detach().contiguous()
    elif isinstance(tex, TexturesVertex):
        vc = tex.verts_features_packed()
        if vc.dim() != 2 or vc.shape[-1] != 3:
            return None
        mode, texture, face_uvs = nat.PR_TEX_VERTEX, vc, None
    else:
        return None
    counts = valid_counts(p2f)
    if counts is not None and (counts.device != dev or tuple(counts.shape) != tuple(p2f.shape[:3])):
        counts = None
    return dict(mode=mode, tex=texture, face_uvs=face_uvs, verts=meshes.verts_packed(),
                normals=meshes.verts_normals_packed(), faces=meshes.faces_packed().to(torch.int64).contiguous(),
                light=_rows(lights.location, N, dev), camera=_rows(cameras.get_camera_center(), N, dev),
                rows=_param_rows(lights, materials, N, dev), directional=_is_directional(lights), counts=counts)


def phong_shading(meshes, fragments, lights, cameras, materials, texels):
    """PyTorch3D phong_shading(meshes, fragments, lights, cameras, materials, texels)."""
    if _native_ok(fragments, lights, materials):
        return _shade_native(meshes, fragments, lights, cameras, materials, nat.PR_TEX_GIVEN, texels)
    return phong_shading_reference(meshes, fragments, lights, cameras, materials, texels)


def textured_phong_shading(meshes, fragments, lights, cameras, materials, live_only=False):
    """phong_shading(..., texels=meshes.sample_textures(fragments)) with the texel lookup fused
    into the shading kernel for TexturesUV (maps of one size) and 3-channel TexturesVertex.
    live_only (an extension for callers that read the valid prefix only, with the rasterizer's
    counts attached): the padded slots' colours, and their d bary, are left unwritten."""
    from .textures import TexturesUV
    tex = getattr(meshes, "textures", None)
    if _native_ok(fragments, lights, materials):
        if isinstance(tex, TexturesUV) and tex.fusable():
            maps = tex.maps_padded().to(fragments.pix_to_face.device)
            if maps.shape[0] == fragments.pix_to_face.shape[0] and maps.shape[-1] == 3:
                fuv = tex.faces_verts_uvs_packed().to(device=maps.device, dtype=F32).detach().contiguous()
                return _shade_native(meshes, fragments, lights, cameras, materials, nat.PR_TEX_UV, maps, fuv,
                                     live_only=live_only)
        if isinstance(tex, TexturesVertex):
            vc = tex.verts_features_packed()
            if vc.dim() == 2 and vc.shape[-1] == 3:
                return _shade_native(meshes, fragments, lights, cameras, materials, nat.PR_TEX_VERTEX, vc,
                                     live_only=live_only)
    return phong_shading(meshes, fragments, lights, cameras, materials, meshes.sample_textures(fragments))
