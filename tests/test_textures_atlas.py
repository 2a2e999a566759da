"""TexturesAtlas.sample_textures (PyTorch3D 0.4.0's per-face R x R atlas lookup, the colour
producer eval.py's load_objs_as_meshes(create_texture_atlas=True) path feeds).
Known answers worked out by hand for R = 4: texel (x, y) = floor((w0, w1) * R), reflected to
(R-1-x, R-1-y) when (w0 + w1) * R - (x + y) > 1; padded slots give zeros.  PyTorch3D is not
vendored: parity unpinned beyond these hand-computed cases."""
import torch

from pertrenderer_amd.renderer import TexturesAtlas
from pertrenderer_amd.renderer.rasterizer import Fragments


def test_atlas_lookup_known_answers():
    R, F = 4, 2
    atlas = torch.arange(F * R * R * 3, dtype=torch.float32).reshape(F, R, R, 3)
    cases = [  # (face, (w0, w1, w2), (row y, col x)) by hand
        (0, (0.10, 0.20, 0.70), (3, 3)),  # x=0,y=0; 0.3*4 - 0 = 1.2 > 1: reflected
        (0, (0.10, 0.05, 0.85), (0, 0)),  # 0.15*4 = 0.6 <= 1: kept
        (1, (0.60, 0.20, 0.20), (3, 1)),  # x=2,y=0; 0.8*4 - 2 = 1.2 > 1: reflected to x=1, y=3
        (1, (0.30, 0.55, 0.15), (2, 1)),  # x=1,y=2; 0.85*4 - 3 = 0.4: kept
    ]
    K = len(cases) + 1
    p2f = torch.full((1, 1, 1, K), -1, dtype=torch.int64)
    bary = torch.full((1, 1, 1, K, 3), -1.0)
    for k, (f, w, _) in enumerate(cases):
        p2f[0, 0, 0, k] = f
        bary[0, 0, 0, k] = torch.tensor(w)
    frag = Fragments(pix_to_face=p2f, zbuf=torch.zeros_like(p2f, dtype=torch.float32), bary_coords=bary,
                     dists=torch.zeros_like(p2f, dtype=torch.float32))
    tex = TexturesAtlas([atlas]).sample_textures(frag)
    assert tex.shape == (1, 1, 1, K, 3)
    for k, (f, _, (y, x)) in enumerate(cases):
        torch.testing.assert_close(tex[0, 0, 0, k], atlas[f, y, x], rtol=0, atol=0)
    assert torch.equal(tex[0, 0, 0, K - 1], torch.zeros(3))  # padded slot


def test_atlas_constant_face_colours():
    """A face whose whole atlas is one colour renders that colour at every barycentric."""
    R = 3
    cols = torch.tensor([[1.0, 0.0, 0.0], [0.0, 0.5, 1.0]])
    atlas = cols[:, None, None, :].expand(2, R, R, 3).contiguous()
    g = torch.Generator().manual_seed(0)
    w = torch.rand((1, 4, 5, 6, 3), generator=g)
    w = w / w.sum(-1, keepdim=True)
    p2f = torch.randint(-1, 2, (1, 4, 5, 6), generator=g)
    frag = Fragments(pix_to_face=p2f, zbuf=torch.zeros(p2f.shape), bary_coords=w, dists=torch.zeros(p2f.shape))
    tex = TexturesAtlas([atlas]).sample_textures(frag)
    ref = torch.where((p2f >= 0)[..., None], cols[p2f.clamp(min=0)], torch.zeros(3))
    torch.testing.assert_close(tex, ref, rtol=0, atol=0)
