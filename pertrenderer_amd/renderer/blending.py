"""PyTorch3D 0.4.0 blending functions used by the shaders around the perturbed path
(random_rasterizer.py:24-26 imports hard_rgb_blend / softmax_rgb_blend; eval.py renders
its targets with HardPhongShader, eval.py:265-283).  Elementwise torch code: these run
once per target image, not in the optimisation loop."""
import torch


def _bg(bg, like):
    return bg.to(like.device) if torch.is_tensor(bg) else torch.tensor(bg, dtype=like.dtype, device=like.device)


def hard_rgb_blend(colors, fragments, blend_params):
    """Nearest-face colour, background where no face covers the pixel (PyTorch3D hard_rgb_blend)."""
    N, H, W, K = fragments.pix_to_face.shape
    bg = blend_params.background_color
    bg = bg.to(colors.device) if torch.is_tensor(bg) else torch.tensor(bg, dtype=colors.dtype, device=colors.device)
    is_bg = (fragments.pix_to_face[..., 0] < 0)[..., None]
    rgb = torch.where(is_bg, bg.expand(N, H, W, 3), colors[..., 0, :])
    return torch.cat([rgb, (~is_bg).to(colors.dtype)], dim=-1)


def softmax_rgb_blend(colors, fragments, blend_params, znear=1.0, zfar=100):
    """SoftRas softmax blend (PyTorch3D softmax_rgb_blend)."""
    N, H, W, K = fragments.pix_to_face.shape
    bg = blend_params.background_color
    bg = bg.to(colors.device) if torch.is_tensor(bg) else torch.tensor(bg, dtype=colors.dtype, device=colors.device)
    mask = fragments.pix_to_face >= 0
    prob = torch.sigmoid(-fragments.dists / blend_params.sigma) * mask
    alpha = torch.prod(1.0 - prob, dim=-1)
    z_inv = (zfar - fragments.zbuf) / (zfar - znear) * mask
    z_inv_max = torch.max(z_inv, dim=-1).values[..., None].clamp(min=1e-10)
    w = prob * torch.exp((z_inv - z_inv_max) / blend_params.gamma)
    delta = torch.exp((1e-10 - z_inv_max) / blend_params.gamma).clamp(min=1e-10)
    denom = w.sum(dim=-1)[..., None] + delta
    rgb = ((w[..., None] * colors).sum(dim=-2) + delta * bg) / denom
    return torch.cat([rgb, (1.0 - alpha)[..., None]], dim=-1)


def sigmoid_alpha_blend(colors, fragments, blend_params):
    """Silhouette blend: rgb of the nearest face, alpha = 1 - prod_k(1 - sigmoid(-d_k / sigma))
    over the valid slots (PyTorch3D sigmoid_alpha_blend)."""
    N, H, W, K = fragments.pix_to_face.shape
    mask = fragments.pix_to_face >= 0
    prob = torch.sigmoid(-fragments.dists / blend_params.sigma) * mask
    alpha = 1.0 - torch.prod(1.0 - prob, dim=-1)
    return torch.cat([colors[..., 0, :], alpha[..., None]], dim=-1)
