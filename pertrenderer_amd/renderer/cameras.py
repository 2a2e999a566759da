"""Perspective cameras with PyTorch3D 0.4.0 conventions (the subset eval.py uses).

Row-vector convention: X_view = X_world @ R + T; NDC = (X_view_h @ K^T)[:3] / w with
+X left, +Y up, z kept in view space by the rasterizer.  Used at
experiments/eval.py:249-263 (look_at_view_transform + OpenGLPerspectiveCameras) and
random_rasterizer.py:152-153 (the shader's default camera).
"""
import math

import torch
import torch.nn.functional as Fn

F32 = torch.float32


def _as_batch(*args, device="cpu"):
    ts = [a.to(device=device, dtype=F32) if torch.is_tensor(a) else torch.tensor(a, dtype=F32, device=device)
          for a in args]
    ts = [t.reshape(-1) if t.dim() <= 1 else t for t in ts]
    n = max(t.shape[0] for t in ts)
    return [t.expand(n) if t.shape[0] == 1 else t for t in ts]


def camera_position_from_spherical_angles(distance, elevation, azimuth, degrees=True, device="cpu"):
    dist, elev, azim = _as_batch(distance, elevation, azimuth, device=device)
    if degrees:
        elev = math.pi / 180.0 * elev
        azim = math.pi / 180.0 * azim
    x = dist * torch.cos(elev) * torch.sin(azim)
    y = dist * torch.sin(elev)
    z = dist * torch.cos(elev) * torch.cos(azim)
    return torch.stack([x, y, z], dim=1).view(-1, 3)


def look_at_rotation(camera_position, at=((0, 0, 0),), up=((0, 1, 0),), device="cpu"):
    C = camera_position if torch.is_tensor(camera_position) else torch.tensor(camera_position, dtype=F32)
    C = C.to(device=device, dtype=F32).reshape(-1, 3)
    at = torch.as_tensor(at, dtype=F32, device=device).reshape(-1, 3).expand(C.shape[0], 3)
    up = torch.as_tensor(up, dtype=F32, device=device).reshape(-1, 3).expand(C.shape[0], 3)
    z_axis = Fn.normalize(at - C, eps=1e-5)
    x_axis = Fn.normalize(torch.cross(up, z_axis, dim=1), eps=1e-5)
    y_axis = Fn.normalize(torch.cross(z_axis, x_axis, dim=1), eps=1e-5)
    is_close = torch.isclose(x_axis, torch.tensor(0.0, device=device), atol=5e-3).all(dim=1, keepdim=True)
    if is_close.any():
        replacement = Fn.normalize(torch.cross(y_axis, z_axis, dim=1), eps=1e-5)
        x_axis = torch.where(is_close, replacement, x_axis)
    R = torch.cat((x_axis[:, None, :], y_axis[:, None, :], z_axis[:, None, :]), dim=1)
    return R.transpose(1, 2)


def look_at_view_transform(dist=1.0, elev=0.0, azim=0.0, degrees=True, eye=None, at=((0, 0, 0),),
                           up=((0, 1, 0),), device="cpu"):
    """(R, T) of cameras on a sphere looking at `at` (PyTorch3D look_at_view_transform)."""
    if eye is not None:
        C = torch.as_tensor(eye, dtype=F32, device=device).reshape(-1, 3)
    else:
        C = camera_position_from_spherical_angles(dist, elev, azim, degrees=degrees, device=device)
    R = look_at_rotation(C, at, up, device=device)
    T = -torch.bmm(R.transpose(1, 2), C[:, :, None])[:, :, 0]
    return R, T


class Transform:
    """A batch of 4x4 row-vector transforms (points @ M)."""

    def __init__(self, matrix):
        self.matrix = matrix

    def compose(self, other):
        return Transform(torch.bmm(self.matrix, other.matrix))

    def transform_points(self, points, eps=None):
        N = points.shape[0] if points.dim() == 3 else 1
        pts = points if points.dim() == 3 else points[None]
        ones = torch.ones(pts.shape[:-1] + (1,), dtype=pts.dtype, device=pts.device)
        ph = torch.cat([pts, ones], dim=-1)
        M = self.matrix.to(pts.device)
        if M.shape[0] != ph.shape[0]:
            M = M.expand(ph.shape[0], 4, 4) if M.shape[0] == 1 else M
            ph = ph.expand(M.shape[0], -1, -1) if ph.shape[0] == 1 else ph
        out = torch.bmm(ph, M)
        denom = out[..., 3:]
        if eps is not None:
            sign = denom.sign() + (denom == 0.0).type_as(denom)
            denom = sign * torch.clamp(denom.abs(), eps)
        out = out[..., :3] / denom
        return out if points.dim() == 3 or N != 1 else out[0]


def _rotate(R):
    N = R.shape[0]
    M = torch.eye(4, dtype=F32, device=R.device).repeat(N, 1, 1)
    M[:, :3, :3] = R
    return Transform(M)


def _translate(T):
    N = T.shape[0]
    M = torch.eye(4, dtype=F32, device=T.device).repeat(N, 1, 1)
    M[:, 3, :3] = T
    return Transform(M)


class FoVPerspectiveCameras:
    """OpenGL-style perspective camera (PyTorch3D FoVPerspectiveCameras, fov in degrees)."""

    def __init__(self, znear=1.0, zfar=100.0, aspect_ratio=1.0, fov=60.0, degrees=True, R=None, T=None,
                 device="cpu"):
        self.device = torch.device(device)
        R = torch.eye(3, dtype=F32)[None] if R is None else R
        T = torch.zeros((1, 3), dtype=F32) if T is None else T
        self.R = R.to(self.device, F32)
        self.T = T.to(self.device, F32)
        N = max(self.R.shape[0], self.T.shape[0])
        self._N = N
        b = lambda v: (v.to(self.device, F32).reshape(-1) if torch.is_tensor(v)
                       else torch.tensor([float(v)], dtype=F32, device=self.device)).expand(N).clone()
        self.znear, self.zfar, self.aspect_ratio, self.fov = b(znear), b(zfar), b(aspect_ratio), b(fov)
        self.degrees = degrees

    def __len__(self):
        return self._N

    def to(self, device):
        self.device = torch.device(device)
        for k in ("R", "T", "znear", "zfar", "aspect_ratio", "fov"):
            setattr(self, k, getattr(self, k).to(self.device))
        return self

    def compute_projection_matrix(self, znear, zfar, fov, aspect_ratio, degrees):
        K = torch.zeros((self._N, 4, 4), device=self.device, dtype=F32)
        ones = torch.ones((self._N,), dtype=F32, device=self.device)
        if degrees:
            fov = (math.pi / 180) * fov
        tan_half = torch.tan(fov / 2)
        max_y = tan_half * znear
        min_y = -max_y
        max_x = max_y * aspect_ratio
        min_x = -max_x
        K[:, 0, 0] = 2.0 * znear / (max_x - min_x)
        K[:, 1, 1] = 2.0 * znear / (max_y - min_y)
        K[:, 0, 2] = (max_x + min_x) / (max_x - min_x)
        K[:, 1, 2] = (max_y + min_y) / (max_y - min_y)
        K[:, 3, 2] = ones
        K[:, 2, 2] = zfar / (zfar - znear)
        K[:, 2, 3] = -(zfar * znear) / (zfar - znear)
        return K

    def get_projection_transform(self, **kwargs):
        K = self.compute_projection_matrix(kwargs.get("znear", self.znear), kwargs.get("zfar", self.zfar),
                                           kwargs.get("fov", self.fov),
                                           kwargs.get("aspect_ratio", self.aspect_ratio),
                                           kwargs.get("degrees", self.degrees))
        return Transform(K.transpose(1, 2).contiguous())

    def get_world_to_view_transform(self, **kwargs):
        R = kwargs.get("R", self.R)
        T = kwargs.get("T", self.T)
        return _rotate(R).compose(_translate(T))

    def get_full_projection_transform(self, **kwargs):
        return self.get_world_to_view_transform(**kwargs).compose(self.get_projection_transform(**kwargs))

    def transform_points(self, points, eps=None, **kwargs):
        return self.get_full_projection_transform(**kwargs).transform_points(points, eps=eps)

    # -- cached (N,4,4) matrices for the native projection path -------------------
    _PARAMS = ("R", "T", "znear", "zfar", "aspect_ratio", "fov")

    def matrices_need_grad(self):
        return any(getattr(self, k).requires_grad for k in self._PARAMS)

    def _cached(self, slot, key_names, build):
        key = tuple((getattr(self, k).data_ptr(), getattr(self, k)._version) for k in key_names)
        cache = self.__dict__.get(slot)
        if cache is None or cache[0] != key:
            cache = (key, build().contiguous())
            self.__dict__[slot] = cache
        return cache[1]

    def world_to_view_matrix(self):
        """(N,4,4) row-vector world->view matrix, rebuilt only when R/T change."""
        return self._cached("_w2v", ("R", "T"), lambda: self.get_world_to_view_transform().matrix)

    def projection_matrix(self):
        """(N,4,4) row-vector view->clip matrix, rebuilt only when the intrinsics change."""
        return self._cached("_proj", ("znear", "zfar", "aspect_ratio", "fov"),
                            lambda: self.get_projection_transform().matrix)

    def get_camera_center(self, **kwargs):
        """(N,3) camera centres: the translation row of the inverse world->view matrix.  Cached
        while R/T are unchanged and need no gradient (no matrix inverse per render, and none inside
        a captured graph)."""
        if kwargs or self.R.requires_grad or self.T.requires_grad:
            w2v = self.get_world_to_view_transform(**kwargs).matrix
            return torch.linalg.inv(w2v)[:, 3, :3]
        return self._cached("_center", ("R", "T"),
                            lambda: torch.linalg.inv(self.world_to_view_matrix())[:, 3, :3])


def OpenGLPerspectiveCameras(znear=1.0, zfar=100.0, aspect_ratio=1.0, fov=60.0, degrees=True, R=None, T=None,
                             device="cpu"):
    """Deprecated PyTorch3D alias kept because eval.py uses it (eval.py:261-264)."""
    return FoVPerspectiveCameras(znear=znear, zfar=zfar, aspect_ratio=aspect_ratio, fov=fov, degrees=degrees,
                                 R=R, T=T, device=device)
