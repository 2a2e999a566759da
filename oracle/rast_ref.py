"""ctypes wrapper of the C rasterizer oracle (oracle/rast_oracle.c)  —  TEST INFRASTRUCTURE ONLY.

Builds oracle/build/librast_oracle_{f32,f64}.so on first use (gcc, see oracle/Makefile).
PARITY UNPINNED by the reference (PyTorch3D 0.4.0 is absent); see rast_oracle.c.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_libs = {}


def build():
    subprocess.check_call(["make", "-s", "-C", HERE], stdout=subprocess.DEVNULL)


def _lib(dtype):
    key = np.dtype(dtype).name
    if key not in _libs:
        path = os.path.join(HERE, "build", f"librast_oracle_{'f32' if key == 'float32' else 'f64'}.so")
        if not os.path.exists(path):
            build()
        _libs[key] = C.CDLL(path)
    return _libs[key]


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def rast_fwd(face_verts, first, nfaces, H, W, K, blur, perspective_correct=False, clip=False, cull=False,
             dtype=np.float32):
    """-> (p2f int64 (N,H,W,K), zbuf, bary (N,H,W,K,3), dists)"""
    rt = C.c_float if np.dtype(dtype) == np.float32 else C.c_double
    fv = np.ascontiguousarray(face_verts, dtype=dtype)
    first = np.ascontiguousarray(first, dtype=np.int64)
    nfaces = np.ascontiguousarray(nfaces, dtype=np.int64)
    N = first.shape[0]
    p2f = np.empty((N, H, W, K), np.int64)
    zbuf = np.empty((N, H, W, K), dtype)
    bary = np.empty((N, H, W, K, 3), dtype)
    dists = np.empty((N, H, W, K), dtype)
    _lib(dtype).rast_fwd(_p(fv), _p(first), _p(nfaces), C.c_int(N), C.c_int(H), C.c_int(W), C.c_int(K),
                         rt(blur), C.c_int(int(perspective_correct)), C.c_int(int(clip)), C.c_int(int(cull)),
                         _p(p2f), _p(zbuf), _p(bary), _p(dists))
    return p2f, zbuf, bary, dists


def rast_bwd(face_verts, p2f, grad_zbuf, grad_bary, grad_dists, perspective_correct=False, clip=False,
             dtype=np.float32):
    fv = np.ascontiguousarray(face_verts, dtype=dtype)
    p2f = np.ascontiguousarray(p2f, dtype=np.int64)
    N, H, W, K = p2f.shape
    cv = lambda a: None if a is None else np.ascontiguousarray(a, dtype=dtype)
    gz, gb, gd = cv(grad_zbuf), cv(grad_bary), cv(grad_dists)
    out = np.empty_like(fv)
    _lib(dtype).rast_bwd(_p(fv), C.c_int64(fv.shape[0]), _p(p2f), C.c_int(N), C.c_int(H), C.c_int(W),
                         C.c_int(K), C.c_int(int(perspective_correct)), C.c_int(int(clip)), _p(gz), _p(gb),
                         _p(gd), _p(out))
    return out


def interp(p2f, bary, face_attr):
    """PyTorch3D interpolate_face_attributes: sum_i bary_i attr[f, i] (0 where p2f < 0)."""
    p2f = np.asarray(p2f)
    mask = p2f >= 0
    fa = np.asarray(face_attr)[np.where(mask, p2f, 0)]          # (...,3,D)
    b = np.asarray(bary, dtype=fa.dtype)
    out = (b[..., 0:1] * fa[..., 0, :] + b[..., 1:2] * fa[..., 1, :]) + b[..., 2:3] * fa[..., 2, :]
    return np.where(mask[..., None], out, 0).astype(fa.dtype)
