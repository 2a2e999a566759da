"""PyTorch3D 0.4.0 mesh losses that experiments/eval.py imports (eval.py:26-31) and uses
in its vertex-deformation task (mesh_laplacian_smoothing, eval.py:455).  Torch code: they
are regularisers on the (small) optimised mesh, not part of the rendering path.
Parity with PyTorch3D is unpinned (not installable here)."""
import torch


def _edges_packed(meshes):
    f = meshes.faces_packed()
    e = torch.cat([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]], 0)
    e, _ = e.sort(dim=1)
    return torch.unique(e, dim=0)


def _vert_weights(meshes, V):
    """1/num_verts of the mesh a packed vertex belongs to (PyTorch3D's per-mesh averaging)."""
    nv = meshes.num_verts_per_mesh().to(torch.float32)
    idx = torch.repeat_interleave(torch.arange(len(nv), device=nv.device), meshes.num_verts_per_mesh())
    return (1.0 / nv)[idx], len(nv)


def mesh_laplacian_smoothing(meshes, method="uniform"):
    """Uniform Laplacian: L v_i = mean of neighbours - v_i; loss = mean over meshes of the
    per-mesh mean |L v_i| (PyTorch3D's "uniform" method)."""
    if method != "uniform":
        raise NotImplementedError("only method='uniform' is implemented (the one eval.py uses)")
    v = meshes.verts_packed()
    V = v.shape[0]
    e = _edges_packed(meshes)
    deg = torch.zeros(V, dtype=v.dtype, device=v.device)
    deg.index_add_(0, e[:, 0], torch.ones(e.shape[0], dtype=v.dtype, device=v.device))
    deg.index_add_(0, e[:, 1], torch.ones(e.shape[0], dtype=v.dtype, device=v.device))
    s = torch.zeros_like(v)
    s.index_add_(0, e[:, 0], v[e[:, 1]])
    s.index_add_(0, e[:, 1], v[e[:, 0]])
    lap = s / deg.clamp(min=1.0)[:, None] - v
    w, n = _vert_weights(meshes, V)
    return (lap.norm(dim=1) * w.to(v.device)).sum() / n


def mesh_edge_loss(meshes, target_length=0.0):
    """mean over meshes of the per-mesh mean (|e| - target)^2 over unique edges."""
    v = meshes.verts_packed()
    e = _edges_packed(meshes)
    return ((v[e[:, 0]] - v[e[:, 1]]).norm(dim=1) - target_length).pow(2).mean()


def mesh_normal_consistency(meshes):
    """mean over interior edges of 1 - cos(angle between the two adjacent face normals)."""
    v, f = meshes.verts_packed(), meshes.faces_packed()
    n = torch.cross(v[f[:, 1]] - v[f[:, 0]], v[f[:, 2]] - v[f[:, 0]], dim=1)
    n = torch.nn.functional.normalize(n, dim=1, eps=1e-6)
    e = torch.cat([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]], 0).sort(dim=1).values
    fid = torch.arange(f.shape[0], device=f.device).repeat(3)
    key = e[:, 0] * (v.shape[0] + 1) + e[:, 1]
    order = key.argsort()
    k, fo = key[order], fid[order]
    same = k[1:] == k[:-1]
    if not bool(same.any()):
        return v.sum() * 0.0
    a, b = fo[:-1][same], fo[1:][same]
    return (1.0 - (n[a] * n[b]).sum(dim=1)).mean()


def chamfer_distance(x, y, batch_reduction="mean", point_reduction="mean"):
    """Symmetric squared Chamfer distance between point clouds (N,P,3) and (N,Q,3);
    returns (loss, None) like PyTorch3D (no normals)."""
    d = torch.cdist(x, y).pow(2)
    cx, cy = d.min(dim=2).values, d.min(dim=1).values
    red = (lambda t: t.mean(1)) if point_reduction == "mean" else (lambda t: t.sum(1))
    loss = red(cx) + red(cy)
    if batch_reduction == "mean":
        loss = loss.mean()
    elif batch_reduction == "sum":
        loss = loss.sum()
    return loss, None
