"""The mesh topology's vertex -> face-corner index (Meshes.corner_csr), which the native projection
backward and vertex normals gather over (deterministic, no atomics): "gather" lists a vertex's
corners t = 3 f + i in increasing t (the verts[faces] backward's order); "normals" in PyTorch3D's
normal accumulation order (corner 1 of every face, then corner 2, then corner 0)."""
import torch

from pertrenderer_amd.renderer import Meshes


def _mesh():
    faces = [torch.tensor([[0, 1, 2], [2, 1, 3], [3, 0, 2], [1, 1, 3]]), torch.tensor([[0, 2, 1]])]
    verts = [torch.zeros(5, 3), torch.zeros(3, 3)]  # vertex 4 of mesh 0 is isolated
    return Meshes(verts, faces)


def test_gather_order():
    m = _mesh()
    f = m.faces_packed().reshape(-1).tolist()
    start, corners = m.corner_csr("gather")
    V = 8
    assert start.shape == (V + 1,) and corners.shape == (len(f),)
    for v in range(V):
        assert corners[start[v]:start[v + 1]].tolist() == [t for t in range(len(f)) if f[t] == v]
    assert start[4] == start[5]  # isolated vertex: no corners


def test_normals_order():
    m = _mesh()
    faces = m.faces_packed()
    start, corners = m.corner_csr("normals")
    for v in range(8):
        exp = [3 * fi + r for r in (1, 2, 0) for fi in range(faces.shape[0]) if int(faces[fi, r]) == v]
        assert corners[start[v]:start[v + 1]].tolist() == exp


def test_cached_per_topology():
    m = _mesh()
    a = m.corner_csr()
    b = m.update_padded(m.verts_padded() + 1.0).corner_csr()
    assert a[0] is b[0] and a[1] is b[1]
