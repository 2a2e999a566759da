"""Native vertex normals (pr_vert_normals_fwd/bwd behind Meshes.verts_normals_packed) against the
torch composition of PyTorch3D's formula (three corner crosses index-added per vertex, then
F.normalize with eps 1e-6): forward and the gradient of a random linear functional, on the
reference's sphere and cube meshes and on a mesh with an isolated vertex (zero normal)."""
import os

import pytest
import torch

from conftest import ROOT, assert_close
from pertrenderer_amd.renderer import Meshes, load_obj
from pertrenderer_amd.renderer import mesh as mesh_mod

pytestmark = pytest.mark.gpu


def _both(verts, faces):
    out, keep = [], mesh_mod.NATIVE_NORMALS
    for native in (True, False):
        mesh_mod.NATIVE_NORMALS = native
        try:
            v = verts.clone().requires_grad_(True)
            n = Meshes([v], [faces]).verts_normals_packed()
            g = torch.randn(n.shape, generator=torch.Generator().manual_seed(5)).to(n.device)
            (gv,) = torch.autograd.grad((n * g).sum(), v)
            out.append((n.detach(), gv))
        finally:
            mesh_mod.NATIVE_NORMALS = keep
    return out


@pytest.mark.parametrize("name", ["sphere_642.obj", "cube2.obj"])
def test_native_normals_match_torch(name, device):
    verts, faces, _ = load_obj(os.path.join(ROOT, "tests", "golden", name))
    v = (verts * torch.tensor([1.0, 0.7, 1.3])).to(device)  # non-uniform scale: uneven face areas
    (n1, g1), (n0, g0) = _both(v, faces.verts_idx.to(device))
    assert_close(n1, n0, name="normals")
    assert_close(g1, g0, name="d verts")


def test_isolated_vertex_has_zero_normal_and_gradient(device):
    v = torch.tensor([[0.0, 0, 0], [1, 0, 0], [0, 1, 0], [5, 5, 5]], device=device)
    f = torch.tensor([[0, 1, 2]], device=device)
    (n1, g1), (n0, g0) = _both(v, f)
    torch.testing.assert_close(n1, n0, rtol=1e-6, atol=1e-7)
    assert torch.equal(n1[3], torch.zeros(3, device=device))
    torch.testing.assert_close(g1, g0, rtol=1e-5, atol=1e-6)
