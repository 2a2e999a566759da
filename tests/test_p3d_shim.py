"""The pytorch3d import shim serves every PyTorch3D name the reference imports
(tests/golden/p3d_imports.json, generated from the reference's sources), and the
textured OBJ loader reads the reference's cube (eval.py:727-757) on CPU."""
import importlib
import json
import os

import torch

from conftest import ROOT


def test_every_reference_pytorch3d_import_resolves():
    names = json.load(open(os.path.join(ROOT, "tests", "golden", "p3d_imports.json")))
    assert names, "fixture empty"
    missing = []
    for mod, syms in names.items():
        m = importlib.import_module(mod)
        missing += [f"{mod}.{s}" for s in syms if not hasattr(m, s)]
    assert not missing, missing


def test_textured_obj_loader_on_cube_fixture():
    from pytorch3d.io import load_obj
    v, f, aux = load_obj(os.path.join(ROOT, "tests", "golden", "cube2.obj"))
    assert v.shape == (8, 3) and f.verts_idx.shape == (12, 3) and f.textures_idx.shape == (12, 3)
    assert aux.verts_uvs.shape[1] == 2 and int(f.textures_idx.max()) < aux.verts_uvs.shape[0]
    assert f.materials_idx.shape == (12,)
