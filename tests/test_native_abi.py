"""libpertrender.so loads, exports every symbol include/pertrender.h declares, and the
ctypes structs match the C layout (checked against gcc's offsetof).  No GPU calls."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from conftest import ROOT
from pertrenderer_amd import _native as nat

HEADER = os.path.join(ROOT, "include", "pertrender.h")


def _declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(pr_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    lib = nat.load()
    declared = _declared_functions()
    assert len(declared) >= 14
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(nat.EXPORTS), "ctypes binding out of sync with the header"


def test_abi_version_and_error_string():
    lib = nat.load()
    assert lib.pr_abi_version() == nat.ABI_VERSION
    assert isinstance(lib.pr_last_error(), bytes)


def test_argument_validation_without_gpu():
    """Invalid arguments are rejected on the host before any launch."""
    lib = nat.load()
    a = nat.PRBlendFwdArgs()  # all zero: empty shape
    assert lib.pr_blend_fwd(a, None) == -1
    assert b"empty shape" in lib.pr_last_error()
    r = nat.PRRastArgs()
    assert lib.pr_rast_fwd(r, None) == -1
    assert lib.pr_pose_step(nat.PRPoseStepArgs(), None) == -1
    assert b"pose_step" in lib.pr_last_error()
    m = nat.PRRgbMseArgs()
    assert lib.pr_rgb_mse_fwd(m, None) == -1 and lib.pr_rgb_mse_bwd(m, None) == -1
    assert lib.pr_rgb_mse_workspace(65536) >= 1


STRUCTS = {
    "PRBlendParams": nat.PRBlendParams, "PRBlendFwdArgs": nat.PRBlendFwdArgs,
    "PRBlendBwdArgs": nat.PRBlendBwdArgs, "PRHeavisideArgs": nat.PRHeavisideArgs,
    "PRRastArgs": nat.PRRastArgs, "PRInterpArgs": nat.PRInterpArgs, "PRProjectArgs": nat.PRProjectArgs,
    "PRSO3Args": nat.PRSO3Args, "PRRotateArgs": nat.PRRotateArgs, "PRShadeArgs": nat.PRShadeArgs,
    "PRNormalsArgs": nat.PRNormalsArgs, "PRPoseStepArgs": nat.PRPoseStepArgs, "PRRgbMseArgs": nat.PRRgbMseArgs,
}


def test_ctypes_layout_matches_c_header():
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for sname, cls in STRUCTS.items():
        lines.append(f'printf("{sname} %zu\\n", sizeof({sname}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{sname}.{fname} %zu\\n", offsetof({sname}, {fname}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as td:
        c = os.path.join(td, "l.c")
        open(c, "w").write("\n".join(lines))
        exe = os.path.join(td, "l")
        subprocess.check_call(["gcc", "-o", exe, c])
        out = subprocess.check_output([exe]).decode().split("\n")
    got = dict(l.split() for l in out if l)
    for sname, cls in STRUCTS.items():
        assert int(got[sname]) == C.sizeof(cls), sname
        for fname, _ in cls._fields_:
            assert int(got[f"{sname}.{fname}"]) == getattr(cls, fname).offset, f"{sname}.{fname}"


def test_ops_refuse_cpu_tensors():
    import torch
    from pertrenderer_amd import perturbed_heaviside
    with pytest.raises(nat.NativeError):
        perturbed_heaviside(torch.zeros(1, 2, 2, 3), torch.tensor(1e-3), 4)


def test_rast_workspace_counts_the_bin_lists():
    """pr_rast_fwd_workspace_size (host-only): face records + fp16 boxes, plus with bin_size > 0
    the bin counters and lists: N * ceil(H/b) * ceil(W/b) * (1 + cap) ints, b = bin_size rounded
    up to a multiple of 8, cap = min(max_faces_per_bin or max(10000, F/5), F)."""
    lib = nat.load()
    a = nat.PRRastArgs()
    a.F, a.N, a.H, a.W, a.K = 1000, 2, 256, 200, 8
    base = lib.pr_rast_fwd_workspace_size(a)
    assert base == 1000 * (96 + 8)
    a.bin_size, a.max_faces_per_bin = 16, 0
    assert lib.pr_rast_fwd_workspace_size(a) == base + 2 * 16 * 13 * 4 * (1 + 1000)
    a.bin_size, a.max_faces_per_bin = 12, 300  # 12 -> 16-pixel bins, cap 300
    assert lib.pr_rast_fwd_workspace_size(a) == base + 2 * 16 * 13 * 4 * (1 + 300)
    a.bin_size = 0
    assert lib.pr_rast_fwd_workspace_size(a) == base


def test_bin_params_resolve_like_pytorch3d():
    from pertrenderer_amd.renderer.rasterizer import bin_params
    os.environ.pop("PR_RAST_BINS", None)
    assert bin_params(None, None, 256, 256, 5000) == (0, 0)  # None: the naive cull (measured faster)
    assert bin_params(0, 100, 256, 256, 5000) == (0, 0)
    assert bin_params(32, None, 512, 512, 5000) == (32, 10000)
    assert bin_params(8, 77, 64, 64, 5000) == (8, 77)
    os.environ["PR_RAST_BINS"] = "1"
    try:
        assert bin_params(None, None, 64, 64, 100000) == (8, 20000)
        assert bin_params(None, None, 256, 256, 10) == (16, 10000)
        assert bin_params(None, None, 512, 512, 10) == (32, 10000)
        assert bin_params(None, None, 1024, 1024, 10) == (64, 10000)
    finally:
        os.environ.pop("PR_RAST_BINS")
    os.environ["PR_RAST_BINS"] = "0"
    try:
        assert bin_params(16, 50, 256, 256, 10) == (0, 0)
    finally:
        os.environ.pop("PR_RAST_BINS")
