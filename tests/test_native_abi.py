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


STRUCTS = {
    "PRBlendParams": nat.PRBlendParams, "PRBlendFwdArgs": nat.PRBlendFwdArgs,
    "PRBlendBwdArgs": nat.PRBlendBwdArgs, "PRHeavisideArgs": nat.PRHeavisideArgs,
    "PRRastArgs": nat.PRRastArgs, "PRInterpArgs": nat.PRInterpArgs, "PRProjectArgs": nat.PRProjectArgs,
    "PRSO3Args": nat.PRSO3Args, "PRRotateArgs": nat.PRRotateArgs, "PRShadeArgs": nat.PRShadeArgs,
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
