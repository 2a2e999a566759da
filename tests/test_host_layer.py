"""The C++ autograd layer (pertrenderer_amd/host_layer.py, csrc/pr_torch.cpp) without a GPU: the
module builds, loads, binds every entry point of the library and refuses host tensors before any
launch (a host pointer handed to a kernel would fault the device)."""
import pytest
import torch

from pertrenderer_amd import _native as nat
from pertrenderer_amd import host_layer


def _ext():
    if host_layer.layer() != "c++":
        pytest.fail(f"C++ layer not loaded: {host_layer.error()}")
    with host_layer.disabled():
        assert host_layer.get() is None
    return host_layer.get()


def test_layer_loads_and_binds():
    ext = _ext()
    assert ext.ABI_VERSION == nat.ABI_VERSION
    assert ext.PARAMS_BYTES == nat.C.sizeof(nat.PRBlendParams)


def test_timer_routes_to_python_functions():
    from pertrenderer_amd.timing import KernelTimer
    _ext()
    with KernelTimer():
        assert host_layer.get() is None


def test_host_tensors_are_refused():
    ext = _ext()
    with pytest.raises(ValueError, match="ROCm devices only"):
        ext.so3_exp(torch.zeros(2, 3), 1e-4)
    with pytest.raises(ValueError, match="ROCm devices only"):
        ext.rotate(torch.zeros(1, 4, 3), torch.eye(3)[None])
    with pytest.raises(ValueError, match="ROCm devices only"):
        ext.project_rasterize(torch.zeros(3, 3), torch.zeros(1, 3, dtype=torch.int64),
                              torch.zeros(1, dtype=torch.int64), torch.ones(1, dtype=torch.int64),
                              torch.eye(4)[None], torch.eye(4)[None], None, None, [8, 8, 2, 0, 0, 0, 0, 0], 0.0,
                              None, None, 0)
    p = nat.PRBlendParams()
    z = torch.zeros(1, 2, 2, 3)
    with pytest.raises(ValueError, match="ROCm devices only"):
        ext.blend(z, z, torch.zeros(1, 2, 2, 3, 3), None, None, None, None, None, torch.zeros(1, 2, 2, 3, dtype=torch.int64),
                  None, None, torch.ones(1), torch.ones(1), None, None, None, nat.C.addressof(p), True, False)
