"""eval.py:4's CUDA_LAUNCH_BLOCKING=1 mapped to HIP_LAUNCH_BLOCKING=1 (pertrenderer_amd/launch_mode.py).
CPU checks of the mapping; the GPU box runs tools/launch_blocking_check.py --eval-order to see
launches block (tests/test_gpu_launch_mode.py)."""
import os
import subprocess
import sys

from pertrenderer_amd.launch_mode import honour_cuda_launch_blocking

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_mapping_rules():
    env = {"CUDA_LAUNCH_BLOCKING": "1"}
    assert honour_cuda_launch_blocking(env) and env["HIP_LAUNCH_BLOCKING"] == "1"
    env = {}
    assert not honour_cuda_launch_blocking(env) and "HIP_LAUNCH_BLOCKING" not in env
    env = {"CUDA_LAUNCH_BLOCKING": "0"}
    assert not honour_cuda_launch_blocking(env) and "HIP_LAUNCH_BLOCKING" not in env
    env = {"CUDA_LAUNCH_BLOCKING": "1", "HIP_LAUNCH_BLOCKING": "0"}  # an explicit HIP setting wins
    assert not honour_cuda_launch_blocking(env) and env["HIP_LAUNCH_BLOCKING"] == "0"


def test_shim_import_maps_in_a_fresh_process():
    """eval.py's order: set the variable, import torch, import the pytorch3d shim (eval.py:4,22,26)."""
    code = ("import os; os.environ['CUDA_LAUNCH_BLOCKING'] = '1'; import torch; import pytorch3d.loss; "
            "print(os.environ.get('HIP_LAUNCH_BLOCKING'))")
    env = {k: v for k, v in os.environ.items() if k not in ("CUDA_LAUNCH_BLOCKING", "HIP_LAUNCH_BLOCKING")}
    env["PYTHONPATH"] = ROOT
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == "1"


def test_no_mapping_without_request():
    code = "import os; import pytorch3d.loss; print(os.environ.get('HIP_LAUNCH_BLOCKING'))"
    env = {k: v for k, v in os.environ.items() if k not in ("CUDA_LAUNCH_BLOCKING", "HIP_LAUNCH_BLOCKING")}
    env["PYTHONPATH"] = ROOT
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == "None"
