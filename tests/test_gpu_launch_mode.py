"""eval.py's launch-blocking request is honoured under HIP (eval.py:4, :349-355, :368-370): a fresh
process in eval.py's import order launches host-synchronously (tools/launch_blocking_check.py)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_eval_order_launches_block():
    env = {k: v for k, v in os.environ.items() if k not in ("CUDA_LAUNCH_BLOCKING", "HIP_LAUNCH_BLOCKING")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "launch_blocking_check.py"), "--eval-order"],
                         env=env, capture_output=True, text=True, timeout=240)
    print(out.stdout, out.stderr)
    assert out.returncode == 0 and "-> blocking" in out.stdout
