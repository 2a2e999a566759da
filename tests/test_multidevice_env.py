"""CPU checks of the in-process multi-device wiring (multidevice.py, _native.call): the
PR_SAMPLE_DEVICES activation at import, so eval.py (one process pinned to cuda:0,
experiments/eval.py:112-116) shards its Monte-Carlo samples over a node's GPUs unchanged, and the
device guard around every native call (a launch on a tensor of another device than the current
one runs with that device current)."""
import contextlib
import os
import subprocess
import sys
import types

import torch

from conftest import ROOT
from pertrenderer_amd import _native as nat
from pertrenderer_amd import multidevice as md


def test_devices_from_env_forms():
    assert md.devices_from_env("") is None
    assert md.devices_from_env("0,1,3") == ["cuda:0", "cuda:1", "cuda:3"]
    assert md.devices_from_env("cuda:0, cuda:2") == ["cuda:0", "cuda:2"]
    n = torch.cuda.device_count()
    assert md.devices_from_env("all") == ([f"cuda:{i}" for i in range(n)] if n > 1 else None)


def test_activation_at_import():
    code = "import pertrenderer_amd as pa; print([str(d) for d in pa.sample_devices()])"
    env = dict(os.environ, PR_SAMPLE_DEVICES="0,1")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == "['cuda:0', 'cuda:1']"
    env.pop("PR_SAMPLE_DEVICES")
    code = "import pertrenderer_amd as pa; print(pa.sample_devices())"
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.stdout.strip().splitlines()[-1] == "None"


def test_native_call_guards_the_device(monkeypatch):
    entered, calls = [], []

    @contextlib.contextmanager
    def fake_device(idx):
        entered.append(idx)
        yield
        entered.append(-1)

    lib = types.SimpleNamespace(pr_fake=lambda *a: calls.append((list(entered), a)) or 0)
    monkeypatch.setattr(nat, "load", lambda: lib)
    monkeypatch.setattr(nat, "_get_device", lambda: 0)
    monkeypatch.setattr(nat, "stream_of", lambda t: "stream")
    monkeypatch.setattr(torch.cuda, "device", fake_device)
    on = lambda i: types.SimpleNamespace(device=torch.device("cuda", i))
    nat.call("pr_fake", "fake", on(1), "args")
    assert calls[-1] == ([1], ("args", "stream")) and entered == [1, -1]  # guarded, then restored
    entered.clear()
    nat.call("pr_fake", "fake", on(0), "args")
    assert calls[-1] == ([], ("args", "stream")) and entered == []  # current device: no guard


def test_activation_skipped_in_multi_process_jobs():
    """A torchrun rank owns its LOCAL_RANK device: PR_SAMPLE_DEVICES is ignored there (with a warning)."""
    code = "import pertrenderer_amd as pa; print(pa.sample_devices())"
    env = dict(os.environ, PR_SAMPLE_DEVICES="0,1", WORLD_SIZE="2")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == "None" and "ignored" in out.stderr
