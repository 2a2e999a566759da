"""bench.py's own rank launcher on the CPU (no GPU work): `python bench.py --gpus N` without torchrun
starts N rank processes with the torchrun environment (MASTER_ADDR 127.0.0.1), and the ranks find
each other (a gloo all-reduce counts them); under a launcher a --gpus that differs from WORLD_SIZE
exits non-zero (the driver's SCALE runs `bench.py --gpus N`)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


@pytest.mark.parametrize("n", [2, 4])
def test_gpus_n_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--launch-check"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["world_size"] == n and d["ranks_seen"] == n
    assert d["master"].startswith("127.0.0.1:")


def test_gpus_must_match_the_launchers_world_size():
    env = dict(_env(), WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--launch-check"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr


def test_a_failing_rank_fails_the_launch():
    # an unknown option makes every rank exit 2 from argparse: the parent reports it
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--no-such-option"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
