"""bench.py's N > 1 code path on RCCL (torch.distributed "nccl") at one rank, as far as a one-GPU box
allows: torchrun launch, process group, the gradient all-reduce between the captured forward/backward
and Adam graphs, barriers and the max-over-ranks timing (PR_BENCH_DIST=1).  The driver's 8-GPU scaling
run executes the same code with more ranks; exact mode's RCCL collectives: test_gpu_exact_shards.py."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mode", ["graph", "eager"])
def test_bench_distributed_path_on_one_rccl_rank(mode):
    env = dict(os.environ, PR_BENCH_DIST="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "1",
           "--steps", "5", "--warmup", "2", "--mode", mode, "--no-cpu-baseline", "--no-dense"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0 and line["config"]["execution"] == mode
    assert "one nccl rank" in line["config"]["parallelism"], line["config"]["parallelism"]
