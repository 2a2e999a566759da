"""bench.py's N > 1 path on the one-GPU box: two torchrun ranks sharing the GPU over gloo
(PR_BENCH_BACKEND=gloo, bench.py:418-428), both shardings of DESIGN §6.  The driver measures the
same code with RCCL on an 8-GPU node; this checks that the multi-rank step (captured graphs around
the gradient all-reduce, barriers, max-over-ranks timing, rank-0 JSON line) runs end to end."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("shard,extra", [("frames", ["--image-size", "128"]), ("samples", ["--image-size", "128"]),
                                         (None, ["--config", "cfg4", "--batch", "2", "--image-size", "256"])],
                         ids=["frames", "samples", "default-cfg4-reduced"])
def test_bench_two_ranks_gloo(shard, extra):
    """None: bench.py's N > 1 default (--shard samples) on a reduced cfg 4 shape (2 x 256^2 per rank,
    K = 150, 64 samples split 32 / 32)."""
    env = dict(os.environ, PR_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "3", "--warmup", "2", "--no-cpu-baseline", "--no-dense"] + extra
    if shard is not None:
        cmd += ["--shard", shard]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0 and d["ms_per_step"] > 0
    assert d["scaling"] == ("weak" if shard == "frames" else "strong")
    if shard != "frames":
        ss = d["strong_scaling"]
        assert ss["replicated_ms_per_rank"] > 0 and ss["sharded_ms_per_rank"] > 0 and ss["speedup_bound_vs_1gpu"] > 1
        assert "sample-parallel x2" in d["config"]["parallelism"]
    assert d["config"]["execution"] == "graph"  # the captured multi-rank step, not the eager fallback


@pytest.mark.gpu
def test_bench_gpus_2_spawns_two_ranks_without_a_launcher():
    """`python bench.py --gpus 2` (no torchrun, the way the driver runs --gpus 1) starts two rank
    processes itself (bench._launch_ranks); here both share the box's GPU over gloo.  The line reports
    the ranks the process group saw."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PR_BENCH_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "2", "--no-cpu-baseline",
           "--no-dense", "--image-size", "128"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks"] == 2 and d["backend"] == "gloo"
    assert "sample-parallel x2" in d["config"]["parallelism"]
