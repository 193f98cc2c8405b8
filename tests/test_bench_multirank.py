"""bench.py as the driver launches it (torch.distributed.run, one process per rank), rehearsed on the CPU with
gloo: the row-sharded GBM step produces the single-process model (same training AUC) and reports its
collective traffic per tree."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world):
    args = ["bench.py", "--device", "cpu", "--rows", "6000", "--steps", "3", "--warmup", "1", "--no-job"]
    env = dict(os.environ, OMP_NUM_THREADS="2", H2O_AMD_DEVICE="cpu")
    if world == 1:
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l_ for l_ in out.stdout.splitlines() if l_.startswith("{")]
    assert len(lines) == 1, out.stdout        # rank 0 prints ONE line
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [2, 4])
def test_bench_multirank_gloo_matches_single(world):
    one = _run(1)
    many = _run(world)
    assert many["n_gpus"] == world and many["steps"] == 3 and many["config"]["global_batch"] == 6000
    assert many["config"]["collectives_per_tree"] > 0 and many["config"]["comm_bytes_per_tree"] > 0
    # one process: exact AUC; sharded: AUC from the all-reduced 2^18-cell score lattice (mergeable metrics)
    assert abs(many["config"]["train_auc_after_all_trees"] - one["config"]["train_auc_after_all_trees"]) < 5e-5
