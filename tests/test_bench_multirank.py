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


def _run(world, launcher="torchrun", extra=()):
    args = ["bench.py", "--device", "cpu", "--rows", "6000", "--steps", "3", "--warmup", "1", "--no-job", "--no-auto",
            "--gpus", str(world)] + list(extra)
    env = dict(os.environ, OMP_NUM_THREADS="2", H2O_AMD_DEVICE="cpu")
    env.pop("WORLD_SIZE", None)
    if world == 1 or launcher == "self":
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


def test_bench_self_launches_ranks_without_torchrun():
    """``bench.py --gpus 2`` with no launcher starts its own two ranks and reports them (never a silent 1-rank run)."""
    one = _run(1)
    two = _run(2, launcher="self")
    assert two["n_gpus"] == 2 and two["comm_world"] == 2 and two["comm_backend"] == "gloo"
    assert two["config"]["rows_per_rank"] == 3000 and two["config"]["collectives_per_tree"] > 0
    assert abs(two["config"]["train_auc_after_all_trees"] - one["config"]["train_auc_after_all_trees"]) < 5e-5


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, OMP_NUM_THREADS="2", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, "bench.py", "--device", "cpu", "--gpus", "2", "--rows", "2000", "--steps", "1",
                          "--warmup", "0", "--no-job", "--no-auto"], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr
    assert not [l_ for l_ in out.stdout.splitlines() if l_.startswith("{")]


def test_bench_reports_auto_histogram_time():
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, "bench.py", "--device", "cpu", "--rows", "4000", "--steps", "2", "--warmup", "1",
                          "--no-job", "--auto-steps", "2"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([l_ for l_ in out.stdout.splitlines() if l_.startswith("{")][0])
    assert line["config"]["auto_ms_per_tree"] is not None and line["config"]["auto_ms_per_tree"] > 0
    assert line["rccl_world"] == 0
