"""Kubernetes clustering (h2o-k8s): headless-service DNS lookup with the reference's constraints, node ranks and the
leader from the sorted pod list, the /kubernetes/isLeaderNode readiness probe, and the launcher running a 2-process
gloo job through torch.distributed.run."""
import os
import socket
import subprocess
import sys
import urllib.error
import urllib.request

import pytest

from llama_github_io_amd.parallel import k8s

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Clock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t

    def sleep(self, s):
        self.t += s


def test_lookup_until_expected_count():
    seen = [{"10.0.0.9"}, {"10.0.0.9", "10.0.0.10"}, set(), {"10.0.0.2"}]
    calls = []

    def res(name):
        calls.append(name)
        return seen[min(len(calls) - 1, len(seen) - 1)]
    c = _Clock()
    nodes = k8s.lookup_nodes("svc.ns.svc.cluster.local", expected=3, resolver=res, sleep=c.sleep, clock=c)
    assert nodes == ["10.0.0.2", "10.0.0.9", "10.0.0.10"]         # numeric order, union over lookups
    assert len(calls) == 4 and c.t == 3.0


def test_lookup_timeouts():
    c = _Clock()
    nodes = k8s.lookup_nodes("svc", timeout_s=5, resolver=lambda n: {"10.1.0.1"}, sleep=c.sleep, clock=c)
    assert nodes == ["10.1.0.1"] and c.t == 5.0
    c = _Clock()                                                   # neither constraint: the 180 s default
    k8s.lookup_nodes("svc", resolver=lambda n: set(), sleep=c.sleep, clock=c)
    assert c.t == k8s.DEFAULT_TIMEOUT_S
    c = _Clock()                                                   # whichever constraint ends first
    k8s.lookup_nodes("svc", timeout_s=4, expected=9, resolver=lambda n: {"10.1.0.1"}, sleep=c.sleep, clock=c)
    assert c.t == 4.0
    with pytest.raises(ValueError, match="H2O_KUBERNETES_SERVICE_DNS"):
        k8s.lookup_nodes("  ")


def test_cluster_plan_and_probe():
    plan = k8s.cluster_plan(["10.0.0.10", "10.0.0.9", "10.0.1.1"], "10.0.0.10")
    assert plan["node_rank"] == 1 and plan["leader"] == "10.0.0.9" and not plan["is_leader"] and plan["nnodes"] == 3
    with pytest.raises(RuntimeError):
        k8s.cluster_plan(["10.0.0.9"], "10.0.0.8")
    st = k8s.ProbeState()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    srv = k8s.probe_server(st, port, "127.0.0.1")
    url = f"http://127.0.0.1:{port}/kubernetes/isLeaderNode"

    def code():
        try:
            return urllib.request.urlopen(url, timeout=10).status
        except urllib.error.HTTPError as e:
            return e.code
    try:
        assert code() == 200                                       # clustering: every node ready
        st.clustered, st.is_leader = True, False
        assert code() == 404                                       # clustered, not the leader
        st.is_leader = True
        assert code() == 200
    finally:
        srv.shutdown()


def test_launcher_runs_torchrun_job(tmp_path):
    prog = tmp_path / "job.py"
    prog.write_text("import os, torch.distributed as dist\n"
                    "dist.init_process_group('gloo')\n"
                    "print('RANKLINE', dist.get_rank(), dist.get_world_size(), os.environ['H2O_K8S_LEADER'], flush=True)\n"
                    "dist.destroy_process_group()\n")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port, probe = s.getsockname()[1], None
    s.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    probe = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PYTHONPATH=ROOT, H2O_KUBERNETES_SERVICE_DNS="127.0.0.1", H2O_NODE_EXPECTED_COUNT="1",
               POD_IP="127.0.0.1", H2O_KUBERNETES_API_PORT=str(probe), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "llama_github_io_amd.parallel.k8s", "--gpus-per-node", "2",
                        "--master-port", str(port), "--probe-host", "127.0.0.1", "--", str(prog)],
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    import re                                          # (the two ranks share the pipe: lines may interleave)
    assert sorted(re.findall(r"RANKLINE (\d) (\d) (\d)", r.stdout)) == [("0", "2", "1"), ("1", "2", "1")], r.stdout
    assert "[k8s] 1 node(s) ['127.0.0.1']; node rank 0, leader 127.0.0.1" in r.stdout
