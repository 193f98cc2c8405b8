"""Kubernetes clustering (reference: ``h2o-k8s`` — ``water/k8s/lookup/KubernetesDnsLookup.java``,
``LookupConstraintsBuilder.java``, ``ClusterSizeConstraint.java``, ``TimeoutConstraint.java``,
``probe/KubernetesLeaderNodeProbeHandler.java``, ``api/KubernetesRestApi.java``).

The reference discovers its H2O pods through the DNS record of a headless service and clusters the JVMs; here a pod
is one NODE of the SPMD cloud and runs one process per GPU under ``torch.distributed.run``. The same environment
the reference's StatefulSet sets drives it:

* ``H2O_KUBERNETES_SERVICE_DNS`` (mandatory): the headless service, e.g. ``h2o-service.<ns>.svc.cluster.local``;
  every second its records are resolved and the pod addresses collected, until
* ``H2O_NODE_EXPECTED_COUNT`` pods are known, or ``H2O_NODE_LOOKUP_TIMEOUT`` seconds passed (whichever first); with
  neither set, a 180 s timeout (``LookupConstraintsBuilder.K8S_DEFAULT_CLUSTERING_TIMEOUT_SECONDS``).
* The pods sorted by address give the node ranks; the first is the leader (``MASTER_ADDR`` of the rendezvous, and
  the node whose rank 0 serves the REST API).
* ``H2O_KUBERNETES_API_PORT`` (default 8080): ``GET /kubernetes/isLeaderNode`` answers 200 until clustering is done,
  then 200 on the leader and 404 elsewhere — the readiness probe that leaves only the leader behind the service.

``python -m llama_github_io_amd.parallel.k8s --gpus-per-node 8 -- -m llama_github_io_amd.api.server`` resolves the
pods, serves the probe, and runs ``torch.distributed.run --nnodes K --node-rank r --nproc-per-node 8
--master-addr <leader>`` as a child process (its exit code is returned).
"""
from __future__ import annotations

import argparse
import ipaddress
import os
import socket
import subprocess
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

DEFAULT_TIMEOUT_S = 180
SERVICE_ENV, TIMEOUT_ENV, COUNT_ENV, PORT_ENV = ("H2O_KUBERNETES_SERVICE_DNS", "H2O_NODE_LOOKUP_TIMEOUT",
                                                 "H2O_NODE_EXPECTED_COUNT", "H2O_KUBERNETES_API_PORT")


def resolve(name: str) -> set:
    """Addresses behind a (headless-service) DNS name."""
    try:
        infos = socket.getaddrinfo(name, None, type=socket.SOCK_STREAM)
    except socket.gaierror:
        return set()
    return {i[4][0] for i in infos}


def _ip_key(a: str):
    try:
        ip = ipaddress.ip_address(a)
        return (ip.version, int(ip))
    except ValueError:
        return (9, a)


def lookup_nodes(service_dns: str, timeout_s: float | None = None, expected: int | None = None,
                 resolver=resolve, sleep=time.sleep, clock=time.monotonic) -> list:
    """Pods of the service (sorted by address): looked up once a second until ``expected`` are known or
    ``timeout_s`` passed — the reference's lookup constraints, with its 180 s default when neither is set."""
    if not service_dns or not service_dns.strip():
        raise ValueError(f"DNS of H2O service not set. Please set the '{SERVICE_ENV}' variable.")
    if timeout_s is None and expected is None:
        timeout_s = DEFAULT_TIMEOUT_S
    t0 = clock()
    found: set = set()

    def ended():
        return ((expected is not None and len(found) == expected) or
                (timeout_s is not None and clock() - t0 >= timeout_s))
    while not ended():
        found |= resolver(service_dns)
        if ended():
            break
        sleep(1.0)
    return sorted(found, key=_ip_key)


def self_address(nodes) -> str:
    """This pod's address among the discovered ones (``POD_IP`` when the pod spec exports it)."""
    ip = os.environ.get("POD_IP")
    if ip:
        return ip
    cands = set()
    try:
        cands |= {i[4][0] for i in socket.getaddrinfo(socket.gethostname(), None)}
    except socket.gaierror:
        pass
    for n in nodes:
        if n in cands:
            return n
    return socket.gethostbyname(socket.gethostname())


def cluster_plan(nodes, me: str) -> dict:
    """Node rank and leader of this pod: the sorted pod list, the first one leads."""
    nodes = sorted(nodes, key=_ip_key)
    if me not in nodes:
        raise RuntimeError(f"this pod ({me}) is not among the discovered nodes {nodes}")
    return dict(nnodes=len(nodes), node_rank=nodes.index(me), leader=nodes[0], is_leader=nodes[0] == me,
                nodes=nodes)


class ProbeState:
    def __init__(self):
        self.clustered = False
        self.is_leader = False


def probe_server(state: ProbeState, port: int, host: str = "0.0.0.0") -> ThreadingHTTPServer:
    """``/kubernetes/isLeaderNode``: 200 while clustering, then 200 on the leader only (404 elsewhere)."""

    class H(BaseHTTPRequestHandler):
        def do_GET(self):                      # noqa: N802 - http.server API
            if self.path.split("?")[0] != "/kubernetes/isLeaderNode":
                self.send_response(404)
            else:
                self.send_response(200 if (not state.clustered or state.is_leader) else 404)
            self.send_header("Content-Type", "text/plain")
            self.send_header("Content-Length", "0")
            self.end_headers()

        def log_message(self, *a):             # quiet
            pass

    srv = ThreadingHTTPServer((host, port), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def torchrun_cmd(plan: dict, gpus_per_node: int, master_port: int, program: list) -> list:
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", str(plan["nnodes"]),
            "--node-rank", str(plan["node_rank"]), "--nproc-per-node", str(gpus_per_node),
            "--master-addr", plan["leader"], "--master-port", str(master_port)] + list(program)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus-per-node", type=int, default=int(os.environ.get("LOCAL_WORLD_SIZE", "0") or 0) or None)
    ap.add_argument("--master-port", type=int, default=29500)
    ap.add_argument("--probe-host", default="0.0.0.0")
    ap.add_argument("--dry-run", action="store_true", help="print the plan and the launch command, run nothing")
    ap.add_argument("program", nargs=argparse.REMAINDER, help="-- <module / script and its arguments>")
    a = ap.parse_args(argv)
    program = a.program[1:] if a.program[:1] == ["--"] else a.program
    if not program:
        ap.error("no program to run (… -- -m llama_github_io_amd.api.server)")
    gpn = a.gpus_per_node
    if gpn is None:
        import torch                          # device COUNT only: no GPU initialisation in the launcher
        gpn = max(1, torch.cuda.device_count())
    state = ProbeState()
    port = int(os.environ.get(PORT_ENV, "8080"))
    srv = None if a.dry_run else probe_server(state, port, a.probe_host)
    to = os.environ.get(TIMEOUT_ENV)
    cnt = os.environ.get(COUNT_ENV)
    nodes = lookup_nodes(os.environ.get(SERVICE_ENV, ""), float(to) if to else None, int(cnt) if cnt else None)
    plan = cluster_plan(nodes, self_address(nodes))
    state.is_leader, state.clustered = plan["is_leader"], True
    cmd = torchrun_cmd(plan, gpn, a.master_port, program)
    print(f"[k8s] {plan['nnodes']} node(s) {plan['nodes']}; node rank {plan['node_rank']}, leader {plan['leader']}",
          flush=True)
    if a.dry_run:
        print(" ".join(cmd), flush=True)
        return 0
    env = dict(os.environ, H2O_K8S_LEADER="1" if plan["is_leader"] else "0")
    try:
        return subprocess.call(cmd, env=env)
    finally:
        if srv is not None:
            srv.shutdown()


if __name__ == "__main__":
    sys.exit(main())
