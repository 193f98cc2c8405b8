"""Process runtime: device binding, distributed bring-up, cluster status (reference:
``water/H2O.java`` boot, ``water/Paxos.java`` cloud formation, ``water/api/CloudHandler.java``).

MI355X design: one process per GPU. ``torch.distributed`` rendezvous (RCCL = backend ``nccl`` on
ROCm, ``gloo`` on CPU) replaces Paxos; the "cloud" is the process group. Each rank owns the row
shard of every frame it ingests; algorithms all-reduce their sufficient statistics over xGMI
(``parallel/collectives.py``). ``H2O_AMD_DEVICE=cpu`` forces the CPU reference path.
"""
from __future__ import annotations

import os
import socket
import time

import torch

_state = dict(device=None, started=None, name=None, dist_inited_here=False)


def device() -> torch.device:
    d = _state["device"]
    if d is None:
        forced = os.environ.get("H2O_AMD_DEVICE")
        if forced:
            d = torch.device(forced)
        elif torch.cuda.is_available():
            d = torch.device("cuda", int(os.environ.get("LOCAL_RANK", torch.cuda.current_device())))
        else:
            d = torch.device("cpu")
        _state["device"] = d
    return d


def set_device(d) -> torch.device:
    d = torch.device(d)
    if d.type == "cuda":
        torch.cuda.set_device(d)
    _state["device"] = d
    return d


def init(name: str | None = None, distributed: bool | None = None, backend: str | None = None) -> dict:
    """Boot the engine. With ``WORLD_SIZE>1`` in the environment (torchrun) joins the process group:
    RCCL on MI355X, gloo on CPU."""
    import torch.distributed as dist
    if _state["started"] is None:
        _state["started"] = time.time()
        _state["name"] = name or os.environ.get("H2O_CLOUD_NAME", f"h2o_amd_{os.getpid()}")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if distributed is None:
        # (H2O_FORCE_SHARDED=1: a 1-rank group still forms, so the sharded paths run through its collectives)
        distributed = world > 1 or (os.environ.get("H2O_FORCE_SHARDED") == "1" and "MASTER_ADDR" in os.environ)
    if distributed and not dist.is_initialized():
        if torch.cuda.is_available() and os.environ.get("H2O_AMD_DEVICE", "cuda") != "cpu":
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            _state["device"] = torch.device("cuda", local)
            dist.init_process_group(backend or "nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend or "gloo")
        _state["dist_inited_here"] = True
    if distributed:
        from ..parallel import cluster
        cluster.start(float(os.environ.get("H2O_HEARTBEAT_S", "1.0")), float(os.environ.get("H2O_HB_TIMEOUT_S", "30")))
    device()
    from ..utils import log
    log.configure(os.environ.get("H2O_LOG_LEVEL", "INFO"), os.environ.get("H2O_LOG_DIR"))
    return cluster_status()


def shutdown() -> None:
    import torch.distributed as dist
    from ..parallel import cluster
    cluster.stop()
    if _state["dist_inited_here"] and dist.is_initialized():
        dist.destroy_process_group()
        _state["dist_inited_here"] = False
    _state["started"] = None


def is_running() -> bool:
    return _state["started"] is not None


def node_info() -> dict:
    """This rank's entry of the cloud's node list (CloudV3 ``nodes``)."""
    import torch.distributed as dist
    d = device()
    rk = dist.get_rank() if dist.is_initialized() else 0
    if d.type == "cuda":
        props = torch.cuda.get_device_properties(d)
        free, total = torch.cuda.mem_get_info(d)
        return dict(h2o=f"{socket.gethostname()}/rank{rk}", gpu=props.name, gcn_arch=getattr(props, "gcnArchName", ""),
                    num_cus=props.multi_processor_count, mem_total=total, free_mem=free, healthy=True, rank=rk,
                    device=str(d), pid=os.getpid())
    return dict(h2o=f"{socket.gethostname()}/rank{rk}", gpu=None, num_cpus=os.cpu_count(), healthy=True, rank=rk,
                device=str(d), pid=os.getpid())


def cluster_status() -> dict:
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_initialized() else 1
    d = device()
    from ..api import cloud
    ex = cloud.executor()
    if ex is not None:          # the REST cloud: every rank's entry (gathered at cloud start), rank 0's live
        nodes = [dict(n) for n in ex.nodes]
        nodes[0] = node_info()
        from ..parallel import cluster as _cl
        dead = set(_cl.status()["dead"])
        for n in nodes:
            n["healthy"] = n.get("rank") not in dead
    else:
        nodes = [node_info()]
    from ..parallel import cluster
    from ..utils import memory
    hb = cluster.status()
    return dict(version=_version(), cloud_name=_state["name"], cloud_size=world, heartbeat=hb, memory=memory.stats(), cloud_uptime_millis=
                int((time.time() - (_state["started"] or time.time())) * 1000), cloud_healthy=hb["healthy"],
                consensus=True, locked=True, nodes=nodes, device=str(d),
                backend=(dist.get_backend() if dist.is_initialized() else None))


def _version() -> str:
    try:
        import h2o
        return h2o.__version__
    except Exception:  # pragma: no cover
        return "3.46.0.amd0"
