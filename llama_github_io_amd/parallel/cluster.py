"""Cloud membership, heartbeats and failure detection (reference: ``water/Paxos.java`` (cloud
formation / lock), ``water/HeartBeatThread.java`` (periodic heartbeats, ``TIMEOUT``),
``water/init/...`` client disconnect checks, ``H2O.shutdown`` on fatal node loss).

Formation is the ``torch.distributed`` rendezvous (every rank joins before any work: the cloud is
"locked" at init). Each rank runs a daemon heartbeat thread that writes ``hb/<rank> = (time, job
progress)`` into the process group's key-value store (the TCPStore behind the rendezvous) every
``interval`` seconds and reads every peer's entry; a peer silent for longer than ``timeout`` marks
the cloud unhealthy. Running jobs observe it through :func:`check` (called from ``Job.update``), so
a lost GPU/rank fails the job promptly instead of hanging in a collective until the RCCL timeout.
"""
from __future__ import annotations

import json
import os
import threading
import time

_state = dict(thread=None, stop=None, healthy=True, dead=[], last=dict(), interval=1.0, timeout=30.0)


def _store():
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return None
    try:
        from torch.distributed.distributed_c10d import _get_default_store
        return _get_default_store()
    except Exception:  # noqa: BLE001 - store not exposed by this backend
        return None


def _beat(rank, world, store, stop):
    while not stop.is_set():
        now = time.time()
        try:
            store.set(f"h2o_hb/{rank}", json.dumps(dict(t=now, pid=os.getpid())))
            dead = []
            for r in range(world):
                if r == rank:
                    continue
                try:
                    # check() first: a get() of a key the peer has not written yet BLOCKS in the store client for
                    # its whole timeout, and a daemon thread parked in that C++ call at interpreter exit can abort
                    # the process ("terminate called without an active exception")
                    if store.check([f"h2o_hb/{r}"]):
                        v = json.loads(store.get(f"h2o_hb/{r}"))
                        _state["last"][r] = v["t"]
                except Exception:  # noqa: BLE001 - peer has not written yet
                    v = None
                t = _state["last"].get(r)
                if t is not None and now - t > _state["timeout"]:
                    dead.append(r)
            _state["dead"] = dead
            _state["healthy"] = not dead
        except Exception:  # noqa: BLE001 - the store itself is gone: the coordinator died
            _state["healthy"] = False
            _state["dead"] = ["store"]
        stop.wait(_state["interval"])


def start(interval: float = 1.0, timeout: float = 30.0) -> bool:
    """Start the heartbeat thread (no-op outside a multi-process cloud)."""
    import torch.distributed as dist
    if _state["thread"] is not None:
        return True
    store = _store()
    if store is None or dist.get_world_size() < 2:
        return False
    _state.update(interval=float(interval), timeout=float(timeout), healthy=True, dead=[])
    ev = threading.Event()
    th = threading.Thread(target=_beat, args=(dist.get_rank(), dist.get_world_size(), store, ev), daemon=True,
                          name="h2o-heartbeat")
    _state["thread"], _state["stop"] = th, ev
    th.start()
    import atexit
    atexit.register(stop)            # join the thread before the store / process group are torn down
    return True


def stop():
    if _state["stop"] is not None:
        _state["stop"].set()
        _state["thread"].join(timeout=5)
    _state["thread"] = _state["stop"] = None


def healthy() -> bool:
    return bool(_state["healthy"])


def status() -> dict:
    return dict(healthy=_state["healthy"], dead=list(_state["dead"]), last_heartbeat=dict(_state["last"]),
                interval=_state["interval"], timeout=_state["timeout"], running=_state["thread"] is not None)


class CloudUnhealthy(RuntimeError):
    pass


def check():
    """Raise if a peer stopped heartbeating (jobs call this between iterations)."""
    if not _state["healthy"]:
        raise CloudUnhealthy(f"cloud unhealthy: lost ranks {_state['dead']}")
