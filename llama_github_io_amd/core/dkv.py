"""In-process distributed key/value registry (reference: ``h2o-core/src/main/java/water/DKV.java``,
``Key.java``, ``Lockable.java``).

H2O's DKV is a cloud-wide hash map with home nodes and Paxos-backed membership. Here one process
owns one GPU and every rank runs the same program on its own row shard, so the registry is a plain
per-process map; values that must agree across ranks (models, frame metadata) are produced by
collective code paths, never by cross-process DKV gets. ``Lockable`` semantics (a frame cannot be
deleted while a job writes it) are kept with per-key read/write lock counts.
"""
from __future__ import annotations

import itertools
import threading
import time
import weakref

_lock = threading.RLock()
_store: dict = {}
_locks: dict = {}
_counter = itertools.count(1)


def new_key(prefix: str = "key") -> str:
    from ..api import cloud            # inside a REST cloud task every rank must mint the same key
    k = cloud.task_key(prefix) if cloud.active() else None
    return k or f"{prefix}_{int(time.time() * 1000) % 100_000_000:08d}_{next(_counter)}"


def put(key: str, value) -> None:
    with _lock:
        _store[key] = value
    if hasattr(value, "_cols"):                 # a frame entered the store: LRU stamp + HBM back-pressure
        from ..utils import memory
        memory.touch(key)
        memory.pressure_check()


def get(key: str, default=None):
    with _lock:
        v = _store.get(key, default)
    if v is not None and hasattr(v, "_cols"):
        from ..utils import memory
        memory.touch(key)
    return v


def __getitem__(key):  # pragma: no cover - module-level convenience
    return get(key)


def contains(key: str) -> bool:
    with _lock:
        return key in _store


def remove(key: str) -> bool:
    with _lock:
        if _locks.get(key, 0) > 0:
            raise RuntimeError(f"key {key} is write-locked by a running job")
        return _store.pop(key, None) is not None


def keys(prefix: str | None = None, kind=None) -> list:
    with _lock:
        out = []
        for k, v in _store.items():
            if prefix and not k.startswith(prefix):
                continue
            if kind is not None and not isinstance(v, kind):
                continue
            out.append(k)
        return out


def items():
    with _lock:
        return list(_store.items())


def remove_all(retained=()) -> int:
    keep = set(retained or ())
    with _lock:
        victims = [k for k in _store if k not in keep and _locks.get(k, 0) == 0]
        for k in victims:
            del _store[k]
        return len(victims)


class write_lock:
    """``Lockable.write_lock``: held while a job produces/overwrites ``key``."""

    def __init__(self, key: str):
        self.key = key

    def __enter__(self):
        with _lock:
            _locks[self.key] = _locks.get(self.key, 0) + 1
        return self

    def __exit__(self, *exc):
        with _lock:
            _locks[self.key] -= 1
            if _locks[self.key] <= 0:
                del _locks[self.key]
        return False


def locked(key: str) -> bool:
    with _lock:
        return _locks.get(key, 0) > 0
