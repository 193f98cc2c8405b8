"""Memory manager (reference: ``water/MemoryManager.java`` (allocation accounting, out-of-memory
back-pressure) and ``water/Cleaner.java`` (swap cold values to disk)).

On MI355X the working set lives in 288 GB of HBM. This module accounts device bytes per DKV frame,
reports HBM usage (``/3/Cloud`` free_mem), and when usage crosses ``high_water`` (fraction of HBM) spills
the least-recently-used frames' columns to pinned host memory; a spilled column transparently comes
back to the device on its next access (``Column.data``). That is the Cleaner's swap, with host RAM
as the backing store instead of ice files.
"""
from __future__ import annotations

import threading
import time

import torch

_lock = threading.RLock()
_last_use: dict = {}
_state = dict(high_water=0.90, spilled_bytes=0, spills=0, restores=0)


def touch(frame_id: str):
    _last_use[frame_id] = time.time()


def frame_bytes(frame) -> int:
    total = 0
    for c in frame._cols.values():
        d = c.raw_data()
        if d is not None and d.is_cuda:
            total += d.numel() * d.element_size()
    return total


def device_usage(device=None) -> dict:
    if not torch.cuda.is_available():
        return dict(total=0, free=0, used=0, allocated=0)
    free, total = torch.cuda.mem_get_info(device)
    return dict(total=total, free=free, used=total - free, allocated=torch.cuda.memory_allocated(device))


def spill(frame) -> int:
    """Move a frame's device columns to pinned host memory; returns bytes moved."""
    moved = 0
    with _lock:
        for c in frame._cols.values():
            d = c.raw_data()
            if d is not None and d.is_cuda:
                h = torch.empty(d.shape, dtype=d.dtype, pin_memory=True)
                h.copy_(d)
                c.set_raw_data(h, spilled_from=d.device)
                moved += d.numel() * d.element_size()
        _state["spilled_bytes"] += moved
        _state["spills"] += 1 if moved else 0
    return moved


def restore_column(col):
    """Called from ``Column.data`` when a spilled column is touched."""
    with _lock:
        d = col.raw_data()
        dev = col.spilled_device()
        if dev is not None and d is not None and not d.is_cuda:
            col.set_raw_data(d.to(dev, non_blocking=True), spilled_from=None)
            _state["restores"] += 1


def clean(target_fraction: float | None = None) -> int:
    """Spill LRU frames until device usage is under ``target_fraction`` of HBM."""
    from ..core import dkv
    from ..frame import H2OFrame
    if not torch.cuda.is_available():
        return 0
    target = target_fraction if target_fraction is not None else _state["high_water"]
    frames = [(k, v) for k, v in dkv.items() if isinstance(v, H2OFrame) and not dkv.locked(k)]
    frames.sort(key=lambda kv: _last_use.get(kv[0], 0.0))
    moved = 0
    for k, fr in frames:
        u = device_usage()
        if u["total"] == 0 or u["used"] / u["total"] <= target:
            break
        moved += spill(fr)
        torch.cuda.empty_cache()
    return moved


def pressure_check() -> int:
    """Allocation back-pressure (MemoryManager.set_goals): called when frames enter the DKV and before
    every model build; spills LRU frames once HBM usage crosses ``high_water``."""
    if not torch.cuda.is_available():
        return 0
    u = device_usage()
    if u["total"] and u["used"] / u["total"] > _state["high_water"]:
        return clean()
    return 0


def with_backpressure(fn, *args, **kwargs):
    """Run ``fn``; on a device out-of-memory error spill cold frames down to half of HBM, release the
    caching allocator's blocks and retry once (the reference blocks allocations until the Cleaner
    freed memory; here the retry happens after the spill).

    Row-sharded builds run collectives inside ``fn``, so one rank cannot retry alone (its peers would wait
    in a collective it never joins). There the spill decision is collective (every rank cleans when any
    rank is over its high water mark), and an OOM on any rank aborts the process group: every rank fails
    with the error instead of hanging."""
    from ..parallel import collectives as coll
    if coll.is_dist():
        over = 0.0
        if torch.cuda.is_available():
            u = device_usage()
            over = 1.0 if u["total"] and u["used"] / u["total"] > _state["high_water"] else 0.0
        if coll.all_reduce_scalar(over, op=torch.distributed.ReduceOp.MAX) > 0:
            clean()
        try:
            return fn(*args, **kwargs)
        except torch.cuda.OutOfMemoryError as e:
            _state["oom_aborts"] = _state.get("oom_aborts", 0) + 1
            coll.abort_world(f"device out of memory on rank {coll.rank()}: {e}")
            raise RuntimeError(f"device out of memory on rank {coll.rank()}: the sharded build was aborted on "
                               "every rank (it cannot be retried on one rank alone)") from e
    try:
        return fn(*args, **kwargs)
    except torch.cuda.OutOfMemoryError:
        _state["oom_retries"] = _state.get("oom_retries", 0) + 1
        clean(0.5)
        torch.cuda.empty_cache()
        return fn(*args, **kwargs)


def set_high_water(frac: float):
    _state["high_water"] = float(frac)


def stats() -> dict:
    return dict(_state, **device_usage())
