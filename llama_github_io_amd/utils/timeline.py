"""TimeLine / Profiler (reference: ``water/TimeLine.java`` (ring buffer of network/task events),
``water/api/TimelineHandler.java``, ``water/util/JProfile.java`` / ``/3/Profiler`` stack sampling).

Events are recorded on host around the work that matters on this engine — jobs, collectives
(bytes, duration), kernel-library calls wrapped with ``span`` — into a fixed ring buffer;
``device_sync=True`` spans time GPU work accurately. ``stacks()`` samples every Python thread's
stack (the profiler endpoint).
"""
from __future__ import annotations

import collections
import contextlib
import sys
import threading
import time
import traceback

_events = collections.deque(maxlen=1 << 14)
_enabled = [True]


def record(kind: str, name: str, duration_s: float = 0.0, **kw):
    if _enabled[0]:
        _events.append(dict(ts_ms=int(time.time() * 1000), kind=kind, name=name, duration_us=int(duration_s * 1e6),
                            thread=threading.current_thread().name, **kw))


@contextlib.contextmanager
def span(kind: str, name: str, device_sync: bool = False, **kw):
    if device_sync:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if device_sync:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
        record(kind, name, time.perf_counter() - t0, **kw)


def events(n: int = 1000) -> list:
    return list(_events)[-n:]


def clear():
    _events.clear()


def enable(on: bool = True):
    _enabled[0] = bool(on)


def stacks() -> list:
    """``/3/Profiler``: current stack of every thread."""
    names = {t.ident: t.name for t in threading.enumerate()}
    out = []
    for tid, frame in sys._current_frames().items():
        out.append(dict(thread=names.get(tid, str(tid)), stack="".join(traceback.format_stack(frame))))
    return out
