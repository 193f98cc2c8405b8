"""The REST API served by the whole SPMD cloud (reference: ``water/api/RequestServer.java:371`` — any node's
request runs as a cloud-wide job — and ``water/MRTask.java:80-108``, the ``_nlo/_nhi`` fan-out of every task
over all nodes).

MI355X design. The cloud is the ``torch.distributed`` process group, one process per GPU (``torchrun
--nproc-per-node N -m llama_github_io_amd.api.server``). Frames are parsed into row shards and every
trainer reduces its statistics over RCCL, so a request must run on EVERY rank, in the same order, for the
collectives inside it to pair up. Hence:

* rank 0 runs the HTTP server (uvicorn). A request on a *cloud route* (anything that can touch frames,
  models or jobs) is not executed by the server thread: it is handed to rank 0's **cloud executor**, which
  broadcasts its description (method, path, query, headers, body) over a dedicated gloo control group and
  then runs it through the same FastAPI app in-process (ASGI, no socket). Ranks 1..N-1 run the same
  executor loop in their main thread: receive, run the same handler. Rank 0's response goes back to the
  client; the others are discarded.
* the executor is the ONLY thread that runs collectives: cloud requests execute one at a time in broadcast
  order, and a job a request starts (``Job.run_async``: model builds, grids, AutoML, parse) is queued on the
  executor and runs right after that request's response — on every rank at the same point of the sequence.
* *local routes* (``/3/Cloud``, ``/3/Jobs`` polling and cancel, metadata, logs, Flow's static files) are
  answered by rank 0 alone and never wait behind a running job. A cancel is honoured at the job's next
  progress check on every rank at once (:func:`agree_flag`, rank 0's flag broadcast over the control group).
* everything a request names must come out the same on every rank: keys minted inside a cloud task are
  derived from the request's broadcast stamp and a per-cloud sequence (:func:`task_key`), unseeded RNGs
  draw rank 0's entropy (``parallel.collectives.shared_entropy``), and files a request writes for the client
  (uploads, MOJOs, saved models) are written once, by rank 0, at a path every rank derives alike.

Without ``WORLD_SIZE > 1`` nothing here is active and the server behaves as the single-process one.
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import contextvars
import datetime
import itertools
import os
import queue
import re
import secrets
import tempfile
import threading
import time

INTERNAL_HEADER = "x-h2o-cloud-internal"

# routes rank 0 answers alone (method, path regex): reads of rank-0 state and static files. Everything else is a
# cloud route. Classifying a route as cloud is always safe (it only serialises); local is safe only if the route
# runs no collective and mints no key.
_LOCAL = [(m, re.compile(p)) for m, p in [
    ("GET", r"^/3/Cloud$"), ("HEAD", r"^/3/Cloud$"), ("GET", r"^/3/Ping$"),
    ("GET", r"^/3/Jobs(/[^/]+)?$"), ("POST", r"^/3/Jobs/[^/]+/cancel$"),
    ("GET", r"^/3/Metadata/.*$"), ("GET", r"^/3/Capabilities(/.*)?$"), ("GET", r"^/3/About$"),
    ("GET", r"^/3/Timeline$"), ("GET", r"^/3/Logs(/.*)?$"), ("GET", r"^/3/Profiler$"),
    ("GET", r"^/3/Clients$"), ("GET", r"^/3/WaterMeterMemory$"), ("GET", r"^/3/MemoryStats$"),
    ("POST", r"^/4/sessions$"), ("DELETE", r"^/4/sessions/[^/]+$"), ("GET", r"^/3/InitID$"), ("POST", r"^/3/InitID$"),
    ("GET", r"^/3/SessionProperties$"), ("POST", r"^/3/SessionProperties$"), ("POST", r"^/3/LogAndEcho$"),
    ("GET", r"^/$"), ("GET", r"^/flow/[^/]+$"), ("GET", r"^/(login|loginError)$"), ("POST", r"^/j_security_check$"),
]]
# request headers carried to every rank (auth travels too: each rank's login gate sees what rank 0's saw)
_KEEP_HEADERS = ("content-type", "accept", "authorization", "cookie", "x-h2o-client", "user-agent")


class _Task:
    """Identity of the cloud request (or job) being executed: keys minted inside it are deterministic."""

    def __init__(self, stamp: int, serial: int):
        self.stamp, self.serial = int(stamp), int(serial)


_task: contextvars.ContextVar = contextvars.ContextVar("h2o_cloud_task", default=None)
_state = dict(executor=None)
_key_seq = itertools.count(1)


def executor():
    return _state["executor"]


def active() -> bool:
    return _state["executor"] is not None


def in_task() -> bool:
    return _task.get() is not None


def rank() -> int:
    ex = _state["executor"]
    return ex.rank if ex is not None else 0


def world() -> int:
    ex = _state["executor"]
    return ex.world if ex is not None else 1


def task_key(prefix: str) -> str | None:
    """A key minted inside a cloud task: the same string on every rank (the broadcast stamp of the request and a
    per-process sequence that only cloud tasks advance, identically on every rank). None outside a task."""
    t = _task.get()
    if t is None:
        return None
    return f"{prefix}_{t.stamp % 100_000_000:08d}_c{next(_key_seq)}"


def is_local(method: str, path: str) -> bool:
    return any(m == method and rx.match(path) for m, rx in _LOCAL)


def is_internal(headers) -> bool:
    ex = _state["executor"]
    return ex is not None and secrets.compare_digest(headers.get(INTERNAL_HEADER) or "", ex.secret)


def defer_job(job, fn, args, kwargs) -> bool:
    """``Job.run_async`` inside a cloud task: queue the job on the executor (it runs right after the current
    request, on every rank). False outside a task (the caller starts its own thread)."""
    ex = _state["executor"]
    if ex is None or _task.get() is None:
        return False
    ex.pending.append((job, fn, args, kwargs))
    return True


def agree_flag(flag: bool) -> bool:
    """Rank 0's value of a host-side flag on every rank (inside the executor thread only; elsewhere the flag)."""
    ex = _state["executor"]
    if ex is None or _task.get() is None:
        return bool(flag)
    return ex.agree(flag)


def shared_path(name: str) -> str:
    """A file path every rank derives alike for the current cloud task (rank 0 writes it, see :func:`rank0_write`)."""
    t = _task.get()
    ex = _state["executor"]
    d = os.path.join(tempfile.gettempdir(), f"h2o_cloud_{ex.cloud_id if ex else os.getpid()}")
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, f"{t.serial if t else 0}_{os.path.basename(name)}")


def rank0_write(fn):
    """Run ``fn()`` (a file write whose result the client fetches) on rank 0 only, then let every rank pass once it
    is on disk. Returns ``fn()``'s value on rank 0 and None elsewhere. Outside a cloud task: ``fn()``."""
    ex = _state["executor"]
    if ex is None or _task.get() is None:
        return fn()
    out, err = None, None
    if ex.rank == 0:
        try:
            out = fn()
        except BaseException as e:  # noqa: BLE001 - re-raised below once every rank knows
            err = e
    failed = ex.agree(err is not None)
    if failed:
        raise err if err is not None else RuntimeError("rank 0 failed to write the file")
    return out


class CloudExecutor:
    """See the module docstring. ``app``: the FastAPI application every rank builds identically."""

    def __init__(self, app, group_timeout_days: float = 365.0):
        import torch.distributed as dist
        self.app = app
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        # a CPU control group with an effectively unbounded timeout: a worker waits here while the server idles
        self.group = dist.new_group(backend="gloo", timeout=datetime.timedelta(days=group_timeout_days))
        box = [(secrets.token_hex(16), f"{int(time.time())}_{os.getpid()}")] if self.rank == 0 else [None]
        dist.broadcast_object_list(box, 0, group=self.group)
        self.secret, self.cloud_id = box[0]
        from ..core import runtime
        nodes = [None] * self.world
        dist.all_gather_object(nodes, runtime.node_info(), group=self.group)
        self.nodes = nodes
        self.q: queue.Queue = queue.Queue()
        self.pending: list = []
        self.serial = 0
        self.thread = None
        self.stopped = threading.Event()
        self._device = None

    # ---- collectives of the control group (executor thread only)
    def _bcast(self, obj):
        import torch.distributed as dist
        box = [obj]
        dist.broadcast_object_list(box, 0, group=self.group)
        return box[0]

    def agree(self, flag: bool) -> bool:
        return bool(self._bcast(bool(flag) if self.rank == 0 else None))

    def barrier(self):
        import torch.distributed as dist
        dist.barrier(group=self.group)

    # ---- rank 0: requests from the HTTP server
    def submit(self, desc: dict) -> concurrent.futures.Future:
        fut: concurrent.futures.Future = concurrent.futures.Future()
        self.q.put((desc, fut))
        return fut

    def start(self):
        """Rank 0: the executor runs on a background thread (the main thread serves HTTP)."""
        _state["executor"] = self
        self.thread = threading.Thread(target=self.loop, name="h2o-cloud-executor", daemon=True)
        self.thread.start()

    def stop(self):
        if self.rank == 0 and self.thread is not None and not self.stopped.is_set():
            self.q.put((None, None))
            self.thread.join(timeout=60)

    def loop(self):
        """The executor loop (rank 0: background thread; ranks > 0: their main thread). Returns on shutdown."""
        _state["executor"] = self
        from ..core import runtime
        dev = runtime.device()
        if dev.type == "cuda":
            import torch
            torch.cuda.set_device(dev)
        try:
            while True:
                if self.rank == 0:
                    desc, fut = self.q.get()
                    if desc is not None:
                        desc = dict(desc, stamp=int(time.time() * 1000))
                else:
                    desc, fut = None, None
                desc = self._bcast(desc)
                if desc is None:
                    break
                self.serial += 1
                result = self._run(desc, _Task(desc["stamp"], self.serial))
                if fut is not None:
                    fut.set_result(result)
                # jobs the request started, in the order it started them, before the next request
                while self.pending:
                    job, fn, args, kwargs = self.pending.pop(0)
                    self.serial += 1
                    tok = _task.set(_Task(desc["stamp"], self.serial))
                    try:
                        job._execute(fn, args, kwargs)
                    finally:
                        _task.reset(tok)
                if desc.get("path") == "/3/Shutdown":
                    break
        finally:
            self.stopped.set()
            while not self.q.empty():            # requests that raced the shutdown: answer, never hang a client
                d, f = self.q.get_nowait()
                if f is not None:
                    f.set_result((503, [("content-type", "application/json")], b'{"msg": "cloud is shutting down"}'))

    def _run(self, desc: dict, task: _Task):
        tok = _task.set(task)
        try:
            return asyncio.run(self._call(desc))
        except BaseException as e:  # noqa: BLE001 - an unhandled app error becomes a 500 on rank 0
            import json
            return (500, [("content-type", "application/json")],
                    json.dumps({"http_status": 500, "msg": f"{type(e).__name__}: {e}"}).encode())
        finally:
            _task.reset(tok)

    async def _call(self, desc: dict):
        import httpx
        headers = [(k, v) for k, v in desc.get("headers", []) if k.lower() in _KEEP_HEADERS]
        headers.append((INTERNAL_HEADER, self.secret))
        transport = httpx.ASGITransport(app=self.app, raise_app_exceptions=False, client=("127.0.0.1", 0))
        async with httpx.AsyncClient(transport=transport, base_url="http://h2o-cloud") as c:
            url = desc["path"] + (("?" + desc["query"]) if desc.get("query") else "")
            r = await c.request(desc["method"], url, headers=headers, content=desc.get("body") or b"",
                                timeout=None)
            return r.status_code, [(k, v) for k, v in r.headers.items()
                                   if k.lower() not in ("content-length", "transfer-encoding", "content-encoding")], r.content


def install(app):
    """Rank 0's request router (call before the login gate is installed, so it sits inside it)."""
    from starlette.responses import Response

    @app.middleware("http")
    async def cloud_dispatch(request, call_next):
        ex = _state["executor"]
        if ex is None or is_internal(request.headers) or is_local(request.method, request.url.path):
            return await call_next(request)
        if ex.stopped.is_set():
            return Response(b'{"msg": "cloud is shutting down"}', status_code=503, media_type="application/json")
        body = await request.body()
        desc = dict(method=request.method, path=request.url.path, query=request.url.query,
                    headers=[(k, v) for k, v in request.headers.items()], body=body)
        status, headers, content = await asyncio.wrap_future(ex.submit(desc))
        r = Response(content=content, status_code=status)
        for k, v in headers:
            if k.lower() in ("set-cookie",):
                r.headers.append(k, v)
            else:
                r.headers[k] = v
        return r
