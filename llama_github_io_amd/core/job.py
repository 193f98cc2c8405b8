"""Jobs: asynchronous work with progress, cancellation and status (reference:
``h2o-core/src/main/java/water/Job.java``, ``water/api/JobsHandler.java``).

A :class:`Job` wraps a callable. ``run_async`` executes it on a worker thread (the REST layer
polls ``/3/Jobs/{key}``); ``run_sync`` executes inline (the Python facade default). Work loops call
:meth:`Job.update` with their progress and :meth:`Job.check_cancelled`, which raises
:class:`JobCancelled` after :meth:`Job.cancel` — the analogue of ``Job.stop_requested()``.
"""
from __future__ import annotations

import threading
import time
import traceback

from . import dkv

CREATED, RUNNING, DONE, CANCELLED, FAILED = "CREATED", "RUNNING", "DONE", "CANCELLED", "FAILED"

_local = threading.local()


class JobCancelled(Exception):
    pass


class Job:
    def __init__(self, description: str, dest: str | None = None, work: float = 1.0, key: str | None = None):
        self.key = key or dkv.new_key("job")
        self.description = description
        self.dest = dest
        self.work = float(work) if work else 1.0
        self.worked = 0.0
        self.status = CREATED
        self.start_time = None
        self.end_time = None
        self.exception = None
        self.stacktrace = None
        self.result = None
        self.progress_msg = ""
        self._cancel = threading.Event()
        self._thread = None
        self.warnings = []
        dkv.put(self.key, self)

    # ---- progress
    @property
    def progress(self) -> float:
        if self.status == DONE:
            return 1.0
        return min(1.0, self.worked / self.work)

    def update(self, amount: float = 1.0, msg: str | None = None) -> None:
        self.worked += amount
        if msg:
            self.progress_msg = msg
        self.check_cancelled()

    def set_progress(self, frac: float, msg: str | None = None) -> None:
        self.worked = float(frac) * self.work
        if msg:
            self.progress_msg = msg
        self.check_cancelled()

    # ---- cancellation
    def cancel(self) -> None:
        self._cancel.set()

    def stop_requested(self) -> bool:
        return self._cancel.is_set()

    def check_cancelled(self) -> None:
        from ..api import cloud
        # REST cloud: a cancel reaches rank 0 only; every rank stops at the same check (rank 0's flag, broadcast)
        flag = cloud.agree_flag(self._cancel.is_set()) if cloud.active() else self._cancel.is_set()
        if flag:
            raise JobCancelled(self.key)
        from ..parallel import cluster
        cluster.check()

    # ---- execution
    def _execute(self, fn, args, kwargs):
        prev = getattr(_local, "job", None)
        _local.job = self
        self.status = RUNNING
        self.start_time = time.time()
        try:
            dest_lock = dkv.write_lock(self.dest) if self.dest else None
            if dest_lock:
                dest_lock.__enter__()
            try:
                self.result = fn(*args, **kwargs)
            finally:
                if dest_lock:
                    dest_lock.__exit__(None, None, None)
            self.status = DONE
        except JobCancelled:
            self.status = CANCELLED
        except BaseException as e:  # noqa: BLE001 - recorded on the job, re-raised by run_sync
            self.status = FAILED
            self.exception = e
            self.stacktrace = traceback.format_exc()
        finally:
            self.end_time = time.time()
            _local.job = prev
        return self.result

    def run_sync(self, fn, *args, **kwargs):
        self._execute(fn, args, kwargs)
        if self.status == FAILED:
            raise self.exception
        return self.result

    def run_async(self, fn, *args, **kwargs) -> "Job":
        from ..api import cloud
        if cloud.defer_job(self, fn, args, kwargs):     # REST cloud: the executor runs it on every rank, in order
            return self
        self._thread = threading.Thread(target=self._execute, args=(fn, args, kwargs), daemon=True,
                                        name=f"h2o-job-{self.key}")
        self._thread.start()
        return self

    def join(self, timeout: float | None = None):
        if self._thread is not None:
            self._thread.join(timeout)
        if self.status == FAILED:
            raise self.exception
        return self.result

    def is_running(self) -> bool:
        return self.status in (CREATED, RUNNING)

    @property
    def run_time_ms(self) -> int:
        if self.start_time is None:
            return 0
        return int(((self.end_time or time.time()) - self.start_time) * 1000)

    def to_dict(self) -> dict:
        return dict(key=dict(name=self.key, type="Key<Job>"), description=self.description, status=self.status,
                    progress=self.progress, progress_msg=self.progress_msg, start_time=int((self.start_time or 0) * 1000),
                    msec=self.run_time_ms, dest=dict(name=self.dest) if self.dest else None,
                    exception=None if self.exception is None else repr(self.exception), stacktrace=self.stacktrace,
                    warnings=self.warnings)


def current() -> Job | None:
    """The job running on this thread (or None outside any job)."""
    return getattr(_local, "job", None)


def progress(amount: float = 1.0, msg: str | None = None) -> None:
    """Report progress to the current job if any (cheap no-op otherwise)."""
    j = current()
    if j is not None:
        j.update(amount, msg)


def list_jobs() -> list:
    return [v for _, v in dkv.items() if isinstance(v, Job)]
