"""Client liveness (reference: ``water/ClientDisconnectCheckThread.java``, ``H2O.getClients`` /
``H2O.removeClient``, ``-client_disconnect_timeout``).

Every REST request marks its client (remote host, or the ``X-H2O-Client`` header) as heard from; sessions
opened through ``POST /4/sessions`` belong to the client that opened them. A daemon thread wakes every
``timeout`` seconds and drops clients not heard from within ``timeout``: their sessions end and the
callbacks registered with :func:`on_disconnect` run (e.g. releasing what the session held).
"""
from __future__ import annotations

import threading
import time

from ..utils import log

_lock = threading.Lock()
_clients: dict = {}          # client id -> dict(last_heard=float, sessions=set)
_callbacks: list = []
_thread = None
_stop = threading.Event()
_timeout = None


def touch(client: str, session: str | None = None, now: float | None = None) -> None:
    with _lock:
        c = _clients.setdefault(client, dict(last_heard=0.0, sessions=set()))
        c["last_heard"] = time.time() if now is None else now
        if session:
            c["sessions"].add(session)


def end_session(session: str) -> None:
    with _lock:
        for c in _clients.values():
            c["sessions"].discard(session)


def clients() -> dict:
    with _lock:
        return {k: dict(last_heard=v["last_heard"], sessions=sorted(v["sessions"])) for k, v in _clients.items()}


def on_disconnect(fn) -> None:
    """``fn(client_id, sessions)`` runs for every client dropped by the check."""
    _callbacks.append(fn)


def check(timeout: float, now: float | None = None) -> list:
    """One pass of ClientDisconnectCheckThread.run: drop the clients silent for >= ``timeout`` seconds."""
    now = time.time() if now is None else now
    dropped = []
    with _lock:
        for k in list(_clients):
            if now - _clients[k]["last_heard"] >= timeout:
                dropped.append((k, sorted(_clients.pop(k)["sessions"])))
    for k, sessions in dropped:
        log.get().warning(f"client {k} not heard from for {timeout:.1f}s: disconnected ({len(sessions)} session(s) ended)")
        for fn in list(_callbacks):
            try:
                fn(k, sessions)
            except Exception as e:  # noqa: BLE001 - a failing callback must not stop the check thread
                log.get().warning(f"client disconnect callback failed: {e}")
    return [k for k, _ in dropped]


def start(timeout: float) -> None:
    """Start the check thread (idempotent); ``timeout`` in seconds."""
    global _thread, _timeout
    _timeout = float(timeout)
    if _thread is not None and _thread.is_alive():
        return
    _stop.clear()

    def run():
        while not _stop.wait(_timeout):
            check(_timeout)
    _thread = threading.Thread(target=run, name="ClientDisconnectCheckThread", daemon=True)
    _thread.start()


def stop() -> None:
    global _thread
    _stop.set()
    _thread = None


def reset() -> None:
    with _lock:
        _clients.clear()
