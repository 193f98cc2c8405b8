"""Logging (reference: ``h2o-logging``, ``water/util/Log.java``): H2O-style line format
``MM-DD HH:MM:SS.mmm <ip>:<port> <pid> <thread> <LEVEL> <logger>: message``, per-process log file under
``log_dir`` (one per rank), and an in-memory ring buffer served by ``/3/Logs``."""
from __future__ import annotations

import collections
import logging
import os
import socket
import threading

_ring = collections.deque(maxlen=10000)
_configured = [False]
_lock = threading.Lock()


class _RingHandler(logging.Handler):
    def emit(self, record):
        _ring.append(self.format(record))


class _H2OFormatter(logging.Formatter):
    def __init__(self):
        super().__init__()
        self.host = socket.gethostname()
        self.rank = os.environ.get("RANK", "0")

    def format(self, record):
        import time
        t = time.localtime(record.created)
        ms = int(record.msecs)
        return (f"{time.strftime('%m-%d %H:%M:%S', t)}.{ms:03d} {self.host}:r{self.rank} {os.getpid():5d} "
                f"{record.threadName[:12]:12s} {record.levelname:5s} {record.name}: {record.getMessage()}")


def configure(level: str = "INFO", log_dir: str | None = None) -> logging.Logger:
    with _lock:
        root = logging.getLogger("h2o")
        root.setLevel(getattr(logging, str(level).upper(), logging.INFO))
        if not _configured[0]:
            fmt = _H2OFormatter()
            rh = _RingHandler()
            rh.setFormatter(fmt)
            root.addHandler(rh)
            _configured[0] = True
        if log_dir:
            os.makedirs(log_dir, exist_ok=True)
            path = os.path.join(log_dir, f"h2o_amd_r{os.environ.get('RANK', '0')}.log")
            if not any(isinstance(h, logging.FileHandler) and h.baseFilename == os.path.abspath(path) for h in root.handlers):
                fh = logging.FileHandler(path)
                fh.setFormatter(_H2OFormatter())
                root.addHandler(fh)
        return root


def get(name: str = "h2o") -> logging.Logger:
    if not _configured[0]:
        configure()
    return logging.getLogger(name if name.startswith("h2o") else f"h2o.{name}")


def recent(n: int = 500) -> list:
    return list(_ring)[-n:]
