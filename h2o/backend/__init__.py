"""``h2o.backend`` (reference: h2o-py/h2o/backend): the connection to a running server, a locally started
server process, and the cluster view."""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time

from .._conn import RemoteConnection as H2OConnection


class H2OLocalServer:
    """A REST server started as a child process (``python -m llama_github_io_amd.api.server``)."""

    def __init__(self, proc, ip, port, scheme="http"):
        self._process, self._ip, self._port, self._scheme = proc, ip, port, scheme

    @staticmethod
    def start(ip="127.0.0.1", port=None, verbose=True, extra_args=None, timeout=120, **_):
        if port is None:
            s = socket.socket()
            s.bind((ip, 0))
            port = s.getsockname()[1]
            s.close()
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
        cmd = [sys.executable, "-m", "llama_github_io_amd.api.server", "--ip", ip, "--port", str(port)] + \
            list(extra_args or [])
        proc = subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        t0 = time.time()
        while time.time() - t0 < timeout:
            if proc.poll() is not None:
                raise RuntimeError(f"server exited with {proc.returncode}")
            try:
                with socket.create_connection((ip, port), timeout=0.5):
                    break
            except OSError:
                time.sleep(0.2)
        else:
            proc.kill()
            raise RuntimeError("server did not start")
        if verbose:
            print(f"H2O server started at http://{ip}:{port}")
        return H2OLocalServer(proc, ip, port)

    @property
    def ip(self):
        return self._ip

    @property
    def port(self):
        return self._port

    @property
    def scheme(self):
        return self._scheme

    @property
    def url(self):
        return f"{self._scheme}://{self._ip}:{self._port}"

    def is_running(self):
        return self._process is not None and self._process.poll() is None

    def shutdown(self):
        if self._process is not None and self._process.poll() is None:
            self._process.terminate()
            try:
                self._process.wait(10)
            except subprocess.TimeoutExpired:
                self._process.kill()
        self._process = None


def H2OCluster():
    from .. import cluster
    return cluster()


__all__ = ["H2OConnection", "H2OLocalServer", "H2OCluster"]
