"""Connections (reference: ``h2o-py/h2o/backend/connection.py`` ``H2OConnection``).

* :class:`InProcessConnection` (default after ``h2o.init()``): ``h2o.api(...)`` is served by the REST
  application of this process (``api/server.py``) through one cached ASGI test client, no socket.
* :class:`RemoteConnection` (``h2o.connect(url=...)`` / ``ip=, port=``): a real HTTP session to a
  running server (this framework's ``python -m llama_github_io_amd.api.server`` or any server speaking
  the H2O V3 wire format): the cloud is verified on ``GET /3/Cloud``, a session is opened on
  ``POST /4/sessions`` and closed on ``close()``. Every ``h2o.api`` call, ``h2o.ls``, ``h2o.remove``,
  ``h2o.cluster().show_status`` and ``h2o.get_frame(...).as_data_frame`` style REST round-trips then
  go to that server. (The stock h2o-py client is wire-compatible with the server as well.)
"""
from __future__ import annotations

import json as _json


class _Base:
    def request(self, endpoint, data=None, json=None, filename=None, save_to=None):
        method, _, path = endpoint.partition(" ")
        method = method.upper()
        files = None
        if filename is not None:
            files = {"file": open(filename, "rb")}
        try:
            r = self._send(method, path, data, json, files)
        finally:
            if files:
                files["file"].close()
        if r.status_code >= 400:
            try:
                body = r.json()
                msg = body.get("msg") or body.get("exception_msg") or str(body)
            except ValueError:
                msg = r.text
            raise RuntimeError(f"{endpoint}: HTTP {r.status_code}: {msg}")
        if save_to:
            with open(save_to, "wb") as f:
                f.write(r.content)
            return save_to
        ctype = r.headers.get("content-type", "")
        return r.json() if "json" in ctype else r.content

    @staticmethod
    def _encode(data):
        if data is None:
            return None
        out = {}
        for k, v in data.items():
            if v is None:
                continue
            out[k] = _json.dumps(v) if isinstance(v, (list, dict)) else (str(v).lower() if isinstance(v, bool) else v)
        return out


class InProcessConnection(_Base):
    url = "inproc://"
    _client = None

    def _send(self, method, path, data, json, files):
        if InProcessConnection._client is None:
            from fastapi.testclient import TestClient
            from llama_github_io_amd.api.server import create_app
            InProcessConnection._client = TestClient(create_app())
        c = InProcessConnection._client
        enc = self._encode(data)
        return c.request(method, path, params=enc if method in ("GET", "DELETE") else None,
                         data=None if method in ("GET", "DELETE") or files else enc, json=json, files=files)

    def close(self):
        pass


class RemoteConnection(_Base):
    def __init__(self, url, verify_ssl_certificates=True, auth=None, timeout=None):
        import requests
        self.url = url.rstrip("/")
        self._s = requests.Session()
        self._s.verify = verify_ssl_certificates
        if auth is not None:
            self._s.auth = auth
        self._timeout = timeout
        self.cloud = self.request("GET /3/Cloud")
        self.session_id = self.request("POST /4/sessions").get("session_key")

    def _send(self, method, path, data, json, files):
        enc = self._encode(data)
        return self._s.request(method, self.url + path, params=enc if method in ("GET", "DELETE") else None,
                               data=None if method in ("GET", "DELETE") or files else enc, json=json, files=files,
                               timeout=self._timeout)

    def close(self):
        try:
            if getattr(self, "session_id", None):
                self.request(f"DELETE /4/sessions/{self.session_id}")
        finally:
            self._s.close()


_current = [None]


def current():
    return _current[0]


def set_current(c):
    old = _current[0]
    _current[0] = c
    if old is not None and old is not c:
        old.close()
    return c


def in_process():
    if _current[0] is None:
        _current[0] = InProcessConnection()
    return _current[0]


def is_remote() -> bool:
    return isinstance(_current[0], RemoteConnection)
