"""Object-store persist backends over REST (io/persist_store.py; reference PersistS3 / PersistGcs / PersistHdfs):
AWS Signature V4 against the published get-vanilla vector, then ``import_file`` of s3:// (signed, path style,
ListObjectsV2 prefixes), gs:// (JSON API) and hdfs:// (WebHDFS with the datanode redirect) from local mock servers,
and the ``set_s3_credentials`` client / ``/3/PersistS3`` REST route."""
import http.server
import json
import threading
import urllib.parse

import numpy as np
import pandas as pd
import pytest

import h2o
from llama_github_io_amd.io import persist_store as PS
from llama_github_io_amd.io import persist_url as PU

KEY, SECRET = "AKIDEXAMPLE", "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY"


def test_sigv4_get_vanilla_vector():
    """aws-sig-v4-test-suite get-vanilla: GET / on example.amazonaws.com, service 'service', 20150830T123600Z."""
    h = PS.sigv4_headers("GET", "https://example.amazonaws.com/", "us-east-1", "service", KEY, SECRET,
                         amz_date="20150830T123600Z")
    assert h["Authorization"] == ("AWS4-HMAC-SHA256 Credential=AKIDEXAMPLE/20150830/us-east-1/service/aws4_request, "
                                  "SignedHeaders=host;x-amz-date, "
                                  "Signature=5fa00fa31553b73ebf1942676e86291e8372ff2a2260956d9b8aae1d763fbf31")


def _csv(seed, n=50):
    rng = np.random.default_rng(seed)
    return pd.DataFrame({"a": rng.normal(size=n), "b": rng.integers(0, 4, n)}).to_csv(index=False).encode()


class _Store(http.server.BaseHTTPRequestHandler):
    objects: dict = {}
    seen: list = []

    def log_message(self, *a, **k):
        pass

    def _send(self, code, body=b"", ctype="application/octet-stream", extra=None):
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        for k, v in (extra or {}).items():
            self.send_header(k, v)
        self.end_headers()
        self.wfile.write(body)

    def do_GET(self):  # noqa: N802
        u = urllib.parse.urlsplit(self.path)
        q = dict(urllib.parse.parse_qsl(u.query, keep_blank_values=True))
        self.seen.append((u.path, q, dict(self.headers)))
        path = urllib.parse.unquote(u.path)
        if path.startswith("/webhdfs/v1"):
            return self._hdfs(path[len("/webhdfs/v1"):], q)
        if path.startswith("/storage/v1/b/"):
            return self._gcs(path, q)
        return self._s3(u, path, q)

    # --- S3, path style: /bucket/key; checks the SigV4 signature of what was actually sent
    def _s3(self, u, path, q):
        auth = self.headers.get("Authorization", "")
        amz = self.headers.get("x-amz-date", "")
        url = f"http://{self.headers['Host']}{u.path}" + (f"?{u.query}" if u.query else "")
        want = PS.sigv4_headers("GET", url, "us-east-1", "s3", KEY, SECRET, amz_date=amz,
                                payload_hash=self.headers.get("x-amz-content-sha256"))["Authorization"]
        if auth != want:
            return self._send(403, b"<Error><Code>SignatureDoesNotMatch</Code></Error>", "application/xml")
        bucket, _, key = path.lstrip("/").partition("/")
        if q.get("list-type") == "2":
            keys = sorted(k for (b, k) in self.objects if b == bucket and k.startswith(q.get("prefix", "")))
            body = ('<?xml version="1.0"?><ListBucketResult xmlns="http://s3.amazonaws.com/doc/2006-03-01/">'
                    + "".join(f"<Contents><Key>{k}</Key></Contents>" for k in keys)
                    + "<IsTruncated>false</IsTruncated></ListBucketResult>").encode()
            return self._send(200, body, "application/xml")
        if (bucket, key) in self.objects:
            return self._send(200, self.objects[(bucket, key)])
        return self._send(404, b"<Error><Code>NoSuchKey</Code></Error>", "application/xml")

    # --- GCS JSON API
    def _gcs(self, path, q):
        rest = path[len("/storage/v1/b/"):]
        bucket, _, tail = rest.partition("/o")
        if tail in ("", "/") and "prefix" in q:
            items = [{"name": k} for (b, k) in sorted(self.objects) if b == bucket and k.startswith(q["prefix"])]
            return self._send(200, json.dumps({"items": items}).encode(), "application/json")
        name = tail.lstrip("/")
        if q.get("alt") == "media" and (bucket, name) in self.objects:
            return self._send(200, self.objects[(bucket, name)])
        return self._send(404, b"{}", "application/json")

    # --- WebHDFS: OPEN answers with a redirect to a "datanode" URL on the same server
    def _hdfs(self, path, q):
        op = q.get("op")
        files = {k: v for (b, k), v in self.objects.items() if b == "hdfs"}
        if op == "GETFILESTATUS":
            if path in files:
                return self._send(200, json.dumps({"FileStatus": {"type": "FILE"}}).encode(), "application/json")
            if any(k.startswith(path.rstrip("/") + "/") for k in files):
                return self._send(200, json.dumps({"FileStatus": {"type": "DIRECTORY"}}).encode(), "application/json")
            return self._send(404, b"{}", "application/json")
        if op == "LISTSTATUS":
            base = path.rstrip("/") + "/"
            st = [{"pathSuffix": k[len(base):], "type": "FILE"} for k in files if k.startswith(base)]
            return self._send(200, json.dumps({"FileStatuses": {"FileStatus": st}}).encode(), "application/json")
        if op == "OPEN":
            if q.get("datanode") == "1":
                return self._send(200, files[path])
            loc = f"http://{self.headers['Host']}/webhdfs/v1{urllib.parse.quote(path)}?op=OPEN&datanode=1"
            return self._send(307, b"", extra={"Location": loc})
        return self._send(400, b"{}")


@pytest.fixture()
def store(monkeypatch):
    _Store.objects = {("bkt", "data/x.csv"): _csv(1), ("bkt", "data/y.csv"): _csv(2), ("bkt", "solo.csv"): _csv(3),
                      ("gbk", "p/q.csv"): _csv(4), ("gbk", "p/r.csv"): _csv(5),
                      ("hdfs", "/user/h2o/t1.csv"): _csv(6), ("hdfs", "/user/h2o/dir/a.csv"): _csv(7),
                      ("hdfs", "/user/h2o/dir/b.csv"): _csv(8)}
    _Store.seen = []
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _Store)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    port = srv.server_address[1]
    monkeypatch.setenv("H2O_S3_ENDPOINT", f"http://127.0.0.1:{port}")
    monkeypatch.setenv("H2O_S3_REGION", "us-east-1")
    monkeypatch.setenv("H2O_GCS_ENDPOINT", f"http://127.0.0.1:{port}")
    monkeypatch.setenv("H2O_WEBHDFS_PORT", str(port))
    monkeypatch.setattr(PU, "_cache", {})
    h2o.init(verbose=False)
    yield port
    PS.remove_s3_credentials()
    srv.shutdown()


def test_s3_signed_object_and_prefix(store):
    PS.set_s3_credentials(KEY, SECRET)
    fr = h2o.import_file("s3://bkt/solo.csv")
    assert fr.shape == (50, 2)
    ref = pd.read_csv(pd.io.common.BytesIO(_csv(3)))
    np.testing.assert_allclose(fr.as_data_frame()["a"].to_numpy(float), ref["a"].to_numpy(), rtol=1e-12)
    both = h2o.import_file("s3a://bkt/data/")                 # a prefix: every object under it
    assert both.shape == (100, 2)
    lists = [q for (p, q, h) in _Store.seen if q.get("list-type") == "2"]
    assert lists and lists[0]["prefix"] == "data/"
    assert all("AWS4-HMAC-SHA256 Credential=AKIDEXAMPLE/" in h.get("Authorization", "") for (p, q, h) in _Store.seen)


def test_s3_bad_credentials_and_missing(store):
    PS.set_s3_credentials(KEY, "wrong-secret")
    with pytest.raises(FileNotFoundError):
        h2o.import_file("s3://bkt/solo.csv")
    PS.set_s3_credentials(KEY, SECRET)
    with pytest.raises(FileNotFoundError, match="not found"):
        h2o.import_file("s3://bkt/nothing/here.csv")
    with pytest.raises(ValueError, match="must not be empty"):
        PS.set_s3_credentials("", "x")


def test_gcs_and_webhdfs(store):
    g = h2o.import_file("gs://gbk/p/")
    assert g.shape == (100, 2)
    one = h2o.import_file("gs://gbk/p/q.csv")
    assert one.shape == (50, 2)
    f = h2o.import_file("hdfs://127.0.0.1/user/h2o/t1.csv")
    assert f.shape == (50, 2)
    d = h2o.import_file("hdfs://127.0.0.1/user/h2o/dir")
    assert d.shape == (100, 2)
    ref = pd.concat([pd.read_csv(pd.io.common.BytesIO(_csv(s))) for s in (7, 8)])
    np.testing.assert_allclose(np.sort(d.as_data_frame()["a"].to_numpy(float)), np.sort(ref["a"].to_numpy()), rtol=1e-12)


def test_set_s3_credentials_client_and_rest(store):
    pytest.importorskip("fastapi")
    from fastapi.testclient import TestClient
    from llama_github_io_amd.api.server import create_app
    h2o.set_s3_credentials(KEY, SECRET)
    assert PS._credentials()["secret"] == SECRET
    h2o.remove_s3_credentials()
    assert PS._credentials() is None
    c = TestClient(create_app(), raise_server_exceptions=False)
    r = c.post("/3/PersistS3", data={"secret_key_id": KEY, "secret_access_key": SECRET})
    assert r.status_code == 200 and r.json()["secret_key_id"] == KEY
    assert PS._credentials()["key"] == KEY
    r = c.request("DELETE", "/3/PersistS3", data={"secret_key_id": "delete", "secret_access_key": "delete"})
    assert r.status_code == 200 and PS._credentials() is None
