"""Object-store persist backends over their REST protocols (reference: ``h2o-persist-s3/.../PersistS3.java``,
``h2o-persist-gcs/.../PersistGcs.java``, ``h2o-persist-hdfs/.../PersistHdfs.java`` and
``h2o-py/h2o/persist/persist.py``).

The reference links the vendor SDKs (AWS SDK, google-cloud-storage, the Hadoop client). No SDK is part of this build,
so each store is spoken to through its documented HTTP API with the standard library only:

* ``s3://`` / ``s3a://`` / ``s3n://``: S3 REST with AWS Signature V4 (GetObject, ListObjectsV2 for prefixes).
  Credentials: :func:`set_s3_credentials` (``POST /3/PersistS3``, as ``h2o.set_s3_credentials``), else the
  ``AWS_ACCESS_KEY_ID`` / ``AWS_SECRET_ACCESS_KEY`` / ``AWS_SESSION_TOKEN`` environment; no credentials = anonymous.
  PersistS3's system properties map to environment variables: ``sys.ai.h2o.persist.s3.endPoint`` ->
  ``H2O_S3_ENDPOINT`` (e.g. ``http://127.0.0.1:9000`` for MinIO), ``...s3.region`` -> ``H2O_S3_REGION`` (default
  ``AWS_REGION`` or us-east-1), ``...s3.enable.path.style`` -> ``H2O_S3_PATH_STYLE`` (on by default with a custom
  endpoint).
* ``gs://``: the Cloud Storage JSON API (``/storage/v1/b/{bucket}/o/{object}?alt=media``, object listing for
  prefixes); ``GOOGLE_OAUTH_ACCESS_TOKEN`` is sent as a bearer token when set; ``H2O_GCS_ENDPOINT`` overrides
  ``https://storage.googleapis.com``.
* ``hdfs://host[:port]/path``: WebHDFS (``/webhdfs/v1/path?op=OPEN`` / ``LISTSTATUS``) on ``H2O_WEBHDFS_PORT`` (default
  9870, the NameNode HTTP port); ``HADOOP_USER_NAME`` becomes ``user.name``.

Objects are downloaded whole into the persist cache (``persist_url``), like the reference's eager HTTP persist; a
prefix ending in ``/`` (or naming no object) imports every object under it.
"""
from __future__ import annotations

import datetime as _dt
import hashlib
import hmac
import json
import os
import threading
import urllib.error
import urllib.parse
import urllib.request
import xml.etree.ElementTree as ET

S3_SCHEMES = ("s3", "s3a", "s3n")
_creds_lock = threading.Lock()
_s3_creds: dict | None = None


# ------------------------------------------------------------------------------------------------ credentials
def set_s3_credentials(secret_key_id: str, secret_access_key: str, session_token: str | None = None) -> None:
    """PersistS3Handler.setS3Credentials: credentials used by every later ``s3://`` import of this process."""
    if secret_key_id is None:
        raise ValueError("Secret key ID must be specified")
    if secret_access_key is None:
        raise ValueError("Secret access key must be specified")
    if not secret_key_id:
        raise ValueError("Secret key ID must not be empty")
    if not secret_access_key:
        raise ValueError("Secret access key must not be empty")
    global _s3_creds
    with _creds_lock:
        _s3_creds = dict(key=str(secret_key_id), secret=str(secret_access_key),
                         token=None if session_token in (None, "") else str(session_token))


def remove_s3_credentials() -> None:
    global _s3_creds
    with _creds_lock:
        _s3_creds = None


def _credentials() -> dict | None:
    with _creds_lock:
        if _s3_creds is not None:
            return dict(_s3_creds)
    k, s = os.environ.get("AWS_ACCESS_KEY_ID"), os.environ.get("AWS_SECRET_ACCESS_KEY")
    if k and s:
        return dict(key=k, secret=s, token=os.environ.get("AWS_SESSION_TOKEN") or None)
    return None


# ------------------------------------------------------------------------------------------------ SigV4
def _sha256(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def _hmac(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode("utf-8"), hashlib.sha256).digest()


def sigv4_headers(method: str, url: str, region: str, service: str, key: str, secret: str,
                  token: str | None = None, amz_date: str | None = None, payload_hash: str | None = None,
                  extra_headers: dict | None = None) -> dict:
    """Headers (``Authorization``, ``x-amz-date``, ... ) of an AWS Signature Version 4 request."""
    u = urllib.parse.urlsplit(url)
    host = u.netloc
    if amz_date is None:
        amz_date = _dt.datetime.now(_dt.timezone.utc).strftime("%Y%m%dT%H%M%SZ")
    date = amz_date[:8]
    hdrs = {"host": host, "x-amz-date": amz_date}
    if payload_hash is not None:
        hdrs["x-amz-content-sha256"] = payload_hash
    if token:
        hdrs["x-amz-security-token"] = token
    for k, v in (extra_headers or {}).items():
        hdrs[k.lower()] = str(v).strip()
    # canonical URI: every path segment URI-encoded once (S3: no double encoding), '/' kept
    path = u.path or "/"
    curi = "/".join(urllib.parse.quote(urllib.parse.unquote(seg), safe="-_.~") for seg in path.split("/"))
    q = urllib.parse.parse_qsl(u.query, keep_blank_values=True)
    cq = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}"
                  for k, v in sorted(q))
    names = sorted(hdrs)
    ch = "".join(f"{n}:{hdrs[n]}\n" for n in names)
    sh = ";".join(names)
    creq = "\n".join([method, curi, cq, ch, sh, payload_hash or _sha256(b"")])
    scope = f"{date}/{region}/{service}/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, _sha256(creq.encode("utf-8"))])
    k = _hmac(("AWS4" + secret).encode("utf-8"), date)
    k = _hmac(k, region)
    k = _hmac(k, service)
    k = _hmac(k, "aws4_request")
    sig = hmac.new(k, sts.encode("utf-8"), hashlib.sha256).hexdigest()
    out = {n: hdrs[n] for n in names if n != "host"}
    out["Authorization"] = f"AWS4-HMAC-SHA256 Credential={key}/{scope}, SignedHeaders={sh}, Signature={sig}"
    return out


# ------------------------------------------------------------------------------------------------ S3
def _s3_config():
    ep = os.environ.get("H2O_S3_ENDPOINT") or os.environ.get("SYS_AI_H2O_PERSIST_S3_ENDPOINT")
    region = os.environ.get("H2O_S3_REGION") or os.environ.get("AWS_REGION") or "us-east-1"
    ps = os.environ.get("H2O_S3_PATH_STYLE")
    path_style = (ps.lower() in ("1", "true", "yes")) if ps else bool(ep)
    return ep, region, path_style


def _s3_url(bucket: str, key: str, query: str = "") -> str:
    ep, region, path_style = _s3_config()
    k = urllib.parse.quote(key, safe="/-_.~")
    if ep:
        base = ep.rstrip("/")
        if "://" not in base:
            base = "https://" + base
        url = f"{base}/{bucket}/{k}" if path_style else \
            urllib.parse.urlunsplit((urllib.parse.urlsplit(base).scheme, f"{bucket}.{urllib.parse.urlsplit(base).netloc}",
                                     "/" + k, "", ""))
    else:
        url = f"https://{bucket}.s3.{region}.amazonaws.com/{k}" if not path_style else \
            f"https://s3.{region}.amazonaws.com/{bucket}/{k}"
    return url + (("?" + query) if query else "")


def _s3_request(url: str, timeout: float):
    _, region, _ = _s3_config()
    c = _credentials()
    hdrs = {"User-Agent": "h2o-mi355x/persist-s3"}
    if c is not None:
        hdrs.update(sigv4_headers("GET", url, region, "s3", c["key"], c["secret"], c["token"],
                                  payload_hash="UNSIGNED-PAYLOAD"))
    return urllib.request.urlopen(urllib.request.Request(url, headers=hdrs), timeout=timeout)


def _s3_list(bucket: str, prefix: str, timeout: float) -> list:
    """ListObjectsV2 (continuation tokens followed): object keys under ``prefix``."""
    keys, token = [], None
    while True:
        q = {"list-type": "2", "prefix": prefix}
        if token:
            q["continuation-token"] = token
        url = _s3_url(bucket, "", urllib.parse.urlencode(sorted(q.items())))
        with _s3_request(url, timeout) as r:
            root = ET.fromstring(r.read())
        ns = root.tag[: root.tag.index("}") + 1] if root.tag.startswith("{") else ""
        for c in root.findall(f"{ns}Contents"):
            k = c.findtext(f"{ns}Key")
            if k and not k.endswith("/"):
                keys.append(k)
        if (root.findtext(f"{ns}IsTruncated") or "false").lower() != "true":
            break
        token = root.findtext(f"{ns}NextContinuationToken")
        if not token:
            break
    return keys


# ------------------------------------------------------------------------------------------------ GCS
def _gcs_base() -> str:
    return (os.environ.get("H2O_GCS_ENDPOINT") or "https://storage.googleapis.com").rstrip("/")


def _gcs_request(url: str, timeout: float):
    hdrs = {"User-Agent": "h2o-mi355x/persist-gcs"}
    tok = os.environ.get("GOOGLE_OAUTH_ACCESS_TOKEN")
    if tok:
        hdrs["Authorization"] = f"Bearer {tok}"
    return urllib.request.urlopen(urllib.request.Request(url, headers=hdrs), timeout=timeout)


def _gcs_list(bucket: str, prefix: str, timeout: float) -> list:
    names, page = [], None
    while True:
        q = {"prefix": prefix}
        if page:
            q["pageToken"] = page
        url = f"{_gcs_base()}/storage/v1/b/{urllib.parse.quote(bucket, safe='')}/o?{urllib.parse.urlencode(q)}"
        with _gcs_request(url, timeout) as r:
            d = json.loads(r.read())
        names += [it["name"] for it in d.get("items", []) if not it["name"].endswith("/")]
        page = d.get("nextPageToken")
        if not page:
            break
    return names


def _gcs_object_url(bucket: str, name: str) -> str:
    return (f"{_gcs_base()}/storage/v1/b/{urllib.parse.quote(bucket, safe='')}/o/"
            f"{urllib.parse.quote(name, safe='')}?alt=media")


# ------------------------------------------------------------------------------------------------ WebHDFS
def _webhdfs_url(host: str, path: str, op: str) -> str:
    port = int(os.environ.get("H2O_WEBHDFS_PORT", "9870"))
    q = {"op": op}
    user = os.environ.get("HADOOP_USER_NAME")
    if user:
        q["user.name"] = user
    scheme = os.environ.get("H2O_WEBHDFS_SCHEME", "http")
    return f"{scheme}://{host}:{port}/webhdfs/v1{urllib.parse.quote(path or '/', safe='/-_.~')}?{urllib.parse.urlencode(q)}"


def _webhdfs_list(host: str, path: str, timeout: float) -> list:
    with urllib.request.urlopen(_webhdfs_url(host, path, "GETFILESTATUS"), timeout=timeout) as r:
        st = json.loads(r.read())["FileStatus"]
    if st.get("type") != "DIRECTORY":
        return [path]
    with urllib.request.urlopen(_webhdfs_url(host, path, "LISTSTATUS"), timeout=timeout) as r:
        items = json.loads(r.read())["FileStatuses"]["FileStatus"]
    base = path.rstrip("/")
    return [f"{base}/{it['pathSuffix']}" for it in sorted(items, key=lambda it: it["pathSuffix"])
            if it.get("type") == "FILE"]


# ------------------------------------------------------------------------------------------------ resolve
def resolve(path: str, fetch, timeout: float = 600.0) -> list:
    """Local cache files of every object a store URL names (one object, or all under a prefix / directory).
    ``fetch(url, opener, name)`` downloads one object through ``opener(timeout)`` into the persist cache."""
    try:
        return _resolve(path, fetch, timeout)
    except urllib.error.URLError as e:           # listing / status calls: the reference's framing of import errors
        raise FileNotFoundError(f"Unable to import file from URL {path}: {e}") from e


def _resolve(path: str, fetch, timeout: float) -> list:
    u = urllib.parse.urlsplit(str(path))
    s = u.scheme.lower()
    if s in S3_SCHEMES:
        bucket, key = u.netloc, urllib.parse.unquote(u.path.lstrip("/"))
        keys = [key] if key and not key.endswith("/") else []
        if keys:
            try:
                return [fetch(f"s3://{bucket}/{key}", lambda t, k=key: _s3_request(_s3_url(bucket, k), t),
                              os.path.basename(key))]
            except FileNotFoundError:
                keys = []
        keys = _s3_list(bucket, key, timeout)
        if not keys:
            raise FileNotFoundError(f"Object not found: {path}")
        return [fetch(f"s3://{bucket}/{k}", lambda t, k=k: _s3_request(_s3_url(bucket, k), t), os.path.basename(k))
                for k in keys]
    if s == "gs":
        bucket, name = u.netloc, urllib.parse.unquote(u.path.lstrip("/"))
        if name and not name.endswith("/"):
            try:
                return [fetch(f"gs://{bucket}/{name}",
                              lambda t, n=name: _gcs_request(_gcs_object_url(bucket, n), t), os.path.basename(name))]
            except FileNotFoundError:
                pass
        names = _gcs_list(bucket, name, timeout)
        if not names:
            raise FileNotFoundError(f"Object not found: {path}")
        return [fetch(f"gs://{bucket}/{n}", lambda t, n=n: _gcs_request(_gcs_object_url(bucket, n), t),
                      os.path.basename(n)) for n in names]
    if s == "hdfs":
        host = u.hostname or "localhost"
        files = _webhdfs_list(host, urllib.parse.unquote(u.path), timeout)
        return [fetch(f"hdfs://{host}{f}",
                      lambda t, f=f: urllib.request.urlopen(_webhdfs_url(host, f, "OPEN"), timeout=t),
                      os.path.basename(f)) for f in files]
    raise ValueError(f"not an object-store URL: {path}")
