"""URL persist backends for ``import_file`` / ``/3/ImportFiles`` (reference: ``water/persist/PersistManager.java``
``importFiles`` and ``PersistEagerHTTP.java``, ``h2o-persist-http/.../PersistHTTP.java``).

``http://`` and ``https://`` sources are fetched whole (the reference's eager HTTP persist reads the body into one
``Key`` before the parse); the body lands in a per-process cache file that keeps the URL's file name, so the parse
type guess (``.csv``, ``.gz``, ``.zip``, ``.parquet``, ...) and the destination frame name work as for a local file.
A URL that was already fetched in this process is not fetched again unless ``refresh`` is asked for.

Object stores (``s3://``, ``s3a://``, ``s3n://``, ``gs://``, ``hdfs://``) are read through their REST protocols
(``persist_store``: S3 with Signature V4, the Cloud Storage JSON API, WebHDFS) into the same cache; ``maprfs://``
fails with an error naming the scheme.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import tempfile
import threading
import urllib.parse
import urllib.request

HTTP_SCHEMES = ("http", "https")
STORE_SCHEMES = ("s3", "s3a", "s3n", "gs", "hdfs", "maprfs")

_lock = threading.Lock()
_cache: dict[str, str] = {}
_dir: str | None = None


def scheme(path) -> str:
    s = urllib.parse.urlsplit(str(path)).scheme.lower()
    return s if len(s) > 1 else ""          # "C:\\..." style drive letters are not schemes


def is_url(path) -> bool:
    return scheme(path) in HTTP_SCHEMES


def _cache_dir() -> str:
    global _dir
    if _dir is None:
        _dir = tempfile.mkdtemp(prefix="h2o_persist_http_")
    return _dir


def _file_name(url: str) -> str:
    p = urllib.parse.urlsplit(url)
    base = os.path.basename(urllib.parse.unquote(p.path.rstrip("/"))) or "index"
    return base


def fetch(url: str, refresh: bool = False, timeout: float = 600.0) -> str:
    """Download ``url`` (GET, redirects followed) into the cache; returns the local file path.
    PersistEagerHTTP: a non-2xx answer is an error, the body is taken whole."""
    req = urllib.request.Request(url, headers={"User-Agent": "h2o-mi355x/persist-http"})
    return download(url, lambda t: urllib.request.urlopen(req, timeout=t), _file_name(url), refresh, timeout)


def download(key: str, opener, name: str, refresh: bool = False, timeout: float = 600.0) -> str:
    """Body of ``opener(timeout)`` (a urllib response) into the cache under ``key`` (file name ``name``)."""
    url = key
    with _lock:
        if not refresh and url in _cache and os.path.exists(_cache[url]):
            return _cache[url]
        sub = os.path.join(_cache_dir(), hashlib.sha1(url.encode()).hexdigest()[:16])
        os.makedirs(sub, exist_ok=True)
        dst = os.path.join(sub, name or "object")
        try:
            with opener(timeout) as r, open(dst + ".part", "wb") as f:
                code = getattr(r, "status", 200)
                if code // 100 != 2:
                    raise OSError(f"HTTP {code} for {url}")
                shutil.copyfileobj(r, f, 1 << 20)
        except Exception as e:        # noqa: BLE001 - re-raised with the reference's framing
            if os.path.exists(dst + ".part"):
                os.remove(dst + ".part")
            raise FileNotFoundError(f"Unable to import file from URL {url}: {e}") from e
        os.replace(dst + ".part", dst)
        _cache[url] = dst
        return dst


def resolve(path) -> list | None:
    """Local files for a URL source, or None when ``path`` is not a URL."""
    s = scheme(path)
    if s in HTTP_SCHEMES:
        return [fetch(str(path))]
    if s in ("s3", "s3a", "s3n", "gs", "hdfs"):
        from . import persist_store
        return persist_store.resolve(str(path), lambda key, opener, name: download(key, opener, name))
    if s in STORE_SCHEMES:
        raise ValueError(f"persist backend for '{s}://' is not available in this build (the reference reads it "
                         f"through its {s.upper()} SDK; copy the file to a local or http(s) location instead)")
    return None
