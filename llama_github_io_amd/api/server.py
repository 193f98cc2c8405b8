"""REST API (reference: ``h2o-core/src/main/java/water/api/RegisterV3Api.java`` routes and the V3/V99
schemas: ``CloudV3``, ``FramesV3``, ``ParseSetupV3``, ``ModelBuildersV3``, ``ModelsV3``,
``JobsV3``, ``ModelMetricsListSchemaV3``, ``RapidsSchemaV3``, ``GridSearchSchema``, ``AutoMLV99``).

FastAPI app exposing the endpoints the h2o clients use, on top of the in-process engine (frames in
HBM, models trained by the HIP kernels). Model builds and AutoML/grid searches run as async
``Job``s (``/3/Jobs/{key}`` polling, ``/3/Jobs/{key}/cancel``). Run with
``python -m llama_github_io_amd.api.server --port 54321``.
"""
from __future__ import annotations

import json
import math
import os
import time

import numpy as np

from ..core import dkv, runtime
from ..core.job import Job, list_jobs
from ..frame import H2OFrame
from ..models import builder
from ..models.base import Model
from . import v3

try:
    from fastapi import FastAPI, HTTPException, Request
    from fastapi.responses import FileResponse, JSONResponse
except ImportError:  # pragma: no cover
    FastAPI = None

_timeline = []


def _clean(o):
    """JSON-safe conversion (NaN/inf -> None, numpy/torch -> python)."""
    import torch
    if isinstance(o, dict):
        return {str(k): _clean(v) for k, v in o.items() if not str(k).startswith("_")}
    if isinstance(o, (list, tuple)):
        return [_clean(v) for v in o]
    if isinstance(o, (np.floating, float)):
        f = float(o)
        return None if math.isnan(f) or math.isinf(f) else f
    if isinstance(o, (np.integer,)):
        return int(o)
    if isinstance(o, np.ndarray):
        return _clean(o.tolist())
    if isinstance(o, torch.Tensor):
        return _clean(o.detach().cpu().tolist())
    if isinstance(o, (str, int, bool)) or o is None:
        return o
    return str(o)


def _frame_json_legacy(fr: H2OFrame, row_offset=0, row_count=10, full=False):
    cols = []
    for n in fr.names:
        c = fr._col(n)
        entry = dict(label=n, type={"real": "real", "int": "int", "enum": "enum", "string": "string",
                                    "time": "time"}.get(c.type, c.type))
        if c.type == "enum":
            entry["domain"] = list(c.domain)
            entry["domain_cardinality"] = len(c.domain)
        if c.type in ("real", "int", "time") and full:
            v = c.data
            ok = ~v.isnan()
            vv = v[ok]
            entry.update(mins=[float(vv.min())] if vv.numel() else [None], maxs=[float(vv.max())] if vv.numel() else [None],
                         mean=float(vv.mean()) if vv.numel() else None, sigma=float(vv.std()) if vv.numel() > 1 else None,
                         missing_count=int((~ok).sum()))
        data = c.to_numpy()[row_offset:row_offset + row_count]
        entry["data"] = [None if x is None or (isinstance(x, float) and math.isnan(x)) else
                         (x if not isinstance(x, (np.floating, np.integer)) else x.item()) for x in data]
        cols.append(entry)
    return dict(frame_id=dict(name=fr.frame_id, type="Key<Frame>"), rows=fr.nrows, row_count=min(row_count, fr.nrows),
                row_offset=row_offset, num_columns=fr.ncols, columns=cols, is_text=False)


def _model_json(m: Model):
    return v3.model(m)


def _model_json_legacy(m: Model):
    out = dict(model_id=dict(name=m.key, type="Key<Model>"), algo=m.algo, algo_full_name=m.algo,
               response_column_name=m.info.response, parameters=[dict(name=k, actual_value=v) for k, v in m.params.items()],
               output=dict(m.output, model_category=m.model_category, names=m.info.x + ([m.info.response] if m.info.response else []),
                           domains=m.info.domains + ([m.info.response_domain] if m.info.response else [])))
    return _clean(out)


def _unquote(v):
    if isinstance(v, str) and len(v) >= 2 and v[0] == v[-1] == '"':
        return v[1:-1]
    if isinstance(v, list):
        return [_unquote(x) for x in v]
    return v


def _parse_params(raw: dict) -> dict:
    out = {}
    for k, v in raw.items():
        if isinstance(v, str):
            s = v.strip()
            if s in ("null", "None"):
                out[k] = None
                continue
            if s.startswith("[") or s.startswith("{"):
                try:
                    v = _unquote(json.loads(s))
                except ValueError:
                    try:
                        v = _unquote(json.loads(s.replace("'", '"')))
                    except ValueError:
                        v = [x.strip().strip('"') for x in s.strip("[]").split(",") if x.strip()]
            elif s.lower() in ("true", "false"):
                v = s.lower() == "true"
            else:
                try:
                    v = int(s)
                except ValueError:
                    try:
                        v = float(s)
                    except ValueError:
                        pass
        out[k] = v
    return out


async def _params(request: Request) -> dict:
    q = dict(request.query_params)
    ct = request.headers.get("content-type", "")
    if "json" in ct:
        body = await request.json()
        q.update(body or {})
    else:  # application/x-www-form-urlencoded (python-multipart is not needed for this)
        from urllib.parse import parse_qsl
        raw = (await request.body()).decode("utf-8", "replace")
        q.update(dict(parse_qsl(raw, keep_blank_values=True)))
    return _parse_params(q)


def _multipart_first_file(body: bytes, boundary: str):
    """The first file part of a multipart/form-data body (python-multipart is not in the image)."""
    sep = b"--" + boundary.encode()
    for part in body.split(sep):
        if b"\r\n\r\n" not in part:
            continue
        head, _, data = part.partition(b"\r\n\r\n")
        if b"filename=" in head or b"name=" in head:
            fname = "upload"
            h = head.decode("latin-1")
            if 'filename="' in h:
                fname = h.split('filename="', 1)[1].split('"', 1)[0]
            if data.endswith(b"\r\n"):
                data = data[:-2]
            return data, fname
    return body, "upload"


def create_app(client_disconnect_timeout: float | None = None, login=None):
    """``client_disconnect_timeout`` (seconds; env ``H2O_CLIENT_DISCONNECT_TIMEOUT``) starts the
    ClientDisconnectCheckThread equivalent (``api/clients.py``). ``login`` (``api/security.LoginConfig``): the
    ``-hash_login -login_conf [-form_auth -session_timeout]`` authentication of every route."""
    if FastAPI is None:
        raise RuntimeError("fastapi is not installed")
    runtime.init()
    app = FastAPI(title="H2O (MI355X-native) REST API", version="3.46.0.amd0")
    from . import clients as _clients
    cdt = client_disconnect_timeout
    if cdt is None and os.environ.get("H2O_CLIENT_DISCONNECT_TIMEOUT"):
        cdt = float(os.environ["H2O_CLIENT_DISCONNECT_TIMEOUT"])
    if cdt:
        _clients.start(cdt)

    def _client_id(request):
        return request.headers.get("X-H2O-Client") or (request.client.host if request.client else "local")

    @app.middleware("http")
    async def timeline(request, call_next):
        _clients.touch(_client_id(request))
        t0 = time.time()
        resp = await call_next(request)
        _timeline.append(dict(time=int(t0 * 1000), method=request.method, url=str(request.url.path),
                              duration_ms=int((time.time() - t0) * 1000), status=resp.status_code))
        del _timeline[:-1000]
        return resp

    @app.exception_handler(Exception)
    async def errors(request, exc):
        status = 404 if isinstance(exc, KeyError) else (412 if isinstance(exc, (ValueError, TypeError)) else 500)
        return JSONResponse(status_code=status, content=v3.error(str(exc), exc, status))

    # ---- cloud, sessions, metadata
    @app.get("/3/Cloud")
    @app.head("/3/Cloud")
    def cloud():
        return v3.cloud(runtime.cluster_status())

    @app.get("/3/Ping")
    def ping():
        st = runtime.cluster_status()
        return {"__meta": v3.meta("PingV3", "Iced"), "cloud_uptime_millis": st["cloud_uptime_millis"],
                "cloud_healthy": bool(st["cloud_healthy"]), "nodes": v3.cloud(st)["nodes"]}

    @app.get("/3/Metadata/schemas/{name}")
    def schema_meta(name: str):
        if name not in v3.SCHEMA_FIELDS and (name.startswith("AutoML") or name.endswith(("V3", "V4", "V99"))):
            v3.SCHEMA_FIELDS.setdefault(name, [])
        r = v3.schema_metadata(name)
        if r is None:
            raise KeyError(f"unknown schema {name}")
        return r

    @app.post("/4/sessions")
    def new_session(request: Request):
        sid = dkv.new_key("_sid")
        _clients.touch(_client_id(request), sid)
        return {"__meta": v3.meta("SessionIdV4", "Iced", 4), "session_key": sid}

    @app.get("/3/Clients")
    def list_clients():
        now = time.time()
        return {"__meta": v3.meta("ClientsV3", "Iced"), "client_disconnect_timeout": cdt,
                "clients": [dict(client=k, last_heard_ms_ago=int((now - v["last_heard"]) * 1000), sessions=v["sessions"])
                            for k, v in _clients.clients().items()]}

    @app.delete("/4/sessions/{sid}")
    def end_session(sid: str):
        _clients.end_session(sid)
        return {"__meta": v3.meta("SessionIdV4", "Iced", 4), "session_key": sid}

    @app.get("/3/SessionProperties")
    @app.post("/3/SessionProperties")
    async def session_props(request: Request):
        p = await _params(request)
        return {"__meta": v3.meta("SessionPropertyV3", "Iced"), "session_key": p.get("session_key"),
                "key": p.get("key"), "value": p.get("value")}

    @app.get("/3/Capabilities")
    @app.get("/3/Capabilities/{kind}")
    def capabilities(kind: str = "All"):
        caps = [dict(name="GPU", value="MI355X (HIP)"), dict(name="Algos", value=",".join(sorted(builder.REGISTRY)))]
        return {"__meta": v3.meta("CapabilitiesV3", "Iced"),
                "capabilities": [{"__meta": v3.meta("CapabilityEntryV3", "Iced"), "name": c["name"]} for c in caps]}

    @app.post("/3/LogAndEcho")
    async def log_and_echo(request: Request):
        p = await _params(request)
        from ..utils import log
        log.info(str(p.get("message", "")))
        return {"__meta": v3.meta("LogAndEchoV3", "Iced"), "message": p.get("message", "")}

    @app.get("/3/About")
    def about():
        st = runtime.cluster_status()
        return dict(entries=[dict(name="Build project version", value=st["version"]),
                             dict(name="Device", value=st["device"])])

    @app.get("/3/Metadata/endpoints")
    def endpoints():
        return dict(routes=[dict(http_method=list(r.methods)[0] if getattr(r, "methods", None) else "GET", url_pattern=r.path)
                            for r in app.routes])

    @app.post("/3/InitID")
    @app.get("/3/InitID")
    def init_id():
        return dict(session_key=dkv.new_key("_sid"))

    @app.post("/3/Shutdown")
    def shutdown():
        runtime.shutdown()
        return dict(status="shutdown")

    @app.get("/3/Timeline")
    def tl():
        from ..utils import timeline
        return _clean(dict(events=timeline.events(1000), http=_timeline[-200:]))

    @app.get("/3/Logs")
    @app.get("/3/Logs/nodes/{node}/files/{name}")
    def logs(node: str = "self", name: str = "default"):
        from ..utils import log
        return dict(log="\n".join(log.recent(2000)))

    @app.get("/3/Profiler")
    def profiler(depth: int = 10):
        from ..utils import timeline
        return dict(nodes=[dict(node_name="self", profile=timeline.stacks())])

    @app.get("/3/WaterMeterMemory")
    @app.get("/3/MemoryStats")
    def memstats():
        from ..utils import memory
        return _clean(memory.stats())

    @app.post("/3/GarbageCollect")
    def gc():
        from ..utils import memory
        return dict(spilled_bytes=memory.clean())

    @app.delete("/3/DKV")
    def dkv_clear():
        return dict(removed=dkv.remove_all())

    @app.delete("/3/DKV/{key}")
    def dkv_rm(key: str):
        dkv.remove(key)
        return {"__meta": v3.meta("RemoveV3", "Iced"), "key": v3.key(key)}

    # ---- object-store credentials (PersistS3Handler: POST sets, DELETE removes; the schema is echoed back)
    @app.post("/3/PersistS3")
    async def persist_s3_set(request: Request):
        from ..io import persist_store
        p = await _params(request)
        kid, sec, tok = p.get("secret_key_id"), p.get("secret_access_key"), p.get("session_token")
        if kid is None:
            raise ValueError("The field 'S3_SECRET_KEY_ID' may not be null.")
        if sec is None:
            raise ValueError("The field 'S3_SECRET_ACCESS_KEY' may not be null.")
        kid, sec = str(kid).strip(), str(sec).strip()
        tok = None if tok in (None, "None") else str(tok).strip()
        if tok is not None and not tok:
            raise ValueError("The field 'S3_SESSION_TOKEN' may not be empty")
        persist_store.set_s3_credentials(kid, sec, tok)
        return {"__meta": v3.meta("PersistS3CredentialsV3", "Iced"), "secret_key_id": kid, "secret_access_key": sec,
                "session_token": tok}

    @app.delete("/3/PersistS3")
    async def persist_s3_remove(request: Request):
        from ..io import persist_store
        p = await _params(request)
        persist_store.remove_s3_credentials()
        return {"__meta": v3.meta("PersistS3CredentialsV3", "Iced"), "secret_key_id": p.get("secret_key_id"),
                "secret_access_key": p.get("secret_access_key"), "session_token": p.get("session_token")}

    # ---- ingest
    @app.post("/3/ImportFiles")
    @app.get("/3/ImportFiles")
    async def import_files(request: Request):
        from ..io import parse as P
        p = await _params(request)
        path = p.get("path")
        files = P._expand(path)
        pat = p.get("pattern")
        if pat:
            import re
            files = [f for f in files if re.search(pat, os.path.basename(f))]
        return {"__meta": v3.meta("ImportFilesV3", "Iced"), "path": path, "pattern": pat, "files": files,
                "destination_frames": files, "fails": [], "dels": []}

    @app.post("/3/ImportFilesMulti")
    async def import_files_multi(request: Request):
        from ..io import parse as P
        p = await _params(request)
        paths = p.get("paths") or []
        paths = paths if isinstance(paths, list) else [paths]
        files, fails = [], []
        pat = p.get("pattern")
        import re
        for pth in paths:
            try:
                fl = P._expand(pth)
                files += [f for f in fl if not pat or re.search(pat, os.path.basename(f))]
            except FileNotFoundError:
                fails.append(pth)
        return {"__meta": v3.meta("ImportFilesMultiV3", "Iced"), "paths": paths, "pattern": pat, "files": files,
                "destination_frames": files, "fails": fails, "dels": []}

    @app.post("/3/ParseSetup")
    async def parse_setup(request: Request):
        from ..io import parse as P
        p = await _params(request)
        src = p.get("source_frames")
        src = [_unquote(x) for x in (src if isinstance(src, list) else [src])]
        sep = p.get("separator")
        sep = chr(sep) if isinstance(sep, int) else sep
        dt = p.get("decrypt_tool")
        dt = _unquote(dt.get("name") if isinstance(dt, dict) else dt) or None
        st = P.parse_setup(src[0], header=int(p.get("check_header", 0) or 0), separator=sep, decrypt_tool=dt)
        st = _clean(st)
        tmap = {"real": "Numeric", "int": "Numeric", "enum": "Enum", "string": "String", "time": "Time"}
        ctypes_ = [tmap.get(t, t) for t in (st.get("column_types") or [])]
        sepv = st.get("separator", ",")
        out = {"__meta": v3.meta("ParseSetupV3", "ParseSetup"),
               "source_frames": [v3.frame_key(f) for f in src], "parse_type": st.get("parse_type", "CSV"),
               "separator": ord(sepv) if isinstance(sepv, str) and sepv else 44, "single_quotes": False,
               "check_header": st.get("check_header", 1), "column_names": st.get("column_names"),
               "column_types": ctypes_, "na_strings": None, "column_name_filter": None, "column_offset": 0,
               "column_count": 0, "destination_frame": st.get("destination_frame") or P._dest_name(src[0]),
               "header_lines": 0, "number_columns": len(st.get("column_names") or []), "data": st.get("data"),
               "chunk_size": 4194304, "total_filtered_column_count": len(st.get("column_names") or []),
               "warnings": [], "skipped_columns": None, "custom_non_data_line_markers": None, "partition_by": None,
               "escapechar": 0, "force_col_types": False, "tz_adjust_to_local": False}
        return out

    @app.post("/3/Parse")
    async def parse(request: Request):
        from ..io import parse as P
        p = await _params(request)
        src = p.get("source_frames")
        src = [_unquote(x) for x in (src if isinstance(src, list) else [src])]
        dest = _unquote(p.get("destination_frame")) or P._dest_name(src[0])
        sep = p.get("separator")
        if isinstance(sep, int):
            sep = chr(sep)
        ct = p.get("column_types")
        if isinstance(ct, list):
            tmap = {"numeric": "real", "enum": "enum", "string": "string", "time": "time", "uuid": "string",
                    "categorical": "enum", "factor": "enum", "real": "real", "int": "int"}
            ct = [tmap.get(str(t).lower(), None) for t in ct]
        dt = p.get("decrypt_tool")
        dt = _unquote(dt.get("name") if isinstance(dt, dict) else dt) or None
        job = Job("Parse", dest=dest)
        job.run_async(P.import_file, src, dest, True, int(p.get("check_header", 0) or 0), sep,
                      p.get("column_names"), ct, p.get("na_strings"), decrypt_tool=dt)
        return {"__meta": v3.meta("ParseV3", "Iced"), "job": v3.job(job), "destination_frame": v3.frame_key(dest),
                "rows": 0}

    # ---- frames
    def _get_frame(fid):
        fr = dkv.get(fid)
        if not isinstance(fr, H2OFrame):
            raise KeyError(f"Object '{fid}' not found for argument: key")
        return fr

    @app.get("/3/Frames")
    def frames():
        out = []
        for k, v in dkv.items():
            if isinstance(v, H2OFrame):
                out.append({"__meta": v3.meta("FrameBaseV3", "Frame"), "frame_id": v3.frame_key(k), "rows": v.nrows,
                            "columns": v.ncols, "num_columns": v.ncols, "byte_size": 0, "is_text": False})
        return v3.frames(out)

    @app.get("/3/Frames/{fid}")
    def frame(fid: str, row_offset: int = 0, row_count: int = 10, column_offset: int = 0, column_count: int = -1,
              full_column_count: int = -1):
        fr = _get_frame(fid)
        return v3.frames([v3.frame(fr, row_offset, row_count, column_offset, column_count)])

    @app.get("/3/Frames/{fid}/light")
    def frame_light(fid: str, row_offset: int = 0, row_count: int = 10, column_offset: int = 0, column_count: int = -1):
        fr = _get_frame(fid)
        return v3.frames([v3.frame(fr, row_offset, row_count, column_offset, column_count, full=False)])

    @app.get("/3/Frames/{fid}/summary")
    def frame_summary(fid: str, row_offset: int = 0, row_count: int = 10):
        return v3.frames([v3.frame(_get_frame(fid), row_offset, row_count)])

    @app.get("/3/Frames/{fid}/columns")
    def frame_columns(fid: str):
        fr = _get_frame(fid)
        return v3.frames([v3.frame(fr, 0, 0, full=False)])

    @app.get("/3/Frames/{fid}/columns/{col}")
    @app.get("/3/Frames/{fid}/columns/{col}/summary")
    def frame_column(fid: str, col: str, row_offset: int = 0, row_count: int = 10):
        fr = _get_frame(fid)
        fj = v3.frame(fr, row_offset, row_count, full=True)
        fj["columns"] = [c for c in fj["columns"] if c["label"] == col]
        if not fj["columns"]:
            raise KeyError(f"column {col} not found")
        return v3.frames([fj])

    @app.get("/3/Frames/{fid}/columns/{col}/domain")
    def frame_column_domain(fid: str, col: str):
        fr = _get_frame(fid)
        c = fr._col(col)
        return v3.frames([]) | {"domain": [list(c.domain) if c.type == "enum" else None]}

    @app.delete("/3/Frames/{fid}")
    def frame_del(fid: str):
        dkv.remove(fid)
        return v3.frames([]) | {"frame_id": v3.frame_key(fid)}

    @app.delete("/3/Frames")
    def frames_del_all():
        for k, v in list(dkv.items()):
            if isinstance(v, H2OFrame):
                dkv.remove(k)
        return v3.frames([])

    @app.get("/3/DownloadDataset")
    @app.get("/3/DownloadDataset.bin")
    def download_dataset(frame_id: str, hex_string: bool = False):
        from fastapi.responses import Response
        fr = _get_frame(frame_id)
        return Response(content=fr.get_frame_data(), media_type="text/csv",
                        headers={"Content-Disposition": f'attachment; filename="{frame_id}.csv"'})

    @app.post("/3/Frames/{fid}/export")
    async def frame_export(fid: str, request: Request):
        from ..io import parse as P
        p = await _params(request)
        P.export_file(dkv.get(fid), p["path"], bool(p.get("force", False)))
        return dict(job=dict(status="DONE"), path=p["path"])

    @app.post("/3/SplitFrame")
    async def split_frame(request: Request):
        p = await _params(request)
        fr = dkv.get(p["dataset"])
        ratios = p.get("ratios") or [0.75]
        ratios = ratios if isinstance(ratios, list) else [ratios]
        dests = p.get("destination_frames")
        parts = fr.split_frame([float(r) for r in ratios[:-1] if float(r) < 1] or [float(ratios[0])], dests,
                               p.get("seed", None))
        return dict(destination_frames=[dict(name=x.frame_id) for x in parts])

    @app.post("/3/CreateFrame")
    async def create_frame(request: Request):
        from ..frame_ops import create_frame as cf
        p = await _params(request)
        dest = p.pop("dest", None)
        fr = cf(**{k: v for k, v in p.items() if k in cf.__code__.co_varnames}, frame_id=dest)
        return dict(key=dict(name=fr.frame_id), job=dict(status="DONE"))

    @app.post("/99/Rapids")
    async def rapids_ep(request: Request):
        from ..rapids import rapids
        p = await _params(request)
        ast = p["ast"]
        r = rapids(ast if isinstance(ast, str) else json.dumps(ast))
        base = {"__meta": v3.meta("RapidsSchemaV3", "Iced"), "ast": ast, "session_id": p.get("session_id")}
        if isinstance(r, H2OFrame):
            return base | {"__meta": v3.meta("RapidsFrameV3", "Iced"), "key": v3.frame_key(r.frame_id),
                           "num_rows": r.nrows, "num_cols": r.ncols}
        if isinstance(r, (list, tuple)):
            if all(isinstance(x, str) for x in r):
                return base | {"__meta": v3.meta("RapidsStringsV3", "Iced"), "string": list(r)}
            return base | {"__meta": v3.meta("RapidsNumbersV3", "Iced"),
                           "scalar": [None if x is None or (isinstance(x, float) and math.isnan(x)) else float(x)
                                      for x in r]}
        if isinstance(r, str):
            return base | {"__meta": v3.meta("RapidsStringV3", "Iced"), "string": r}
        return base | {"__meta": v3.meta("RapidsNumberV3", "Iced"), "scalar": _clean(r)}

    # ---- model builders
    @app.get("/3/ModelBuilders")
    def model_builders():
        return dict(model_builders={a: dict(algo=a, supervised=s.supervised, parameters=[
            dict(name=k, default_value=_clean(v)) for k, v in s.defaults.items()]) for a, s in builder.REGISTRY.items()})

    @app.get("/3/ModelBuilders/{algo}")
    def model_builder(algo: str):
        s = builder.REGISTRY[algo]
        from ..models.params import schema
        sch = schema(algo) or {}
        params = [{"__meta": v3.meta("ModelParameterSchemaV3", "Iced"), "name": k, "label": k, "help": k,
                   "required": k == "training_frame", "type": v3._param_type(v), "default_value": v3._json_value(v),
                   "actual_value": v3._json_value(v), "level": "critical", "values": [], "gridable": False,
                   "is_member_of_frames": [], "is_mutually_exclusive_with": []} for k, v in sch.items()]
        return {"__meta": v3.meta("ModelBuildersV3", "Iced"),
                "model_builders": {algo: {"__meta": v3.meta("ModelBuilderV3", "ModelBuilder"), "algo": algo,
                                          "algo_full_name": v3._FULL.get(algo, algo), "can_build": ["Binomial",
                                                                                                    "Multinomial",
                                                                                                    "Regression"],
                                          "supervised": s.supervised, "parameters": params, "visibility": "Stable"}}}

    _RESERVED = ("training_frame", "validation_frame", "response_column", "model_id")

    def _builder_args(algo, p):
        fr = dkv.get(_unquote(p.pop("training_frame", None)))
        if fr is None:
            raise ValueError("training_frame is required")
        vf = _unquote(p.pop("validation_frame", None))
        vf = dkv.get(vf) if vf else None
        y = _unquote(p.pop("response_column", None))
        mid = _unquote(p.pop("model_id", None)) or builder.make_key(algo)
        ig = p.pop("ignored_columns", None)
        ig = [_unquote(c) for c in (ig if isinstance(ig, list) else ([ig] if ig else []))]
        special = {p.get("weights_column"), p.get("offset_column"), p.get("fold_column"), y}
        x = [n for n in fr.names if n not in ig and n not in special] if ig else None
        for k in ("weights_column", "offset_column", "fold_column"):
            if k in p:
                p[k] = _unquote(p[k])
        if isinstance(p.get("lambda"), list):
            p["lambda_"] = p.pop("lambda")
        elif "lambda" in p:
            p["lambda_"] = p.pop("lambda")
        return fr, vf, y, mid, x

    @app.post("/3/ModelBuilders/{algo}")
    async def build(algo: str, request: Request):
        p = await _params(request)
        fr, vf, y, mid, x = _builder_args(algo, p)
        builder._validate(builder.REGISTRY[algo], algo, p)       # ModelBuilder.init errors before the job starts
        job = Job(f"{algo} build", dest=mid)
        job.run_async(builder.train, algo, p, x, y, fr, vf, job, mid)
        return {"__meta": v3.meta("ModelBuilderV3", "ModelBuilder"), "job": v3.job(job), "messages": [],
                "error_count": 0, "algo": algo, "parameters": [], "__http_response": {}}

    @app.post("/3/ModelBuilders/{algo}/parameters")
    async def validate(algo: str, request: Request):
        p = await _params(request)
        unknown = [k for k in p if builder.REGISTRY[algo].defaults and k not in builder.REGISTRY[algo].defaults
                   and k not in builder.COMMON and k != "response_column"]
        return dict(messages=[dict(message_type="WARN", field_name=k, message="unknown parameter") for k in unknown],
                    error_count=0)

    # ---- jobs
    @app.get("/3/Jobs")
    def jobs():
        return {"__meta": v3.meta("JobsV3", "Iced"), "job_id": None, "jobs": [v3.job(j) for j in list_jobs()]}

    @app.get("/3/Jobs/{key}")
    def job(key: str):
        j = dkv.get(key)
        if not isinstance(j, Job):
            raise KeyError(f"job {key} not found")
        return {"__meta": v3.meta("JobsV3", "Iced"), "job_id": v3.key(key, "Key<Job>"), "jobs": [v3.job(j)]}

    @app.post("/3/Jobs/{key}/cancel")
    def cancel(key: str):
        dkv.get(key).cancel()
        return dict(key=key)

    # ---- models
    def _get_model(mid):
        m = dkv.get(mid)
        if not isinstance(m, Model):
            raise KeyError(f"Object '{mid}' not found for argument: key")
        return m

    @app.get("/3/Models")
    def models():
        return {"__meta": v3.meta("ModelsV3", "Models"), "model_id": None, "preview": False,
                "find_compatible_frames": False, "models": [_model_json(v) for k, v in dkv.items() if isinstance(v, Model)]}

    @app.get("/3/Models/{mid}")
    def model(mid: str):
        return {"__meta": v3.meta("ModelsV3", "Models"), "model_id": v3.model_key(mid), "preview": False,
                "find_compatible_frames": False, "models": [_model_json(_get_model(mid))]}

    @app.delete("/3/Models/{mid}")
    def model_del(mid: str):
        dkv.remove(mid)
        return {"__meta": v3.meta("ModelsV3", "Models"), "model_id": v3.model_key(mid), "models": []}

    @app.delete("/3/Models")
    def models_del_all():
        for k, v in list(dkv.items()):
            if isinstance(v, Model):
                dkv.remove(k)
        return {"__meta": v3.meta("ModelsV3", "Models"), "models": []}

    @app.get("/3/Models.java/{mid}")
    @app.get("/3/Models.java/{mid}/preview")
    def model_pojo(mid: str):
        from fastapi.responses import Response
        from ..mojo.pojo import pojo_source
        m = _get_model(mid)
        return Response(content=pojo_source(m), media_type="text/plain",
                        headers={"Content-Disposition": f'attachment; filename="{mid}.java"'})

    @app.get("/3/Models/{mid}/mojo")
    def mojo(mid: str):
        import tempfile
        from ..mojo.writer import write_mojo
        from . import cloud
        m = _get_model(mid)
        path = cloud.shared_path(f"{mid}.zip") if cloud.in_task() else os.path.join(tempfile.gettempdir(), f"{mid}.zip")
        cloud.rank0_write(lambda: write_mojo(m, path))
        if cloud.in_task() and cloud.rank() != 0:
            from fastapi.responses import Response
            return Response(b"")
        return FileResponse(path, filename=f"{mid}.zip", headers={"Content-Disposition": f'attachment; filename="{mid}.zip"'})

    @app.get("/99/Models.bin/{mid}")
    def save_bin(mid: str, dir: str = "/tmp", force: bool = True):
        from ..persist import save_model
        return dict(dir=save_model(dkv.get(mid), dir, force))

    @app.post("/99/Models.bin/")
    async def load_bin(request: Request):
        from ..persist import load_model
        p = await _params(request)
        m = load_model(p["dir"])
        return dict(models=[_model_json(m)])

    @app.post("/99/Models.mojo/")
    async def upload_mojo(request: Request):
        from ..mojo.reader import import_mojo
        p = await _params(request)
        m = import_mojo(p["dir"], p.get("model_id"))
        return dict(models=[_model_json(m)])

    # ---- predictions & metrics
    @app.post("/3/Predictions/models/{mid}/frames/{fid}")
    async def predict(mid: str, fid: str, request: Request):
        p = await _params(request)
        m, fr = _get_model(mid), _get_frame(fid)
        pred = m.predict(fr)
        dest = _unquote(p.get("predictions_frame"))
        if dest:
            dkv.remove(pred.frame_id)
            pred.frame_id = dest
            dkv.put(dest, pred)
        mm = None
        if m.info.response and m.info.response in fr.names:
            try:
                mm = v3.metrics(m.model_performance(fr), m.model_category, mid, fid, m.algo)
            except Exception:  # noqa: BLE001 - predictions without a usable response column
                mm = None
        return {"__meta": v3.meta("ModelMetricsListSchemaV3", "ModelMetricsList"), "model": v3.model_key(mid),
                "frame": v3.frame_key(fid), "predictions_frame": v3.frame_key(pred.frame_id),
                "model_metrics": [mm] if mm else [], "deviances_frame": None, "reconstruction_error": False,
                "leaf_node_assignment": False, "exemplar_index": -1, "deep_features_hidden_layer": -1}

    @app.post("/4/Predictions/models/{mid}/frames/{fid}")
    async def predict4(mid: str, fid: str, request: Request):
        p = await _params(request)
        m, fr = _get_model(mid), _get_frame(fid)
        dest = _unquote(p.get("predictions_frame")) or f"prediction_{mid}_on_{fid}"
        job = Job("Predictions", dest=dest)

        def run():
            pred = m.predict(fr)
            dkv.remove(pred.frame_id)
            pred.frame_id = dest
            dkv.put(dest, pred)
            return pred
        job.run_async(run)
        return {"__meta": v3.meta("JobV4", "Job", 4), "job": v3.job(job), "key": v3.key(job.key, "Key<Job>"),
                "status": "RUNNING", "dest": v3.frame_key(dest)}

    @app.post("/3/ModelMetrics/models/{mid}/frames/{fid}")
    def metrics(mid: str, fid: str):
        m, fr = _get_model(mid), _get_frame(fid)
        mm = m.model_performance(fr)
        return {"__meta": v3.meta("ModelMetricsListSchemaV3", "ModelMetricsList"), "model": v3.model_key(mid),
                "frame": v3.frame_key(fid), "model_metrics": [v3.metrics(mm, m.model_category, mid, fid, m.algo)]}

    @app.get("/3/ModelMetrics")
    @app.get("/3/ModelMetrics/models/{mid}")
    @app.get("/3/ModelMetrics/models/{mid}/frames/{fid}")
    @app.get("/3/ModelMetrics/frames/{fid}")
    @app.get("/3/ModelMetrics/frames/{fid}/models/{mid}")
    def metrics_list(mid: str | None = None, fid: str | None = None):
        out = []
        for k, v in dkv.items():
            if isinstance(v, Model) and (mid is None or k == mid):
                for which in ("training_metrics", "validation_metrics"):
                    mm = v.output.get(which)
                    fk = v.output.get("training_frame" if which == "training_metrics" else "validation_frame")
                    if mm is not None and (fid is None or fk == fid):
                        out.append(v3.metrics(mm, v.model_category, k, fk, v.algo))
        return {"__meta": v3.meta("ModelMetricsListSchemaV3", "ModelMetricsList"), "model_metrics": out}

    # ---- grid & automl
    @app.post("/99/Grid/{algo}")
    async def grid(algo: str, request: Request):
        from ..grid import grid_search
        p = await _params(request)
        hyper = p.pop("hyper_parameters")
        crit = p.pop("search_criteria", None)
        gid = p.pop("grid_id", None) or dkv.new_key(f"Grid_{algo}")
        fr = dkv.get(p.pop("training_frame"))
        vf = p.pop("validation_frame", None)
        y = p.pop("response_column", None)
        rdir = p.pop("recovery_dir", None)
        y = _unquote(y)
        ig = p.pop("ignored_columns", None)
        ig = [_unquote(c) for c in (ig if isinstance(ig, list) else ([ig] if ig else []))]
        x = [n for n in fr.names if n not in ig and n != y] if ig else None
        p.pop("parallelism", None)
        job = Job(f"grid {algo}", dest=gid)
        job.run_async(grid_search, algo, hyper, p, x, y, fr, dkv.get(_unquote(vf)) if vf else None, gid, crit, 1, job, rdir)
        return {"__meta": v3.meta("GridSearchSchemaV99", "GridSearch", 99), "job": v3.job(job),
                "grid_id": v3.key(gid, "Key<Grid>"), "hyper_parameters": hyper, "search_criteria": crit}

    @app.post("/3/Recovery/resume")
    async def recovery_resume(request: Request):
        """hex/faulttolerance/Recovery.java: continue an interrupted grid from its recovery_dir."""
        from ..grid import resume
        p = await _params(request)
        job = Job("recovery resume", dest=None)
        job.run_async(resume, p["recovery_dir"])
        return dict(job=_clean(job.to_dict()), recovery_dir=p["recovery_dir"])

    @app.get("/99/Grids/{gid}")
    def get_grid(gid: str, sort_by: str | None = None, decreasing: bool | None = None):
        g = dkv.get(gid)
        if g is None:
            raise KeyError(f"grid {gid} not found")
        rows, key = g.sorted_models(sort_by, decreasing)
        hn = list(g.hyper_params)
        table = v3.twodim("Hyper-Parameter Search Summary", [(h, "string", "%s") for h in hn] +
                          [("model_ids", "string", "%s"), (key, "double", "%.5f")],
                          [[str(x) for x in h] + [m.key, v] for m, h, v in rows],
                          f"ordered by {'decreasing' if decreasing else 'increasing'} {key}")
        fails = g.failures or []
        return {"__meta": v3.meta("GridSchemaV99", "Grid", 99), "grid_id": v3.key(gid, "Key<Grid>"),
                "model_ids": [v3.model_key(m.key) for m, _, _ in rows], "hyper_names": hn,
                "failed_params": [f.get("params") if isinstance(f, dict) else f for f in fails],
                "failure_details": [str(f.get("error") if isinstance(f, dict) else f) for f in fails],
                "failure_stack_traces": [str(f.get("error") if isinstance(f, dict) else f) for f in fails],
                "failed_raw_params": [], "warning_details": [], "summary_table": table, "scoring_history": None,
                "cross_validation_metrics_summary": None, "training_metrics": [], "validation_metrics": [],
                "cross_validation_metrics": [], "export_checkpoints_dir": None, "sort_by": sort_by or key,
                "decreasing": bool(decreasing)}

    @app.get("/99/Models/{mid}")
    def model99(mid: str):
        return {"__meta": v3.meta("ModelsV99", "Models", 99), "model_id": v3.model_key(mid),
                "models": [_model_json(_get_model(mid))]}

    @app.post("/3/PostFile")
    @app.post("/3/PostFile.bin")
    async def post_file(request: Request, destination_frame: str | None = None):
        """Client uploads (multipart/form-data or raw body) land in a server-side temp file whose path
        is the raw key the following ParseSetup/Parse use (h2o-py H2OFrame(python_obj), upload_file)."""
        import tempfile
        body = await request.body()
        ct = request.headers.get("content-type", "")
        data, fname = body, "upload"
        if "multipart/form-data" in ct and "boundary=" in ct:
            data, fname = _multipart_first_file(body, ct.split("boundary=", 1)[1].strip().strip('"'))
        ext = os.path.splitext(fname)[1] or ".csv"
        from . import cloud
        if cloud.in_task():          # REST cloud: one copy, written by rank 0, at a path every rank derives
            path = cloud.shared_path(f"upload{ext}")

            def write():
                with open(path + ".part", "wb") as f:
                    f.write(data)
                os.replace(path + ".part", path)
            cloud.rank0_write(write)
        else:
            fd, path = tempfile.mkstemp(prefix="h2o_upload_", suffix=ext)
            with os.fdopen(fd, "wb") as f:
                f.write(data)
        return {"__meta": v3.meta("PostFileV3", "Iced"), "destination_frame": path, "total_bytes": len(data)}

    @app.post("/99/AutoMLBuilder")
    async def automl_build(request: Request):
        from ..automl import AutoML
        p = await _params(request)
        spec = p.get("input_spec", p)
        bs = p.get("build_control", {}) or {}
        bm = p.get("build_models", {}) or {}
        sc = bs.get("stopping_criteria", {}) if isinstance(bs, dict) else {}

        def name_of(v):
            return v.get("name") if isinstance(v, dict) else _unquote(v)
        inc = bm.get("include_algos")
        exc = bm.get("exclude_algos")
        mono = None
        for ap in bm.get("algo_parameters") or []:       # AutoMLCustomParameters: [{scope, name, value}]
            if isinstance(ap, dict) and ap.get("name") == "monotone_constraints":
                v = ap.get("value")
                mono = {d["key"]: d["value"] for d in v} if isinstance(v, list) else v
        aml = AutoML(project_name=bs.get("project_name"), max_models=sc.get("max_models"),
                     max_runtime_secs=sc.get("max_runtime_secs") or None,
                     max_runtime_secs_per_model=sc.get("max_runtime_secs_per_model") or 0, nfolds=bs.get("nfolds", 5),
                     seed=sc.get("seed"), include_algos=inc, exclude_algos=exc,
                     sort_metric=spec.get("sort_metric") or "AUTO",
                     stopping_metric=sc.get("stopping_metric") or "AUTO", stopping_rounds=sc.get("stopping_rounds", 3),
                     stopping_tolerance=sc.get("stopping_tolerance"),
                     balance_classes=bool(bs.get("balance_classes", False)),
                     class_sampling_factors=bs.get("class_sampling_factors"),
                     max_after_balance_size=bs.get("max_after_balance_size", 5.0),
                     keep_cross_validation_predictions=bool(bs.get("keep_cross_validation_predictions", False)),
                     keep_cross_validation_models=bool(bs.get("keep_cross_validation_models", False)),
                     keep_cross_validation_fold_assignment=bool(bs.get("keep_cross_validation_fold_assignment", False)),
                     export_checkpoints_dir=bs.get("export_checkpoints_dir"),
                     exploitation_ratio=bm.get("exploitation_ratio", -1), modeling_plan=bm.get("modeling_plan"),
                     preprocessing=bm.get("preprocessing"), monotone_constraints=mono)
        fr = dkv.get(name_of(spec["training_frame"]))
        y = name_of(spec.get("response_column"))
        ig = spec.get("ignored_columns") or []
        x = [n for n in fr.names if n not in ig and n != y] if ig else None
        vf = dkv.get(name_of(spec["validation_frame"])) if spec.get("validation_frame") else None
        lb = dkv.get(name_of(spec["leaderboard_frame"])) if spec.get("leaderboard_frame") else None
        bf = dkv.get(name_of(spec["blending_frame"])) if spec.get("blending_frame") else None
        job = Job("AutoML", dest=aml.project_name)
        job.run_async(aml.train, x, y, fr, vf, lb, bf, spec.get("fold_column"), spec.get("weights_column"), job)
        return {"__meta": v3.meta("AutoMLBuilderV99", "AutoMLBuilder", 99), "job": v3.job(job),
                "build_control": {"project_name": aml.project_name}, "automl_id": v3.key(aml.project_name, "Key<AutoML>")}

    def _leaderboard_table(aml):
        rows, cols = aml.leaderboard_rows()
        return rows, v3.twodim("Leaderboard", [("model_id", "string", "%s")] + [(c, "double", "%.6f") for c in cols[1:]],
                               [[r["model_id"]] + [r[c] for c in cols[1:]] for r in rows],
                               f"models sorted by {cols[1] if len(cols) > 1 else ''}",
                               row_headers=[str(i) for i in range(len(rows))])

    def _automl(pid):
        """An AutoML by project name, or by H2O's AutoML key ``<project>@@<response>`` (AutoML.java key naming,
        what Flow's getLeaderboard cells name)."""
        aml = dkv.get(pid)
        if aml is None and "@@" in pid:
            aml = dkv.get(pid.split("@@", 1)[0])
        return aml

    @app.get("/99/AutoML/{pid}")
    def automl_get(pid: str):
        aml = _automl(pid)
        if aml is None:
            raise KeyError(f"AutoML {pid} not found")
        rows, table = _leaderboard_table(aml)
        ev = v3.twodim("Event Log", [("timestamp", "string", "%s"), ("level", "string", "%s"), ("stage", "string", "%s"),
                                     ("message", "string", "%s"), ("name", "string", "%s"), ("value", "string", "%s")],
                       [[time.strftime("%H:%M:%S", time.localtime(e["timestamp"])), "Info", "ModelTraining",
                         e["message"], "", ""] for e in aml.event_log],
                       row_headers=[str(i) for i in range(len(aml.event_log))])
        return {"__meta": v3.meta("AutoMLV99", "AutoML", 99), "automl_id": v3.key(pid, "Key<AutoML>"),
                "project_name": pid, "leaderboard": {"__meta": v3.meta("LeaderboardV99", "Leaderboard", 99),
                                                     "project_name": pid,
                                                     "models": [v3.model_key(r["model_id"]) for r in rows]},
                "leaderboard_table": table, "event_log": {"events": aml.event_log}, "event_log_table": ev,
                "modeling_steps": [], "leader": v3.model_key(rows[0]["model_id"]) if rows else None}

    from .routes_more import register as _register_more
    _register_more(app, _params, _unquote, _model_json)
    from .routes_v4 import register as _register_v4
    _register_v4(app, _params)

    @app.get("/99/Leaderboards/{pid}")
    def leaderboard_get(pid: str):
        aml = _automl(pid)
        if aml is None:
            raise KeyError(f"AutoML {pid} not found")
        rows, table = _leaderboard_table(aml)
        return {"__meta": v3.meta("LeaderboardV99", "Leaderboard", 99), "project_name": pid,
                "models": [v3.model_key(r["model_id"]) for r in rows], "table": table}

    # ---- Flow web UI (h2o-web): the notebook page and its command layer (api/flow/)
    flow_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "flow")

    @app.get("/")
    def root():
        from fastapi.responses import RedirectResponse
        return RedirectResponse("/flow/index.html")

    @app.get("/flow/{name}")
    def flow_file(name: str):
        path = os.path.join(flow_dir, os.path.basename(name))
        if not os.path.isfile(path):
            raise KeyError(f"no Flow file {name}")
        media = "text/html" if name.endswith(".html") else "application/javascript"
        return FileResponse(path, media_type=media)

    # multi-rank cloud: rank 0 routes every cloud request through the executor (inside the login gate)
    from . import cloud
    cloud.install(app)
    if login is not None:
        from . import security
        security.install(app, login.validate())
    return app


def main(argv=None):
    import argparse
    import uvicorn
    from .security import LoginConfig
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", "-port", type=int, default=54321)
    ap.add_argument("--ip", "-ip", default="127.0.0.1")
    # H2O.java login options (single dash accepted as in `java -jar h2o.jar -hash_login -login_conf realm.properties`)
    for flag in ("hash_login", "ldap_login", "kerberos_login", "spnego_login", "pam_login", "form_auth"):
        ap.add_argument(f"--{flag}", f"-{flag}", action="store_true")
    ap.add_argument("--login_conf", "-login_conf", default=None)
    ap.add_argument("--spnego_properties", "-spnego_properties", default=None)
    ap.add_argument("--session_timeout", "-session_timeout", type=int, default=0)
    # HTTPS from a Java KeyStore (H2O.java -jks / -jks_pass / -jks_alias / -hostname_as_jks_alias; api/tls.py)
    ap.add_argument("--jks", "-jks", default=None)
    ap.add_argument("--jks_pass", "-jks_pass", default=None)
    ap.add_argument("--jks_alias", "-jks_alias", default=None)
    ap.add_argument("--hostname_as_jks_alias", "-hostname_as_jks_alias", action="store_true")
    a = ap.parse_args(argv)
    login = LoginConfig(hash_login=a.hash_login, ldap_login=a.ldap_login, kerberos_login=a.kerberos_login,
                        spnego_login=a.spnego_login, pam_login=a.pam_login, login_conf=a.login_conf,
                        form_auth=a.form_auth, session_timeout=a.session_timeout,
                        spnego_properties=a.spnego_properties)
    try:
        login.validate()
    except ValueError as e:
        ap.error(str(e))
    ssl_kw = {}
    if a.jks:
        from .tls import pem_files
        try:
            cf, kf = pem_files(a.jks, a.jks_pass, a.jks_alias, a.hostname_as_jks_alias)
        except (OSError, ValueError) as e:
            ap.error(f"-jks {a.jks}: {e}")
        ssl_kw = dict(ssl_certfile=cf, ssl_keyfile=kf)
        login.secure_cookies = True
    app = create_app(login=login)
    from . import cloud
    from ..parallel import collectives as coll
    if coll.world_active():
        # the SPMD cloud: every rank builds the same app; rank 0 serves HTTP, the others execute its requests
        ex = cloud.CloudExecutor(app)
        if ex.rank != 0:
            ex.loop()
            runtime.shutdown()
            return
        ex.start()
        try:
            _serve(app, a.ip, a.port, ssl_kw)
        finally:
            ex.stop()
            runtime.shutdown()
        return
    _serve(app, a.ip, a.port, ssl_kw)


def uvicorn_config(app, host, port, ssl_kw):
    """uvicorn config with the TLS context built up front: the unsealed private key's PEM file (``-jks``) is deleted
    as soon as the SSL context holds it, so it never outlives startup on disk."""
    import shutil
    import uvicorn
    cfg = uvicorn.Config(app, host=host, port=port, log_level="warning", **ssl_kw)
    if ssl_kw:
        try:
            cfg.load()
        finally:
            shutil.rmtree(os.path.dirname(ssl_kw["ssl_keyfile"]), ignore_errors=True)
    return cfg


def _serve(app, host, port, ssl_kw):
    import uvicorn
    uvicorn.Server(uvicorn_config(app, host, port, ssl_kw)).run()


if __name__ == "__main__":
    main()
