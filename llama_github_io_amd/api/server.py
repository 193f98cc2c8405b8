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


def _frame_json(fr: H2OFrame, row_offset=0, row_count=10, full=False):
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
    out = dict(model_id=dict(name=m.key, type="Key<Model>"), algo=m.algo, algo_full_name=m.algo,
               response_column_name=m.info.response, parameters=[dict(name=k, actual_value=v) for k, v in m.params.items()],
               output=dict(m.output, model_category=m.model_category, names=m.info.x + ([m.info.response] if m.info.response else []),
                           domains=m.info.domains + ([m.info.response_domain] if m.info.response else [])))
    return _clean(out)


def _parse_params(raw: dict) -> dict:
    out = {}
    for k, v in raw.items():
        if isinstance(v, str):
            s = v.strip()
            if s.startswith("[") or s.startswith("{"):
                try:
                    v = json.loads(s.replace("'", '"'))
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


def create_app():
    if FastAPI is None:
        raise RuntimeError("fastapi is not installed")
    runtime.init()
    app = FastAPI(title="H2O (MI355X-native) REST API", version="3.46.0.amd0")

    @app.middleware("http")
    async def timeline(request, call_next):
        t0 = time.time()
        resp = await call_next(request)
        _timeline.append(dict(time=int(t0 * 1000), method=request.method, url=str(request.url.path),
                              duration_ms=int((time.time() - t0) * 1000), status=resp.status_code))
        del _timeline[:-1000]
        return resp

    @app.exception_handler(Exception)
    async def errors(request, exc):
        return JSONResponse(status_code=500 if not isinstance(exc, (ValueError, KeyError)) else 412,
                            content=dict(__meta=dict(schema_type="H2OError"), msg=str(exc), exception_type=type(exc).__name__,
                                         http_status=412))

    # ---- cloud
    @app.get("/3/Cloud")
    def cloud():
        return _clean(runtime.cluster_status())

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
        return dict(key=key)

    # ---- ingest
    @app.post("/3/ImportFiles")
    @app.get("/3/ImportFiles")
    async def import_files(request: Request):
        from ..io import parse as P
        p = await _params(request)
        path = p.get("path")
        files = P._expand(path)
        return dict(path=path, files=files, destination_frames=files, fails=[], dels=[])

    @app.post("/3/ParseSetup")
    async def parse_setup(request: Request):
        from ..io import parse as P
        p = await _params(request)
        src = p.get("source_frames")
        src = src if isinstance(src, list) else [src]
        return _clean(P.parse_setup(src[0], header=int(p.get("check_header", 0) or 0), separator=p.get("separator")))

    @app.post("/3/Parse")
    async def parse(request: Request):
        from ..io import parse as P
        p = await _params(request)
        src = p.get("source_frames")
        src = src if isinstance(src, list) else [src]
        dest = p.get("destination_frame")
        sep = p.get("separator")
        if isinstance(sep, int):
            sep = chr(sep)
        job = Job("Parse", dest=dest)
        job.run_async(P.import_file, src, dest, True, int(p.get("check_header", 0) or 0), sep,
                      p.get("column_names"), p.get("column_types"), p.get("na_strings"))
        return dict(job=job.to_dict(), destination_frame=dict(name=dest))

    # ---- frames
    @app.get("/3/Frames")
    def frames():
        return dict(frames=[dict(frame_id=dict(name=k), rows=v.nrows, columns=v.ncols) for k, v in dkv.items()
                            if isinstance(v, H2OFrame)])

    @app.get("/3/Frames/{fid}")
    def frame(fid: str, row_offset: int = 0, row_count: int = 10):
        fr = dkv.get(fid)
        if not isinstance(fr, H2OFrame):
            raise KeyError(f"frame {fid} not found")
        return _clean(dict(frames=[_frame_json(fr, row_offset, row_count)]))

    @app.get("/3/Frames/{fid}/summary")
    def frame_summary(fid: str):
        fr = dkv.get(fid)
        return _clean(dict(frames=[_frame_json(fr, 0, 10, full=True)]))

    @app.delete("/3/Frames/{fid}")
    def frame_del(fid: str):
        dkv.remove(fid)
        return dict(frame_id=fid)

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
        r = rapids(p["ast"])
        if isinstance(r, H2OFrame):
            return dict(key=dict(name=r.frame_id), num_rows=r.nrows, num_cols=r.ncols)
        if isinstance(r, (list, tuple)):
            return _clean(dict(scalar=None, vals=list(r)))
        if isinstance(r, str):
            return dict(string=r)
        return _clean(dict(scalar=r))

    # ---- model builders
    @app.get("/3/ModelBuilders")
    def model_builders():
        return dict(model_builders={a: dict(algo=a, supervised=s.supervised, parameters=[
            dict(name=k, default_value=_clean(v)) for k, v in s.defaults.items()]) for a, s in builder.REGISTRY.items()})

    @app.get("/3/ModelBuilders/{algo}")
    def model_builder(algo: str):
        s = builder.REGISTRY[algo]
        return dict(model_builders={algo: dict(algo=algo, supervised=s.supervised)})

    @app.post("/3/ModelBuilders/{algo}")
    async def build(algo: str, request: Request):
        p = await _params(request)
        fr = dkv.get(p.pop("training_frame"))
        vf = p.pop("validation_frame", None)
        vf = dkv.get(vf) if vf else None
        y = p.pop("response_column", None)
        ignored = p.get("ignored_columns")
        mid = p.pop("model_id", None) or builder.make_key(algo)
        x = None
        job = Job(f"{algo} build", dest=mid)
        job.run_async(builder.train, algo, p, x, y, fr, vf, job, mid)
        return dict(job=_clean(job.to_dict()), messages=[], error_count=0)

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
        return dict(jobs=[_clean(j.to_dict()) for j in list_jobs()])

    @app.get("/3/Jobs/{key}")
    def job(key: str):
        j = dkv.get(key)
        if not isinstance(j, Job):
            raise KeyError(f"job {key} not found")
        return dict(jobs=[_clean(j.to_dict())])

    @app.post("/3/Jobs/{key}/cancel")
    def cancel(key: str):
        dkv.get(key).cancel()
        return dict(key=key)

    # ---- models
    @app.get("/3/Models")
    def models():
        return dict(models=[_model_json(v) for k, v in dkv.items() if isinstance(v, Model)])

    @app.get("/3/Models/{mid}")
    def model(mid: str):
        m = dkv.get(mid)
        if not isinstance(m, Model):
            raise KeyError(f"model {mid} not found")
        return dict(models=[_model_json(m)])

    @app.delete("/3/Models/{mid}")
    def model_del(mid: str):
        dkv.remove(mid)
        return dict(model_id=mid)

    @app.get("/3/Models/{mid}/mojo")
    def mojo(mid: str):
        from ..mojo.writer import write_mojo
        path = os.path.join("/tmp", f"{mid}.zip")
        write_mojo(dkv.get(mid), path)
        return FileResponse(path, filename=f"{mid}.zip")

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
        m, fr = dkv.get(mid), dkv.get(fid)
        pred = m.predict(fr)
        dest = p.get("predictions_frame")
        if dest:
            dkv.remove(pred.frame_id)
            pred.frame_id = dest
            dkv.put(dest, pred)
        return dict(predictions_frame=dict(name=pred.frame_id), model_metrics=[])

    @app.post("/3/ModelMetrics/models/{mid}/frames/{fid}")
    def metrics(mid: str, fid: str):
        m, fr = dkv.get(mid), dkv.get(fid)
        mm = m.model_performance(fr)
        return _clean(dict(model_metrics=[dict(mm or {}, model=dict(name=mid), frame=dict(name=fid))]))

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
        job = Job(f"grid {algo}", dest=gid)
        job.run_async(grid_search, algo, hyper, p, None, y, fr, dkv.get(vf) if vf else None, gid, crit, 1, job, rdir)
        return dict(job=_clean(job.to_dict()), grid_id=dict(name=gid))

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
        rows, key = g.sorted_models(sort_by, decreasing)
        return _clean(dict(grid_id=dict(name=gid), model_ids=[dict(name=m.key) for m, _, _ in rows],
                           hyper_names=list(g.hyper_params), failed_params=g.failures,
                           summary_table=[dict(zip(g.hyper_params, h), model_id=m.key, **{key: v}) for m, h, v in rows]))

    @app.post("/99/AutoMLBuilder")
    async def automl_build(request: Request):
        from ..automl import AutoML
        p = await _params(request)
        spec = p.get("input_spec", p)
        bs = p.get("build_control", {})
        bm = p.get("build_models", {})
        sc = bs.get("stopping_criteria", {}) if isinstance(bs, dict) else {}
        aml = AutoML(project_name=bs.get("project_name"), max_models=sc.get("max_models"),
                     max_runtime_secs=sc.get("max_runtime_secs"), nfolds=bs.get("nfolds", 5), seed=sc.get("seed"),
                     include_algos=bm.get("include_algos"), exclude_algos=bm.get("exclude_algos"))
        fr = dkv.get(spec["training_frame"]) if isinstance(spec.get("training_frame"), str) else dkv.get(spec["training_frame"]["name"])
        job = Job("AutoML", dest=aml.project_name)
        job.run_async(aml.train, None, spec.get("response_column"), fr, None, None, None, None, None, job)
        return dict(job=_clean(job.to_dict()), automl_id=dict(name=aml.project_name))

    @app.get("/99/AutoML/{pid}")
    @app.get("/99/Leaderboards/{pid}")
    def automl_get(pid: str):
        aml = dkv.get(pid)
        rows, cols = aml.leaderboard_rows()
        return _clean(dict(project_name=pid, leaderboard_table=dict(columns=cols, data=rows),
                           leader=dict(name=rows[0]["model_id"]) if rows else None, event_log=aml.event_log))

    return app


def main():
    import argparse
    import uvicorn
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=54321)
    ap.add_argument("--ip", default="127.0.0.1")
    a = ap.parse_args()
    uvicorn.run(create_app(), host=a.ip, port=a.port, log_level="warning")


if __name__ == "__main__":
    main()
