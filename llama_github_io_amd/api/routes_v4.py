"""REST API v4 (reference: ``h2o-core/src/main/java/water/api/RegisterV4Api.java:13-42``).

* ``GET /4/endpoints``         MetadataHandler.listRoutes4 -> EndpointsListV4 (every registered /4 route)
* ``POST /4/sessions``         (server.py) SessionIdV4;  ``DELETE /4/sessions/{session_key}`` ends it
* ``GET /4/modelsinfo``        ModelBuildersHandler.modelsInfo -> ModelsInfoV4 (algo, maturity, POJO / MOJO support)
* ``POST /4/Frames/$simple``   CreateFrameHandler.CreateSimpleFrame: SimpleCreateFrameRecipe run as a Job -> JobV4
* ``GET /4/jobs/{job_id}``     JobsHandler.FetchJob -> JobV4
"""
from __future__ import annotations

import numpy as np
from fastapi import Request

from ..core import dkv
from ..core.job import Job
from . import v3

# algorithms with a POJO writer here (mojo/pojo.py) and their MOJO format versions (the *MojoWriter.mojoVersion())
_POJO = {"gbm", "drf", "isolationforest", "glm", "kmeans", "deeplearning", "naivebayes", "pca", "svd", "xgboost"}
_MOJO_VERSION = {"gbm": "1.40", "drf": "1.40", "isolationforest": "1.40", "extendedisolationforest": "1.00",
                 "glm": "1.00", "kmeans": "1.00", "deeplearning": "1.10", "pca": "1.00", "word2vec": "1.00",
                 "isotonicregression": "1.00", "stackedensemble": "1.01", "coxph": "1.00", "targetencoder": "1.00",
                 "xgboost": "1.00", "glrm": "1.10", "rulefit": "1.00", "gam": "1.00", "upliftdrf": "1.40"}
_ALPHA = {"psvm", "modelselection", "anovaglm", "upliftdrf", "infogram", "hglm", "adaboost", "decisiontree"}
_BETA = {"extendedisolationforest", "gam", "rulefit", "aggregator", "coxph", "word2vec", "generic", "targetencoder",
         "isotonicregression", "grep"}


def _meta4(name: str) -> dict:
    return v3.meta(name, "Iced", 4)


def job_v4(j: Job) -> dict:
    """JobV4.fillFromImpl."""
    d = v3.job(j)
    st = d["status"]
    if st not in ("RUNNING", "DONE", "STOPPING", "CANCELLED", "FAILED"):
        st = "RUNNING" if st == "CREATED" else st
    dest = getattr(j, "dest", None)
    target_type = None
    if dest is not None:
        obj = dkv.get(dest)
        target_type = type(obj).__name__ if obj is not None else None
        if target_type == "H2OFrame":
            target_type = "Frame"
    return {"__meta": _meta4("JobV4"), "job_id": j.key, "status": st, "progress": d["progress"],
            "progress_msg": d["progress_msg"], "start_time": d["start_time"], "duration": d["msec"],
            "target_id": dest if st == "DONE" else None, "target_type": target_type,
            "exception": d["exception"], "stacktrace": d["stacktrace"] if d["exception"] else None}


def simple_create_frame(dest=None, seed=-1, nrows=100, ncols_real=0, ncols_int=0, ncols_enum=0, ncols_bool=0,
                        ncols_str=0, ncols_time=0, real_lb=-100.0, real_ub=100.0, int_lb=-100, int_ub=100,
                        enum_nlevels=10, bool_p=0.3, time_lb=365 * 24 * 3600 * 1000 * 30,
                        time_ub=365 * 24 * 3600 * 1000 * 50, str_length=8, missing_fraction=0.0,
                        response_type="none", response_lb=0.0, response_ub=10.0, response_p=0.6,
                        response_nlevels=25):
    """hex/createframe/recipes/SimpleCreateFrameRecipe: typed column makers (response, R*, I*, E*, B*, T*, S*), the
    MissingInserter post-process, then ShuffleColumnsCfps(reassignNames=true, responseFirst=true)."""
    from ..frame import H2OFrame
    chk = [(ncols_real >= 0, "Number of real columns cannot be negative"),
           (ncols_int >= 0, "Number of integer columns cannot be negative"),
           (ncols_bool >= 0, "Number of bool (binary) columns cannot be negative"),
           (ncols_enum >= 0, "Number of enum (categorical) columns cannot be negative"),
           (ncols_str >= 0, "Number of string columns cannot be negative"),
           (ncols_time >= 0, "Number of time columns cannot be negative"),
           (real_lb <= real_ub, "Invalid real range interval: lower bound exceeds the upper bound"),
           (int_lb <= int_ub, "Invalid integer range interval: lower bound exceeds the upper bound"),
           (0 <= bool_p <= 1, "Boolean frequency parameter must be in the range 0..1"),
           (time_lb <= time_ub, "Invalid time range interval: lower bound exceeds the upper bound"),
           (0 <= missing_fraction <= 1, "Missing fraction must be in the range 0..1"),
           (response_lb <= response_ub, "Invalid interval for response column: lower bound exceeds the upper bound"),
           (0 <= response_p <= 1, "Response binary frequency (response_p) should be in the range 0..1"),
           (response_nlevels >= 2, "Number of categorical levels for the response column must be 2 or more")]
    for ok, msg in chk:
        if not ok:
            raise ValueError(msg)
    rng = np.random.default_rng(None if int(seed) in (-1,) else int(seed) & ((1 << 63) - 1))
    n = int(nrows)
    cols: list[tuple[str, object]] = []

    def real(lb, ub):
        return rng.uniform(lb, ub, n)

    def integer(lb, ub):
        return rng.integers(int(lb), int(ub) + 1, n).astype(np.float64)

    def enum(k):
        return np.array([f"c{int(i)}" for i in rng.integers(0, int(k), n)], dtype=object)

    def boolean(p):
        return (rng.random(n) < p).astype(np.float64)

    def timec(lb, ub):
        return rng.integers(int(lb), int(ub) + 1, n).astype(np.float64)

    def string(m):
        al = np.array(list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789"))
        return np.array(["".join(al[rng.integers(0, len(al), int(m))]) for _ in range(n)], dtype=object)

    rt = str(response_type).lower()
    if rt == "real":
        cols.append(("response", real(response_lb, response_ub)))
    elif rt == "int":
        cols.append(("response", integer(response_lb, response_ub)))
    elif rt == "enum":
        cols.append(("response", enum(response_nlevels)))
    elif rt == "bool":
        cols.append(("response", boolean(response_p)))
    elif rt == "time":
        cols.append(("response", timec(response_lb, response_ub)))
    cols += [(f"R{i}", real(real_lb, real_ub)) for i in range(1, int(ncols_real) + 1)]
    cols += [(f"I{i}", integer(int_lb, int_ub)) for i in range(1, int(ncols_int) + 1)]
    cols += [(f"E{i}", enum(enum_nlevels)) for i in range(int(ncols_enum))]
    cols += [(f"B{i}", boolean(bool_p)) for i in range(1, int(ncols_bool) + 1)]
    cols += [(f"T{i}", timec(time_lb, time_ub)) for i in range(int(ncols_time))]
    cols += [(f"S{i}", string(str_length)) for i in range(int(ncols_str))]
    # MissingInserterCfps: each cell missing with probability missing_fraction
    if missing_fraction > 0:
        out = []
        for name, v in cols:
            m = rng.random(n) < missing_fraction
            if v.dtype == object:
                v = v.copy()
                v[m] = None
            else:
                v = np.where(m, np.nan, v)
            out.append((name, v))
        cols = out
    # ShuffleColumnsCfps(reassignNames, responseFirst)
    idx = list(rng.permutation(len(cols)))
    ri = next((i for i, (nm, _) in enumerate(cols) if nm == "response"), -1)
    if ri >= 0:
        si = idx.index(ri)
        idx[si], idx[0] = idx[0], ri
    cols = [cols[i] for i in idx]
    counts: dict[str, int] = {}
    named = []
    for nm, v in cols:
        pre = nm.rstrip("0123456789")
        counts[pre] = counts.get(pre, 0) + 1
        named.append((nm if nm == "response" else f"{pre}{counts[pre]}", v))
    import pandas as pd
    kinds = {"R": "real", "I": "int", "E": "enum", "B": "int", "T": "time", "S": "string"}
    rkind = {"real": "real", "int": "int", "enum": "enum", "bool": "int", "time": "time"}.get(rt, "real")
    types = {nm: (rkind if nm == "response" else kinds[nm[0]]) for nm, _ in named}
    df = pd.DataFrame({nm: v for nm, v in named})
    fr = H2OFrame(df, column_types=types) if named else H2OFrame(pd.DataFrame())
    key = dest or dkv.new_key("frame_simple")
    fr.frame_id = key
    dkv.put(key, fr)
    return fr


def register(app, _params):
    from ..models import builder

    @app.get("/4/endpoints")
    def endpoints4():
        eps = []
        for r in app.routes:
            path = getattr(r, "path", "")
            if not path.startswith("/4/"):
                continue
            for m in sorted(getattr(r, "methods", None) or {"GET"}):
                if m == "HEAD":
                    continue
                name = getattr(r, "name", "") or ""
                eps.append({"__meta": _meta4("EndpointV4"), "url": f"{m} {path.replace('{sid}', '{session_key}')}",
                            "description": (getattr(r, "endpoint", None).__doc__ or "").strip().split("\n")[0]
                            if getattr(r, "endpoint", None) else "",
                            "name": name, "input_schema": "/4/schemas/" + _IN.get(path, "InputSchemaV4"),
                            "output_schema": "/4/schemas/" + _OUT.get(path, "OutputSchemaV4")})
        return {"__meta": _meta4("EndpointsListV4"), "endpoints": eps}

    @app.get("/4/modelsinfo")
    def models_info():
        """Return basic information about all models available to train."""
        out = []
        for algo in sorted(builder.REGISTRY):
            out.append({"__meta": _meta4("ModelInfoV4"), "algo": algo,
                        "maturity": "alpha" if algo in _ALPHA else ("beta" if algo in _BETA else "stable"),
                        "have_pojo": algo in _POJO, "have_mojo": algo in _MOJO_VERSION,
                        "mojo_version": _MOJO_VERSION.get(algo)})
        return {"__meta": _meta4("ModelsInfoV4"), "models": out}

    @app.post("/4/Frames/$simple")
    async def create_simple_frame(request: Request):
        """Create a frame with random data from the simple recipe; runs as a Job."""
        p = await _params(request)
        dest = p.pop("dest", None)
        if isinstance(dest, dict):
            dest = dest.get("name")
        allowed = simple_create_frame.__code__.co_varnames[:simple_create_frame.__code__.co_argcount]
        kw = {k: v for k, v in p.items() if k in allowed}
        for k, v in list(kw.items()):
            if isinstance(v, str) and k != "response_type":
                try:
                    kw[k] = float(v) if any(c in v for c in ".eE") else int(v)
                except ValueError:
                    pass
        key = dest or dkv.new_key("frame_simple")
        job = Job("CreateFrame: simple recipe", dest=key)
        job.run_async(lambda: simple_create_frame(dest=key, **kw))
        return job_v4(job)

    @app.get("/4/jobs/{job_id}")
    def fetch_job(job_id: str):
        """Fetch a Job by its id."""
        j = dkv.get(job_id)
        if not isinstance(j, Job):
            raise KeyError(f"Job {job_id} not found")
        return job_v4(j)


_IN = {"/4/endpoints": "ListRequestV4", "/4/modelsinfo": "ListRequestV4", "/4/Frames/$simple": "CreateFrameSimpleIV4",
       "/4/jobs/{job_id}": "JobIV4", "/4/sessions": "InputSchemaV4", "/4/sessions/{sid}": "SessionIdV4"}
_OUT = {"/4/endpoints": "EndpointsListV4", "/4/modelsinfo": "ModelsInfoV4", "/4/Frames/$simple": "JobV4",
        "/4/jobs/{job_id}": "JobV4", "/4/sessions": "SessionIdV4", "/4/sessions/{sid}": "SessionIdV4"}
