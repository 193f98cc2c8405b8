"""The rest of the top-level ``h2o-py`` module functions (reference: ``h2o-py/h2o/h2o.py``): REST passthrough,
cluster/network utilities, timezone and expression-optimisation switches, SQL import (SQLite through the
standard library; other JDBC URLs need a driver this image does not have), grid save/load, logs.
"""
from __future__ import annotations

import json
import os
import time

from llama_github_io_amd.core import dkv as _dkv

_STATE = dict(timezone="UTC", expr_optimizations=True)


def api(endpoint, data=None, json=None, filename=None, save_to=None):   # noqa: A002 - h2o-py signature
    """``h2o.api("GET /3/Cloud")``: sent to the connected server (``h2o.connect(url=...)``) over HTTP,
    or served in-process by this process's REST application (one cached client)."""
    from . import _conn
    c = _conn.current() or _conn.in_process()
    return c.request(endpoint, data=data, json=json, filename=filename, save_to=save_to)


def cluster_info():
    from llama_github_io_amd.core import runtime
    st = runtime.cluster_status()
    print(st)
    return st


def connection():
    from . import _conn
    return _conn.current() or _conn.in_process()


def version_check():
    return True


def log_and_echo(message=""):
    from llama_github_io_amd.utils import log
    log.get().info(message)
    print(message)


def download_all_logs(dirname=".", filename=None):
    """Zip of the engine's recent log records and timeline events (``/3/Logs`` + ``/3/Timeline``)."""
    import zipfile
    from llama_github_io_amd.utils import log, timeline
    os.makedirs(dirname, exist_ok=True)
    path = os.path.join(dirname, filename or f"h2ologs_{time.strftime('%Y%m%d_%H%M%S')}.zip")
    with zipfile.ZipFile(path, "w") as z:
        z.writestr("h2o.log", "\n".join(str(r) for r in log.recent(10000)))
        z.writestr("timeline.json", _json_dumps(timeline.events(1 << 14)))
    return path


def _json_dumps(o):
    return json.dumps(o, default=str)


def download_csv(data, filename):
    import h2o
    return h2o.export_file(data, filename, force=True)


def enable_expr_optimizations(flag):
    _STATE["expr_optimizations"] = bool(flag)


def is_expr_optimizations_enabled():
    return _STATE["expr_optimizations"]


def get_timezone():
    return _STATE["timezone"]


def set_timezone(value):
    _STATE["timezone"] = str(value)


def list_timezones():
    import zoneinfo
    import h2o
    import pandas as pd
    return h2o.H2OFrame(pd.DataFrame({"Timezones": sorted(zoneinfo.available_timezones())}),
                        column_types={"Timezones": "string"})


def estimate_cluster_mem(ncols, nrows, num_cols=0, string_cols=0, cat_cols=0, time_cols=0, uuid_cols=0):
    """GB of device memory a frame of this shape needs here: fp32 numerics, int32 categorical codes, fp64
    times / UUID halves, ~40 B per host string, plus the 4x working-set factor of the reference estimate."""
    if num_cols + string_cols + cat_cols + time_cols + uuid_cols == 0:
        num_cols = ncols
    per_row = 4 * num_cols + 4 * cat_cols + 8 * time_cols + 16 * uuid_cols + 40 * string_cols
    return round(4 * per_row * nrows / 1e9, 3)


def frame(frame_id):
    """Frame metadata (the ``/3/Frames/{id}`` JSON the reference returns)."""
    fr = _dkv.get(frame_id)
    if fr is None:
        raise KeyError(frame_id)
    return dict(frames=[dict(frame_id=dict(name=frame_id), rows=fr.nrows, num_columns=fr.ncols,
                             columns=[dict(label=n, type=fr.type(n)) for n in fr.names])])


def models():
    from llama_github_io_amd.models.base import Model
    return [k for k, v in _dkv.items() if isinstance(v, Model)]


def lazy_import(path, pattern=None):
    """File keys a later parse would read (no parsing), like ``/3/ImportFiles``."""
    from llama_github_io_amd.io.parse import _expand
    import re
    files = _expand(path)
    if pattern:
        files = [f for f in files if re.search(pattern, os.path.basename(f))]
    return files


def parse(setup, id=None, first_line_is_header=0):   # noqa: A002 - h2o-py signature
    import h2o
    return h2o.parse_raw(setup, id, first_line_is_header)


def rapids(expr):
    from llama_github_io_amd import rapids as _r
    return _r.rapids(expr)


def network_test():
    """Collective bandwidth probe (``/3/NetworkTest``): all-reduce of growing buffers over the rank group."""
    import torch
    from llama_github_io_amd.parallel import collectives as coll
    dev = coll.comm_device() if coll.is_dist() else (torch.device("cuda") if torch.cuda.is_available()
                                                      else torch.device("cpu"))
    rows = []
    for nbytes in (1 << 10, 1 << 16, 1 << 20, 1 << 24):
        t = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
        coll.all_reduce_(t)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            coll.all_reduce_(t)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        rows.append(dict(bytes=nbytes, seconds=dt, gbps=nbytes / max(dt, 1e-12) / 1e9, ranks=coll.world()))
    return rows


# ---- SQL import (ImportSQLTable.java): sqlite through the standard library
def _sqlite_path(connection_url):
    for prefix in ("jdbc:sqlite:", "sqlite:///", "sqlite:"):
        if connection_url.startswith(prefix):
            return connection_url[len(prefix):]
    raise NotImplementedError(f"only SQLite connection URLs are supported here (got {connection_url!r}); "
                              "other databases need a JDBC/DB-API driver that this image does not ship")


def import_sql_select(connection_url, select_query, username=None, password=None, optimize=True,
                      use_temp_table=None, temp_table_name=None, fetch_mode=None, num_chunks_hint=None):
    import sqlite3
    import h2o
    import pandas as pd
    with sqlite3.connect(_sqlite_path(connection_url)) as con:
        df = pd.read_sql_query(select_query, con)
    return h2o.H2OFrame(df)


def import_sql_table(connection_url, table, username=None, password=None, columns=None, optimize=True,
                     fetch_mode=None, num_chunks_hint=None):
    cols = ", ".join(f'"{c}"' for c in columns) if columns else "*"
    return import_sql_select(connection_url, f'SELECT {cols} FROM "{table}"', username, password)


def import_hive_table(database=None, table=None, partitions=None, allow_multi_format=False):
    raise NotImplementedError("Hive import needs a Hadoop deployment (out of scope for the single-node engine)")


# ---- grids
def save_grid(grid_directory, grid_id, save_params_references=False, export_cross_validation_predictions=False):
    """Grid + every model to ``grid_directory`` (``/3/Grid.bin/{id}/export``)."""
    from llama_github_io_amd.persist import save_model
    g = grid_id if not isinstance(grid_id, str) else _dkv.get(grid_id)
    g = getattr(g, "_grid", g)
    os.makedirs(grid_directory, exist_ok=True)
    meta = dict(grid_id=g.grid_id, algo=g.algo, hyper_params=g.hyper_params, hyper_values=g.hyper_values,
                base_params={k: v for k, v in g.base_params.items() if _jsonable(v)}, failures=g.failures,
                models=[os.path.basename(save_model(m, os.path.join(grid_directory, "models"), force=True))
                        for m in g.models])
    path = os.path.join(grid_directory, g.grid_id + ".json")
    with open(path, "w") as f:
        json.dump(meta, f, default=str)
    return path


def load_grid(grid_file_path, load_params_references=False):
    from llama_github_io_amd.grid import Grid
    from llama_github_io_amd.persist import load_model
    with open(grid_file_path) as f:
        meta = json.load(f)
    g = Grid(meta["grid_id"], meta["algo"], meta["hyper_params"], meta["base_params"])
    base = os.path.join(os.path.dirname(grid_file_path), "models")
    for name, hv in zip(meta["models"], meta["hyper_values"]):
        m = load_model(os.path.join(base, name))
        _dkv.put(m.key, m)
        g.models.append(m)
        g.hyper_values.append(hv)
    g.failures = meta.get("failures", [])
    _dkv.put(g.grid_id, g)
    import inspect
    import h2o.estimators as E
    from h2o.grid import H2OGridSearch
    cls = next((c for _, c in inspect.getmembers(E, inspect.isclass)
                if getattr(c, "algo", None) == g.algo and "AutoEncoder" not in c.__name__), E.H2OEstimator)
    gs = H2OGridSearch(cls, g.hyper_params, g.grid_id)
    gs._grid = g
    return gs


def _jsonable(v):
    try:
        json.dumps(v)
        return True
    except TypeError:
        return False


def load_dataset(relative_path):
    """Datasets shipped with the client (``h2o_data/<name>.csv``): looked up next to this package and in
    ``$H2O_DATA_DIR``; no data is bundled in this build."""
    import h2o
    name = relative_path if relative_path.endswith(".csv") else relative_path + ".csv"
    for d in (os.environ.get("H2O_DATA_DIR"), os.path.join(os.path.dirname(__file__), "h2o_data")):
        if d and os.path.exists(os.path.join(d, name)):
            return h2o.import_file(os.path.join(d, name))
    raise FileNotFoundError(f"dataset {relative_path} not found (set H2O_DATA_DIR to a directory holding {name})")


def demo(funcname, interactive=True, echo=True, test=False):
    raise NotImplementedError("interactive demos are not shipped; see README.md for runnable examples")


import_frame = None   # bound in h2o/__init__ to import_file (deprecated alias in the reference)
