"""H2O-compatible Python API backed by the MI355X-native engine (``llama_github_io_amd``).

Reference: ``h2o-py/h2o/h2o.py``. ``h2o.init()`` boots the in-process engine (no JVM, no REST hop):
frames live in HBM on this process's GPU, models train through the HIP kernels, and with torchrun
(``WORLD_SIZE>1``) every rank joins the RCCL process group and holds its row shard.
"""
from __future__ import annotations

__version__ = "3.46.0.amd0"

import os as _os
import sys as _sys

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from llama_github_io_amd.core import dkv as _dkv  # noqa: E402
from llama_github_io_amd.core import runtime as _rt  # noqa: E402
from llama_github_io_amd.frame import H2OFrame  # noqa: E402
from llama_github_io_amd import frame_ops as _fops  # noqa: E402
from llama_github_io_amd.io import parse as _parse  # noqa: E402

from . import estimators  # noqa: E402,F401

_progress = [True]


class _Cluster:
    def _status(self):
        from . import _conn
        if _conn.is_remote():
            return _conn.current().request("GET /3/Cloud")
        return _rt.cluster_status()

    def show_status(self, detailed=False):
        st = self._status()
        print(st)
        return st

    def status(self):
        return self._status()

    @property
    def cloud_name(self):
        return self._status()["cloud_name"]

    @property
    def cloud_size(self):
        return self._status()["cloud_size"]

    def shutdown(self, prompt=False):
        _rt.shutdown()

    def is_running(self):
        return _rt.is_running()

    @property
    def version(self):
        return __version__


_cluster = _Cluster()


def init(url=None, ip=None, port=None, name=None, nthreads=-1, max_mem_size=None, min_mem_size=None, strict_version_check=None,
         enable_assertions=True, verbose=True, **kwargs):
    """Start (or attach to) the in-process engine. Connection arguments are accepted for API
    compatibility; use ``h2o.connect(url=...)`` semantics via the REST server for remote use."""
    st = _rt.init(name=name)
    if verbose:
        dev = st["device"]
        print(f"H2O (MI355X-native) {__version__} cloud '{st['cloud_name']}' size {st['cloud_size']} on {dev}")
    return _cluster


def connect(server=None, url=None, ip=None, port=None, https=None, verify_ssl_certificates=None, auth=None,
            proxy=None, cookies=None, verbose=True, config=None, strict_version_check=False, **kw):
    """Attach to a running server (``url`` or ``ip``/``port``) over HTTP: ``h2o.api``, ``h2o.ls``,
    ``h2o.remove``, ``h2o.cluster()`` then talk to it. Without an address this is ``h2o.init()``."""
    from . import _conn
    if config:
        url = url or config.get("url")
        ip, port = ip or config.get("ip"), port or config.get("port")
    if server is not None and url is None:
        url = getattr(server, "url", None) or str(server)
    if url is None and ip is None and port is None:
        init(verbose=verbose)
        return _conn.set_current(_conn.InProcessConnection())
    if url is None:
        url = f"{'https' if https else 'http'}://{ip or '127.0.0.1'}:{port or 54321}"
    c = _conn.set_current(_conn.RemoteConnection(url, verify_ssl_certificates=verify_ssl_certificates is not False,
                                                 auth=auth))
    if verbose:
        cl = c.cloud
        print(f"Connected to {url}: cloud '{cl.get('cloud_name')}' size {cl.get('cloud_size')} version {cl.get('version')}")
    return c


def cluster():
    return _cluster


def shutdown(prompt=False):
    _rt.shutdown()


def no_progress():
    _progress[0] = False


def show_progress():
    _progress[0] = True


# ---- frames
def import_file(path=None, destination_frame=None, parse=True, header=0, sep=None, col_names=None, col_types=None,
                na_strings=None, pattern=None, skipped_columns=None, custom_non_data_line_markers=None,
                partition_by=None, quotechar=None, escapechar=None, decrypt_tool=None):
    return _parse.import_file(path, destination_frame, parse, header, sep, col_names, col_types, na_strings, pattern,
                              skipped_columns, custom_non_data_line_markers, partition_by, quotechar, escapechar,
                              decrypt_tool=decrypt_tool)


def decryption_setup(keystore, keystore_type="JCEKS", key_alias=None, password=None, decrypt_tool="",
                     decrypt_impl="water.parser.GenericDecryptionTool", cipher_spec=None):
    """R ``h2o.decryptionSetup`` / ``POST /3/DecryptionSetup``: install a Decryption Tool reading the secret key
    ``key_alias`` of a (JCEKS) keystore file; pass the returned key to ``import_file(decrypt_tool=...)``."""
    from llama_github_io_amd.io import decrypt as _dec
    for n, v in (("key_alias", key_alias), ("password", password), ("cipher_spec", cipher_spec)):
        if not isinstance(v, str) or not v:
            raise ValueError(f"`{n}` must be a non-empty character string")
    ks = getattr(keystore, "frame_id", keystore)
    setup = _dec.DecryptionSetup(keystore_id=ks, keystore_type=keystore_type, key_alias=key_alias,
                                 password=password, cipher_spec=cipher_spec, decrypt_tool_id=decrypt_tool or None,
                                 decrypt_impl=decrypt_impl)
    return _dec.make_tool(setup).key_id


def upload_file(path, destination_frame=None, header=0, sep=None, col_names=None, col_types=None, na_strings=None,
                skipped_columns=None, quotechar=None, escapechar=None):
    return _parse.upload_file(path, destination_frame, header, sep, col_names, col_types, na_strings, skipped_columns)


def parse_setup(raw_frames, destination_frame=None, header=0, separator=None, column_names=None, column_types=None,
                na_strings=None, **kw):
    return _parse.parse_setup(raw_frames, destination_frame, header, separator, column_names, column_types, na_strings)


def parse_raw(setup, id=None, first_line_is_header=0):
    src = setup["source_frames"][0]["name"]
    return _parse.import_file(src, id or setup.get("destination_frame"), header=first_line_is_header,
                              sep=setup.get("separator"), col_names=setup.get("column_names"))


def export_file(frame, path, force=False, sep=",", compression=None, parts=1, header=True, quote_header=True,
                parallel=False, format="csv"):
    return _parse.export_file(frame, path, force, sep, header, quote_header, parts, compression)


def save_frame(frame, dir_path, force=True):
    return _parse.save_frame(frame, dir_path, force)


def load_frame(frame_id, dir_path, force=True):
    return _parse.load_frame(frame_id, dir_path)


def create_frame(frame_id=None, rows=10000, cols=10, randomize=True, real_fraction=None, categorical_fraction=None,
                 integer_fraction=None, binary_fraction=None, time_fraction=None, string_fraction=None, value=0,
                 real_range=100, factors=100, integer_range=100, binary_ones_fraction=0.02, missing_fraction=0.01,
                 has_response=False, response_factors=2, positive_response=False, seed=None, seed_for_column_types=None):
    kw = dict(rows=rows, cols=cols, randomize=randomize, value=value, real_range=real_range, factors=factors,
              integer_range=integer_range, binary_ones_fraction=binary_ones_fraction, missing_fraction=missing_fraction,
              has_response=has_response, response_factors=response_factors, positive_response=positive_response,
              seed=seed, seed_for_column_types=seed_for_column_types, frame_id=frame_id)
    for k, v in (("categorical_fraction", categorical_fraction), ("integer_fraction", integer_fraction),
                 ("binary_fraction", binary_fraction), ("time_fraction", time_fraction),
                 ("string_fraction", string_fraction)):
        if v is not None:
            kw[k] = v
    return _fops.create_frame(**kw)


def interaction(data, factors, pairwise, max_factors, min_occurrence, destination_frame=None):
    return _fops.interaction(data, factors, pairwise, max_factors, min_occurrence)


def insert_missing_values(frame, fraction=0.1, seed=None):
    return _fops.insert_missing_values(frame, fraction, seed)


def dct(frame, dimensions, inverse=False, destination_frame=None):
    """``hex/DCTTransformer``: DCT-II (inverse: DCT-III) of every row laid out as [width, height, depth]."""
    from llama_github_io_amd.models.dct import dct as _dct
    return _dct(frame, dimensions, inverse)


def deep_copy(data, xid):
    cols = [c.copy() for c in data._cols.values()]
    return H2OFrame._from_columns(cols, xid)


def assign(data, xid):
    _dkv.remove(data.frame_id) if _dkv.contains(data.frame_id) else None
    data.frame_id = xid
    _dkv.put(xid, data)
    return data


def as_list(data, use_pandas=True, header=True):
    df = data.as_data_frame(use_pandas=True)
    if use_pandas:
        return df
    rows = df.values.tolist()
    return ([list(df.columns)] + rows) if header else rows


# ---- DKV
def get_frame(frame_id, **kw):
    from . import _conn
    if _conn.is_remote():            # a local copy of the server's frame (CSV download)
        import io as _io
        raw = _conn.current().request("GET /3/DownloadDataset", data={"frame_id": frame_id})
        import pandas as _pd
        return H2OFrame(_pd.read_csv(_io.BytesIO(raw if isinstance(raw, bytes) else str(raw).encode())))
    v = _dkv.get(frame_id)
    return v if isinstance(v, H2OFrame) else None


def get_model(model_id):
    from llama_github_io_amd.models.base import Model
    v = _dkv.get(model_id)
    return v if isinstance(v, Model) else None


def get_grid(grid_id):
    return _dkv.get(grid_id)


def get_job(job_id):
    return _dkv.get(job_id)


def ls():
    import pandas as pd
    from . import _conn
    if _conn.is_remote():
        c = _conn.current()
        keys = [f["frame_id"]["name"] for f in c.request("GET /3/Frames").get("frames", [])]
        keys += [m["model_id"]["name"] for m in c.request("GET /3/Models").get("models", [])]
        return pd.DataFrame({"key": keys})
    return pd.DataFrame({"key": _dkv.keys()})


def frames():
    return [k for k, v in _dkv.items() if isinstance(v, H2OFrame)]


def remove(x, cascade=True):
    from . import _conn
    xs = x if isinstance(x, (list, tuple)) else [x]
    for o in xs:
        key = o if isinstance(o, str) else getattr(o, "frame_id", None) or getattr(o, "model_id", None) or getattr(o, "key", None)
        if key is None:
            continue
        if _conn.is_remote():
            _conn.current().request(f"DELETE /3/DKV/{key}")
        elif _dkv.contains(key):
            _dkv.remove(key)


def remove_all(retained=None):
    keep = []
    for r in retained or []:
        keep.append(r if isinstance(r, str) else getattr(r, "frame_id", None) or getattr(r, "model_id", None))
    _dkv.remove_all(keep)


# ---- models: persistence & MOJO
def save_model(model, path="", force=False, export_cross_validation_predictions=False, filename=None):
    from llama_github_io_amd import persist
    return persist.save_model(getattr(model, "_model", None) or model, path, force, filename)


def load_model(path):
    from llama_github_io_amd import persist
    return persist.load_model(path)


download_model = save_model
upload_model = load_model


def import_mojo(mojo_path, model_id=None):
    from llama_github_io_amd.mojo import reader
    return reader.import_mojo(mojo_path, model_id)


upload_mojo = import_mojo


def mojo_predict_csv(input_csv_path, mojo_zip_path, output_csv_path=None, genmodel_jar_path=None, classpath=None,
                     java_options=None, verbose=False, setInvNumNA=False, predict_contributions=False,
                     predict_calibrated=False, extra_cmd_args=None):
    """Score a CSV file with a MOJO zip and write ``output_csv_path`` (default ``prediction.csv`` next to the zip);
    returns the prediction rows as dicts (reference: ``h2o-py/h2o/utils/shared_utils.py:478``, which runs
    ``hex.genmodel.tools.PredictCsv`` in a JVM). Here the MOJO is scored by the native MOJO reader, so
    ``genmodel_jar_path`` / ``classpath`` / ``java_options`` / ``extra_cmd_args`` are accepted and unused.
    ``setInvNumNA``: unparsable numbers become NA (PredictCsv ``--setConvertInvalidNum``) instead of an error."""
    import csv
    import os
    import pandas as pd
    from llama_github_io_amd.models.generic import GenericModel
    if not os.path.isfile(input_csv_path):
        raise RuntimeError("Input csv cannot be found at %s" % input_csv_path)
    mojo_zip_path = os.path.abspath(mojo_zip_path)
    if not os.path.isfile(mojo_zip_path):
        raise RuntimeError("MOJO zip cannot be found at %s" % mojo_zip_path)
    if output_csv_path is None:
        output_csv_path = os.path.join(os.path.dirname(mojo_zip_path), "prediction.csv")
    m = GenericModel.from_mojo(mojo_zip_path)
    df = pd.read_csv(input_csv_path)
    if "Unnamed: 0" in df.columns and "Unnamed: 0" not in m.info.x:     # pandas index written by to_csv
        df = df.drop(columns=["Unnamed: 0"])
    for j, name in enumerate(m.info.x):
        if name not in df.columns:
            continue
        if m.info.iscat[j]:
            df[name] = df[name].astype("string")
        elif df[name].dtype == object:
            num = pd.to_numeric(df[name], errors="coerce")
            bad = num.isna() & df[name].notna()
            if bad.any() and not setInvNumNA:
                raise ValueError(f"invalid numeric value {df[name][bad].iloc[0]!r} in column {name!r} "
                                 "(setInvNumNA=True turns it into NA)")
            df[name] = num
    types = {n: "enum" for j, n in enumerate(m.info.x) if m.info.iscat[j] and n in df.columns}
    fr = H2OFrame(df, column_types=types or None)
    if verbose:
        print("input_csv:\t%s\nmojo_zip:\t%s\noutput_csv:\t%s" % (input_csv_path, mojo_zip_path, output_csv_path))
    pred = m.predict_contributions(fr) if predict_contributions else m.predict(fr)
    out = pred.as_data_frame()
    if not predict_calibrated:
        out = out[[c for c in out.columns if not str(c).startswith("cal_")]]
    out.to_csv(output_csv_path, index=False)
    with open(output_csv_path) as fh:
        return list(csv.DictReader(fh))


def mojo_predict_pandas(dataframe, mojo_zip_path, genmodel_jar_path=None, classpath=None, java_options=None,
                        verbose=False, setInvNumNA=False, predict_contributions=False, predict_calibrated=False):
    """Score a pandas DataFrame with a MOJO zip (reference: ``h2o-py/h2o/utils/shared_utils.py:442``); returns the
    predictions as a DataFrame."""
    import os
    import shutil
    import tempfile
    import pandas as pd
    if not isinstance(dataframe, pd.DataFrame):
        raise TypeError("dataframe must be a pandas.DataFrame")
    d = tempfile.mkdtemp()
    try:
        inp, outp = os.path.join(d, "input.csv"), os.path.join(d, "prediction.csv")
        dataframe.to_csv(inp)
        mojo_predict_csv(inp, mojo_zip_path, outp, genmodel_jar_path, classpath, java_options, verbose, setInvNumNA,
                         predict_contributions, predict_calibrated)
        return pd.read_csv(outp)
    finally:
        shutil.rmtree(d)


def print_mojo(mojo_path, format="json", tree_index=None):
    from llama_github_io_amd.mojo import reader
    return reader.print_mojo(mojo_path, format, tree_index)


def make_metrics(predicted, actual, domain=None, distribution=None, weights=None, auc_type="NONE"):
    import torch
    from llama_github_io_amd import metrics as mm
    P = predicted.as_tensor(dtype=torch.float32)
    a = actual._col(0)
    if domain is not None or a.type == "enum":
        dom = list(domain or a.domain)
        from llama_github_io_amd.frame import _remap_codes
        y = _remap_codes(a, dom, P.device)
        cat = "Binomial" if len(dom) == 2 else "Multinomial"
        if cat == "Binomial" and P.shape[1] == 1:
            P = P[:, 0]
    else:
        y, dom, cat = a.as_float().float(), None, "Regression"
        P = P[:, 0]
    w = None if weights is None else weights.as_tensor(dtype=torch.float32)[:, 0]
    return mm.make_metrics(cat, y, P, w, dom, distribution)


def resume(recovery_dir=None):
    """Resume an interrupted grid search from its ``recovery_dir`` snapshot (/3/Recovery/resume)."""
    from llama_github_io_amd import grid as _g
    return _g.resume(recovery_dir)


def upload_custom_metric(func, func_file="metrics.py", func_name=None, class_name=None, source_provider=None):
    """Register a CMetricFunc class (map / reduce / metric); returns the ``custom_metric_func`` reference."""
    from llama_github_io_amd import udf
    return udf.upload_custom_metric(func, func_file, func_name, class_name, source_provider)


def upload_custom_distribution(func, func_file="distributions.py", func_name=None, class_name=None,
                               source_provider=None):
    """Register a CDistributionFunc class (link / init / gradient / gamma) for ``distribution="custom"``."""
    from llama_github_io_amd import udf
    return udf.upload_custom_distribution(func, func_file, func_name, class_name, source_provider)


def download_pojo(model, path="", get_jar=True, jar_name=""):
    """Java source of a scoring class extending hex.genmodel.GenModel (GBM/DRF/IF/GLM/KMeans)."""
    from llama_github_io_amd.mojo.pojo import download_pojo as _dp
    return _dp(getattr(model, "_model", model), path, get_jar, jar_name)


_flow_server = {}


def flow(open_browser=True, port=None):
    """Open the Flow notebook UI (h2o.py ``flow``): ``/flow/index.html`` of the connected REST server, or — in
    process — of a REST server started on 127.0.0.1 in a background thread over this process's frames and
    models. Returns the URL."""
    from . import _conn
    if _conn.is_remote():
        url = _conn.current().url + "/flow/index.html"
    else:
        if "url" not in _flow_server:
            import socket
            import threading
            import time as _time
            import uvicorn
            from llama_github_io_amd.api.server import create_app
            if port is None:
                s = socket.socket()
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
                s.close()
            srv = uvicorn.Server(uvicorn.Config(create_app(), host="127.0.0.1", port=int(port), log_level="warning"))
            threading.Thread(target=srv.run, daemon=True, name="h2o-flow").start()
            for _ in range(200):
                if srv.started:
                    break
                _time.sleep(0.05)
            _flow_server.update(url=f"http://127.0.0.1:{port}", server=srv)
        url = _flow_server["url"] + "/flow/index.html"
    if open_browser:
        import webbrowser
        webbrowser.open(url, new=1)
    return url


def explain(models, frame, columns=None, top_n_features=5, **kw):
    from .explanation import explain as _explain
    return _explain(models, frame, columns, top_n_features, **kw)


def explain_row(models, frame, row_index, columns=None, top_n_features=5, **kw):
    from .explanation import explain_row as _explain_row
    return _explain_row(models, frame, row_index, columns, top_n_features, **kw)


def cluster_status():
    return _rt.cluster_status()


def set_s3_credentials(secret_key_id, secret_access_key, session_token=None):
    """Credentials of every later ``s3://`` import (h2o.persist.set_s3_credentials; io/persist_store.py signs the
    S3 REST requests with them, AWS Signature V4)."""
    from .exceptions import H2OValueError
    if secret_key_id is None:
        raise H2OValueError("Secret key ID must be specified")
    if secret_access_key is None:
        raise H2OValueError("Secret access key must be specified")
    if not secret_key_id:
        raise H2OValueError("Secret key ID must not be empty")
    if not secret_access_key:
        raise H2OValueError("Secret access key must not be empty")
    from llama_github_io_amd.io import persist_store
    persist_store.set_s3_credentials(secret_key_id, secret_access_key, session_token)
    print("Credentials successfully set.")


def remove_s3_credentials():
    from llama_github_io_amd.io import persist_store
    persist_store.remove_s3_credentials()
    print("Credentials successfully removed.")


from . import grid, automl  # noqa: E402,F401
from .grid import H2OGridSearch  # noqa: E402,F401
from .automl import H2OAutoML, get_automl, get_leaderboard  # noqa: E402,F401

from ._more import (api, cluster_info, connection, demo, download_all_logs, download_csv,  # noqa: E402,F401
                    enable_expr_optimizations, estimate_cluster_mem, frame, get_timezone, import_hive_table,
                    import_sql_select, import_sql_table, is_expr_optimizations_enabled, lazy_import, list_timezones,
                    load_dataset, load_grid, log_and_echo, models, network_test, parse, rapids, save_grid,
                    set_timezone, version_check)

import_frame = import_file

from .explanation import (model_correlation, model_correlation_heatmap, pareto_front, pd_multi_plot,  # noqa: E402,F401
                          register_explain_methods, varimp, varimp_heatmap)
register_explain_methods()


def make_leaderboard(object, leaderboard_frame=None, sort_metric="AUTO", extra_columns=(), scoring_data="AUTO"):
    """Leaderboard over models / grids / AutoML runs (h2o-py scoring.make_leaderboard)."""
    from .scoring import make_leaderboard as _ml
    return _ml(object, leaderboard_frame, sort_metric, extra_columns, scoring_data)
