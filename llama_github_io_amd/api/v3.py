"""V3 wire schemas (reference: ``h2o-core/src/main/java/water/api/schemas3/*V3.java`` and the h2o-py
client's dispatch on ``__meta.schema_name`` in ``h2o-py/h2o/backend/connection.py:894-915``).

Every response object carries ``__meta = {schema_version, schema_name, schema_type}``; the client turns
``CloudV3`` into ``H2OCluster``, ``TwoDimTableV3`` into ``H2OTwoDimTable``, ``ModelMetrics*V3`` into its
metrics classes and ``H2OErrorV3`` into ``H2OResponseError``. The builders below map the engine's
frames / models / jobs / metrics onto those layouts.
"""
from __future__ import annotations

import math
import time

import numpy as np

VERSION = "3.46.0.amd0"


def meta(name: str, type_: str | None = None, version: int = 3) -> dict:
    return dict(schema_version=version, schema_name=name, schema_type=type_ or name[:-2] if name.endswith(("V3", "V4")) else type_ or name)


def key(name, type_="Key"):
    if name is None:
        return None
    return {"__meta": meta("KeyV3", "Iced"), "name": str(name), "type": type_, "URL": None}


def frame_key(name):
    return key(name, "Key<Frame>") | {"__meta": meta("FrameKeyV3", "Key<Frame>")} if name else None


def model_key(name):
    return key(name, "Key<Model>") | {"__meta": meta("ModelKeyV3", "Key<Model>")} if name else None


def num(v):
    if v is None:
        return None
    try:
        f = float(v)
    except (TypeError, ValueError):
        return v
    if math.isnan(f):
        return "NaN"
    if math.isinf(f):
        return "Infinity" if f > 0 else "-Infinity"
    return f


def twodim(name: str, columns, rows, description: str = "", row_headers=None) -> dict:
    """TwoDimTableV3: ``columns`` = [(name, type, format)], ``rows`` = list of row lists; ``data`` is
    column-major as in the Java schema. ``row_headers`` adds the Java table's leading unnamed
    row-header column (clients drop it with ``fr[1:]``)."""
    if row_headers is not None:
        columns = [("", "string", "%s")] + list(columns)
        rows = [[h] + list(r) for h, r in zip(row_headers, rows)]
    cols = [dict(__meta=meta("ColumnSpecsBase", "Iced"), name=c[0], type=c[1], format=c[2], description=c[0])
            for c in columns]
    data = [[(num(r[j]) if columns[j][1] in ("double", "float", "long", "int") else r[j]) for r in rows]
            for j in range(len(columns))]
    return {"__meta": meta("TwoDimTableV3", "TwoDimTable"), "name": name, "description": description,
            "columns": cols, "rowcount": len(rows), "data": data}


def error(msg: str, exc: Exception | None = None, status: int = 412) -> dict:
    return {"__meta": meta("H2OErrorV3", "H2OError"), "timestamp": int(time.time() * 1000), "error_url": None,
            "msg": msg, "dev_msg": msg, "http_status": status, "values": {},
            "exception_type": type(exc).__name__ if exc else "H2OIllegalArgumentException",
            "exception_msg": msg, "stacktrace": []}


# ------------------------------------------------------------------------------------------------ cloud
def cloud(st: dict) -> dict:
    nodes = []
    for i, n in enumerate(st.get("nodes") or []):
        nodes.append({"__meta": meta("NodeV3", "Iced"), "h2o": n.get("h2o", "127.0.0.1"), "ip_port": n.get("h2o", ""),
                      "healthy": bool(n.get("healthy", True)), "last_ping": int(time.time() * 1000),
                      "pid": int(n.get("pid", 0) or 0), "num_cpus": n.get("num_cpus") or 0, "cpus_allowed": n.get("num_cpus") or 0,
                      "nthreads": n.get("num_cpus") or 0, "sys_load": 0.0, "my_cpu_pct": -1, "sys_cpu_pct": -1,
                      "mem_value_size": 0, "pojo_mem": 0, "free_mem": n.get("free_mem", 0) or 0,
                      "max_mem": n.get("mem_total", 0) or 0, "swap_mem": 0, "num_keys": 0, "free_disk": 0,
                      "max_disk": 0, "rpcs_active": 0, "fjthrds": [], "fjqueue": [], "tcps_active": 0,
                      "open_fds": -1, "gflops": 0.0, "mem_bw": 0.0, "gpu": n.get("gpu"),
                      "gcn_arch": n.get("gcn_arch"), "num_cus": n.get("num_cus")})
    return {"__meta": meta("CloudV3", "Iced"), "skip_ticks": False, "version": VERSION, "branch_name": "mi355x",
            "last_commit_hash": "", "describe": "", "compiled_by": "", "compiled_on": "", "build_number": "0",
            "build_age": "0 days", "build_too_old": False, "node_idx": 0, "cloud_name": st["cloud_name"],
            "cloud_size": st["cloud_size"], "cloud_uptime_millis": st["cloud_uptime_millis"],
            "cloud_internal_timezone": "UTC", "datafile_parser_timezone": "UTC",
            "cloud_healthy": bool(st["cloud_healthy"]), "bad_nodes": 0 if st["cloud_healthy"] else 1,
            "consensus": True, "locked": True, "is_client": False, "nodes": nodes,
            "internal_security_enabled": False, "web_ip": None}


# field lists of the schemas the client introspects at connect (Metadata/schemas/{name})
SCHEMA_FIELDS = {
    "CloudV3": ["skip_ticks", "version", "branch_name", "last_commit_hash", "describe", "compiled_by", "compiled_on",
                "build_number", "build_age", "build_too_old", "node_idx", "cloud_name", "cloud_size",
                "cloud_uptime_millis", "cloud_internal_timezone", "datafile_parser_timezone", "cloud_healthy",
                "bad_nodes", "consensus", "locked", "is_client", "nodes", "internal_security_enabled", "web_ip"],
    "H2OErrorV3": ["timestamp", "error_url", "msg", "dev_msg", "http_status", "values", "exception_type",
                   "exception_msg", "stacktrace"],
    "H2OModelBuilderErrorV3": ["timestamp", "error_url", "msg", "dev_msg", "http_status", "values",
                               "exception_type", "exception_msg", "stacktrace", "parameters", "messages",
                               "error_count"],
    "FrameV3": ["frame_id", "byte_size", "is_text", "row_offset", "row_count", "column_offset", "column_count",
                "full_column_count", "total_column_count", "checksum", "rows", "num_columns", "default_percentiles",
                "columns", "compatible_models", "chunk_summary", "distribution_summary"],
    "JobV3": ["key", "description", "status", "progress", "progress_msg", "start_time", "msec", "dest", "warnings",
              "exception", "stacktrace", "auto_recoverable", "ready_for_view"],
    "ModelSchemaV3": ["model_id", "algo", "algo_full_name", "response_column_name", "data_frame", "timestamp",
                      "have_pojo", "have_mojo", "parameters", "output", "compatible_frames", "checksum"],
}


def schema_metadata(name: str) -> dict:
    fields = SCHEMA_FIELDS.get(name)
    if fields is None:
        return None
    return {"__meta": meta("MetadataV3", "Iced"), "num": 1, "routes": [],
            "schemas": [{"__meta": meta("SchemaMetadataV3", "SchemaMetadata"), "version": 3, "name": name,
                         "superclass": "Schema", "type": name[:-2],
                         "fields": [{"__meta": meta("FieldMetadataV3", "FieldMetadata"), "name": f, "type": "Iced",
                                     "is_schema": False, "schema_name": None, "value": None, "help": f,
                                     "label": f, "required": False, "level": "critical", "direction": "OUTPUT",
                                     "is_inherited": False, "inherited_from": None, "is_gridable": False,
                                     "values": [], "json": False, "is_member_of_frames": [],
                                     "is_mutually_exclusive_with": []} for f in fields]}]}


# ------------------------------------------------------------------------------------------------ frames
_TYPE = {"real": "real", "int": "int", "enum": "enum", "string": "string", "time": "time"}


def column(fr, name, row_offset, row_count, rollups=True) -> dict:
    import torch
    c = fr._col(name)
    col = {"__meta": meta("ColV3", "Vec"), "label": name, "type": _TYPE.get(c.type, c.type), "domain": None,
           "domain_cardinality": 0, "string_data": None, "precision": -1, "histogram_bins": None,
           "histogram_base": 0, "histogram_stride": 0, "percentiles": None}
    n = fr.nrows
    if c.type == "string":
        vals = c.strings[row_offset:row_offset + row_count]
        col["string_data"] = [None if v is None else str(v) for v in vals]
        col["data"] = None
        na = sum(1 for v in c.strings if v is None)
        col.update(missing_count=na, zero_count=0, positive_infinity_count=0, negative_infinity_count=0,
                   mins=[], maxs=[], mean="NaN", sigma="NaN")
        return col
    v = c.data
    if c.type == "enum":
        col["domain"] = list(c.domain)
        col["domain_cardinality"] = len(c.domain)
        data = v[row_offset:row_offset + row_count].double()
        data = torch.where(data < 0, torch.full_like(data, float("nan")), data)
    else:
        data = v[row_offset:row_offset + row_count].double()
    col["data"] = [num(x) for x in data.cpu().tolist()]
    if rollups:
        x = v.double() if c.type != "enum" else torch.where(v < 0, torch.full(v.shape, float("nan"), dtype=torch.float64,
                                                                                device=v.device), v.double())
        ok = ~torch.isnan(x)
        xv = x[ok & torch.isfinite(x)]
        cnt = int(xv.numel())
        col.update(missing_count=int((~ok).sum()), zero_count=int((xv == 0).sum()),
                   positive_infinity_count=int((x == float("inf")).sum()),
                   negative_infinity_count=int((x == float("-inf")).sum()),
                   mins=[num(t) for t in torch.sort(xv)[0][:5].cpu().tolist()] if cnt else [],
                   maxs=[num(t) for t in torch.sort(xv, descending=True)[0][:5].cpu().tolist()] if cnt else [],
                   mean=num(float(xv.mean())) if cnt else "NaN",
                   sigma=num(float(xv.std())) if cnt > 1 else "NaN")
    return col


def frame(fr, row_offset=0, row_count=10, column_offset=0, column_count=-1, full=True) -> dict:
    names = fr.names
    total = len(names)
    if column_count is None or column_count < 0:
        column_count = total - column_offset
    sel = names[column_offset:column_offset + column_count]
    rc = max(0, min(int(row_count if row_count is not None and row_count >= 0 else 10), fr.nrows - row_offset))
    return {"__meta": meta("FrameV3", "Frame"), "frame_id": frame_key(fr.frame_id), "byte_size": 0, "is_text": False,
            "row_offset": row_offset, "row_count": rc, "column_offset": column_offset, "column_count": len(sel),
            "full_column_count": total, "total_column_count": total, "checksum": 0, "rows": fr.nrows,
            "num_columns": total, "default_percentiles": [], "compatible_models": None, "chunk_summary": None,
            "distribution_summary": None,
            "columns": [column(fr, n, row_offset, rc, rollups=full) for n in sel]}


def frames(list_of, **kw) -> dict:
    return {"__meta": meta("FramesV3", "Frames"), "frame_id": None, "row_offset": 0, "row_count": 10,
            "column_offset": 0, "column_count": -1, "find_compatible_models": False, "path": None, "force": False,
            "num_parts": 1, "compression": None, "separator": 44, "header": True, "quote_header": True,
            "job": None, "compatible_models": None, "domain": None, "frames": list_of}


# ------------------------------------------------------------------------------------------------ jobs
def job(j) -> dict:
    d = j.to_dict() if hasattr(j, "to_dict") else dict(j)
    for k in ("key", "dest"):
        if isinstance(d.get(k), dict):
            d[k] = d[k].get("name")
    st = str(d.get("status", "DONE")).upper()
    st = {"SUCCEEDED": "DONE", "FINISHED": "DONE", "ERROR": "FAILED", "CANCELED": "CANCELLED"}.get(st, st)
    exc = d.get("exception")
    dest = d.get("dest")
    return {"__meta": meta("JobV3", "Job"), "key": key(d.get("key"), "Key<Job>"), "description": d.get("description", ""),
            "status": st, "progress": float(d.get("progress", 1.0 if st == "DONE" else 0.0) or 0.0),
            "progress_msg": d.get("progress_msg") or "", "start_time": int(d.get("start_time") or 0),
            "msec": int(d.get("msec", 0) or 0), "dest": key(dest, "Key<Keyed>") if dest else key("", "Key<Keyed>"),
            "warnings": d.get("warnings") or [], "exception": exc, "stacktrace": d.get("stacktrace") or (exc or ""),
            "auto_recoverable": False, "ready_for_view": st == "DONE"}


# ------------------------------------------------------------------------------------------------ metrics
_THR_COLS = ["threshold", "f1", "f2", "f0point5", "accuracy", "precision", "recall", "specificity", "absolute_mcc",
             "min_per_class_accuracy", "mean_per_class_accuracy", "tns", "fns", "fps", "tps"]


def metrics(mm: dict | None, category: str, model_id=None, frame_id=None, algo="") -> dict | None:
    if mm is None:
        return None
    cat = category
    name = {"Binomial": "ModelMetricsBinomialV3", "Multinomial": "ModelMetricsMultinomialV3",
            "Regression": "ModelMetricsRegressionV3", "Clustering": "ModelMetricsClusteringV3",
            "AnomalyDetection": "ModelMetricsAnomalyV3", "AutoEncoder": "ModelMetricsAutoEncoderV3",
            "Ordinal": "ModelMetricsOrdinalV3", "DimReduction": "ModelMetricsPCAV3",
            "CoxPH": "ModelMetricsRegressionCoxPHV3"}.get(cat, "ModelMetricsBaseV3")
    if algo == "glm" and cat in ("Binomial", "Multinomial", "Regression"):
        name = name.replace("ModelMetrics", "ModelMetrics").replace("V3", "GLMV3")
    out = {"__meta": meta(name, name[:-2].replace("ModelMetrics", "ModelMetrics")),
           "model": model_key(model_id), "model_checksum": 0, "frame": frame_key(frame_id), "frame_checksum": 0,
           "description": None, "scoring_time": int(time.time() * 1000), "predictions": None,
           "model_category": cat, "custom_metric_name": mm.get("custom_metric_name"),
           "custom_metric_value": num(mm.get("custom_metric_value", 0.0))}
    for k, v in mm.items():
        if k in ("thresholds_and_metric_scores", "gains_lift_table", "cm", "max_criteria_and_metric_scores",
                 "hit_ratio_table", "confusion_matrix", "withinss", "size", "domain"):
            continue
        if isinstance(v, (int, float, np.floating, np.integer)) and not isinstance(v, bool):
            out[k] = num(v)
        elif isinstance(v, (str, bool)) or v is None:
            out[k] = v
    out.setdefault("nobs", mm.get("nobs", 0))
    if cat == "Binomial":
        thr = mm.get("thresholds_and_metric_scores") or []
        out["domain"] = mm.get("domain")
        out["thresholds_and_metric_scores"] = twodim(
            "Metrics for Thresholds", [(c, "long" if c in ("tns", "fns", "fps", "tps") else "double",
                                       "%d" if c in ("tns", "fns", "fps", "tps") else "%f") for c in _THR_COLS]
            + [("idx", "int", "%d")], [[r[c] for c in _THR_COLS] + [i] for i, r in enumerate(thr)])
        crit = []
        for c in ("f1", "f2", "f0point5", "accuracy", "precision", "recall", "specificity", "absolute_mcc",
                  "min_per_class_accuracy", "mean_per_class_accuracy", "tns", "fns", "fps", "tps"):
            if thr:
                i = max(range(len(thr)), key=lambda k: thr[k][c])
                crit.append(["max " + c, thr[i]["threshold"], thr[i][c], i])
        out["max_criteria_and_metric_scores"] = twodim(
            "Maximum Metrics", [("metric", "string", "%s"), ("threshold", "double", "%f"), ("value", "double", "%f"),
                                ("idx", "long", "%d")], crit, "Maximum Metrics at their respective thresholds")
        cm = mm.get("cm")
        if cm:
            dom = list(mm.get("domain") or ["0", "1"])
            t = cm["table"]
            rows = []
            for i, lab in enumerate(dom):
                tot = t[i][0] + t[i][1]
                err = t[i][1 - i] / tot if tot else 0.0
                rows.append([lab, t[i][0], t[i][1], err, f"{t[i][1 - i]:g} / {tot:g}"])
            tot_err = t[0][1] + t[1][0]
            tot_all = sum(map(sum, t))
            rows.append(["Total", t[0][0] + t[1][0], t[0][1] + t[1][1], tot_err / tot_all if tot_all else 0.0,
                         f"{tot_err:g} / {tot_all:g}"])
            out["cm"] = {"__meta": meta("ConfusionMatrixV3", "ConfusionMatrix"),
                         "table": twodim("Confusion Matrix", [("", "string", "%s")] + [(d, "double", "%f") for d in dom]
                                         + [("Error", "double", "%.4f"), ("Rate", "string", "%s")], rows,
                                         f"Confusion Matrix for max f1 @ threshold = {cm['threshold']}")}
        gl = mm.get("gains_lift_table") or []
        if gl:
            gcols = list(gl[0].keys())
            out["gains_lift_table"] = twodim("Gains/Lift Table", [(c, "int" if c == "group" else "double",
                                                                   "%d" if c == "group" else "%f") for c in gcols],
                                             [[r[c] for c in gcols] for r in gl])
    elif cat == "Multinomial":
        out["domain"] = mm.get("domain")
        cmx = mm.get("confusion_matrix") or ((mm.get("cm") or {}).get("table"))
        if cmx is not None:
            dom = list(mm.get("domain") or [])
            rows = []
            for i, lab in enumerate(dom):
                row = list(cmx[i])
                tot = sum(row)
                err = (tot - row[i]) / tot if tot else 0.0
                rows.append([lab] + row + [err, f"{tot - row[i]:g} / {tot:g}"])
            out["cm"] = {"__meta": meta("ConfusionMatrixV3", "ConfusionMatrix"),
                         "table": twodim("Confusion Matrix", [("", "string", "%s")] + [(d, "double", "%f") for d in dom]
                                         + [("Error", "double", "%.4f"), ("Rate", "string", "%s")], rows)}
        hr = mm.get("hit_ratio_table")
        if hr:
            out["hit_ratio_table"] = twodim("Top-K Hit Ratios", [("k", "int", "%d"), ("hit_ratio", "float", "%f")],
                                            [[i + 1, v] for i, v in enumerate(hr)])
    elif cat == "Clustering":
        ws, sz = mm.get("withinss") or [], mm.get("size") or []
        out["centroid_stats"] = twodim("Centroid Statistics", [("centroid", "int", "%d"), ("size", "double", "%f"),
                                                                ("within_cluster_sum_of_squares", "double", "%f")],
                                       [[i + 1, s, w] for i, (s, w) in enumerate(zip(sz, ws))])
    return out


# ------------------------------------------------------------------------------------------------ models
def _param_type(v):
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, int):
        return "int"
    if isinstance(v, float):
        return "double"
    if isinstance(v, (list, tuple)):
        return "string[]"
    return "string"


def _json_value(v):
    if isinstance(v, float):
        return num(v)
    if isinstance(v, (list, tuple)):
        return [_json_value(x) for x in v]
    if isinstance(v, (str, int, bool)) or v is None:
        return v
    if isinstance(v, dict):
        return {str(k): _json_value(x) for k, x in v.items()}
    return str(v)


def model(m) -> dict:
    from ..models.params import schema
    out = m.output
    cat = m.model_category
    params = []
    sch = schema(m.algo) or {}
    for k in sorted(set(sch) | set(m.params)):
        if k.startswith("_"):
            continue
        v = m.params.get(k, sch.get(k))
        if k in ("training_frame", "validation_frame"):
            v = frame_key(out.get(k) if isinstance(out.get(k), str) else None)
        params.append({"__meta": meta("ModelParameterSchemaV3", "Iced"), "name": k, "label": k, "help": k,
                       "required": False, "type": _param_type(v), "default_value": _json_value(sch.get(k)),
                       "actual_value": _json_value(v), "input_value": _json_value(m.params.get(k)), "level": "critical",
                       "values": [], "is_member_of_frames": [], "is_mutually_exclusive_with": [], "gridable": False})
    names = out.get("names") or (m.info.x + ([m.info.response] if m.info.response else []))
    doms = out.get("domains") or m.info.domains
    doms = list(doms) + ([m.info.response_domain] if m.info.response else [])
    o = {"__meta": meta("ModelOutputSchemaV3", "ModelOutput"), "model_category": cat, "names": names,
         "original_names": None, "column_types": ["Enum" if d is not None else "Numeric" for d in doms[:len(names)]],
         "domains": doms[:len(names)], "cross_validation_models": None, "cross_validation_predictions": None,
         "cross_validation_holdout_predictions_frame_id": None, "cross_validation_fold_assignment_frame_id": None,
         "status": "DONE", "start_time": int(time.time() * 1000) - int(out.get("run_time_ms", 0)),
         "end_time": int(time.time() * 1000), "run_time": int(out.get("run_time_ms", 0)),
         "default_threshold": num(m.default_threshold() if hasattr(m, "default_threshold") else None) or 0.5,
         "help": {}, "response_column_name": m.info.response}
    for which in ("training_metrics", "validation_metrics", "cross_validation_metrics"):
        o[which] = metrics(out.get(which), cat, m.key, out.get("training_frame") if which == "training_metrics" else
                           out.get("validation_frame"), m.algo)
    for k in ("cross_validation_metrics_summary", "model_summary", "scoring_history", "variable_importances",
              "validation_metrics", "cross_validation_metrics"):
        o.setdefault(k, None)
    cvs = out.get("cross_validation_metrics_summary")
    if isinstance(cvs, dict) and cvs:
        nfold = max((len(v.get("values", [])) for v in cvs.values()), default=0)
        cols = [("", "string", "%s"), ("mean", "double", "%f"), ("sd", "double", "%f")] + \
            [(f"cv_{i + 1}_valid", "double", "%f") for i in range(nfold)]
        rows = [[k, v.get("mean"), v.get("sd")] + list(v.get("values", [])) + [None] * (nfold - len(v.get("values", [])))
                for k, v in cvs.items()]
        o["cross_validation_metrics_summary"] = twodim("Cross-Validation Metrics Summary", cols, rows)
    cvm = out.get("cross_validation_models")
    if cvm:
        o["cross_validation_models"] = [model_key(k) for k in cvm]
    if out.get("cross_validation_holdout_predictions_frame_id"):
        o["cross_validation_holdout_predictions_frame_id"] = frame_key(out["cross_validation_holdout_predictions_frame_id"])
    summ = out.get("model_summary")
    if isinstance(summ, dict) and summ:
        o["model_summary"] = twodim("Model Summary", [(k, _tab_type(v), _tab_fmt(v)) for k, v in summ.items()],
                                    [[_json_value(v) for v in summ.values()]])
    hist = out.get("scoring_history")
    if isinstance(hist, list) and hist:
        ks = [k for k in hist[0].keys()]
        o["scoring_history"] = twodim("Scoring History", [(k, _tab_type(hist[0][k]), _tab_fmt(hist[0][k])) for k in ks],
                                      [[_json_value(e.get(k)) for k in ks] for e in hist])
    vi = out.get("variable_importances")
    if vi:
        rows = [list(r) if isinstance(r, (list, tuple)) else [r.get("variable"), r.get("relative_importance"),
                                                               r.get("scaled_importance"), r.get("percentage")] for r in vi]
        o["variable_importances"] = twodim("Variable Importances", [("variable", "string", "%s"),
                                                                    ("relative_importance", "double", "%f"),
                                                                    ("scaled_importance", "double", "%f"),
                                                                    ("percentage", "double", "%f")], rows)
    if m.algo == "kmeans" and out.get("centers") is not None:
        cn = out.get("center_names") or [f"C{j + 1}" for j in range(len(out["centers"][0]))]
        for k in ("centers", "centers_std"):
            if out.get(k) is not None:
                o[k] = twodim("Cluster Means" if k == "centers" else "Standardized Cluster Means",
                              [("centroid", "int", "%d")] + [(c, "double", "%f") for c in cn],
                              [[i + 1] + list(r) for i, r in enumerate(out[k])])
    for k, v in out.items():
        if k in o or k.startswith("_") or k in ("training_frame", "validation_frame"):
            continue
        if isinstance(v, (str, int, float, bool)) or v is None:
            o[k] = _json_value(v)
        elif isinstance(v, (list, tuple)) and v and all(isinstance(r, dict) for r in v):
            cols = list(v[0].keys())
            o[k] = twodim(k, [(c, _tab_type(v[0][c]), _tab_fmt(v[0][c])) for c in cols],
                          [[_json_value(r.get(c)) for c in cols] for r in v])
        elif isinstance(v, (list, tuple)) and v and all(isinstance(r, (list, tuple)) for r in v) and \
                all(isinstance(x, (int, float)) or x is None for r in v for x in r):
            o[k] = twodim(k, [(f"C{j + 1}", "double", "%f") for j in range(max(len(r) for r in v))], [list(r) for r in v])
        elif isinstance(v, (list, tuple, dict)):
            o[k] = _json_value(v)
        elif k in ("coefficients",) and isinstance(v, dict) and "coefficients_table" not in out:
            o["coefficients_table"] = twodim("Coefficients", [("names", "string", "%s"), ("coefficients", "double", "%f"),
                                                              ("standardized_coefficients", "double", "%f")],
                                             [[n, c, (out.get("standardized_coefficients") or {}).get(n)]
                                              for n, c in v.items()])
    return {"__meta": meta("ModelSchemaV3", "Model"), "model_id": model_key(m.key), "algo": m.algo,
            "algo_full_name": _FULL.get(m.algo, m.algo), "response_column_name": m.info.response,
            "data_frame": frame_key(out.get("training_frame")), "timestamp": int(time.time() * 1000),
            "have_pojo": m.algo in ("gbm", "drf", "isolationforest", "glm", "kmeans"), "have_mojo": True,
            "parameters": params, "output": o, "compatible_frames": [], "checksum": 0}


def _tab_type(v):
    return "string" if isinstance(v, str) else ("long" if isinstance(v, int) and not isinstance(v, bool) else "double")


def _tab_fmt(v):
    return "%s" if isinstance(v, str) else ("%d" if isinstance(v, int) and not isinstance(v, bool) else "%f")


_FULL = {"gbm": "Gradient Boosting Machine", "drf": "Distributed Random Forest", "glm": "Generalized Linear Modeling",
         "deeplearning": "Deep Learning", "kmeans": "K-means", "xgboost": "XGBoost", "naivebayes": "Naive Bayes",
         "pca": "Principal Components Analysis", "svd": "Singular Value Decomposition",
         "glrm": "Generalized Low Rank Modeling", "isolationforest": "Isolation Forest",
         "extendedisolationforest": "Extended Isolation Forest", "stackedensemble": "Stacked Ensemble",
         "word2vec": "Word2Vec", "coxph": "Cox Proportional Hazards", "rulefit": "RuleFit",
         "isotonicregression": "Isotonic Regression", "aggregator": "Aggregator", "psvm": "PSVM",
         "targetencoder": "TargetEncoder", "gam": "Generalized Additive Model", "anovaglm": "ANOVA GLM",
         "modelselection": "Model Selection", "upliftdrf": "Uplift Distributed Random Forest",
         "dt": "Decision Tree", "infogram": "Infogram", "generic": "Import MOJO Model"}
