"""``h2o.make_leaderboard`` (reference: h2o-py/h2o/scoring.py): one leaderboard over models, grids and AutoML
runs, scored on a frame or on their own train / valid / xval metrics."""
from __future__ import annotations


def _model_ids(obj):
    if isinstance(obj, (list, tuple)):
        out = []
        for o in obj:
            r = _model_ids(o)
            out.extend(r if isinstance(r, list) else [r])
        return out
    if hasattr(obj, "_aml"):                                 # H2OAutoML
        return [r["model_id"] for r in obj._aml.leaderboard_rows()[0]]
    if hasattr(obj, "model_ids"):                            # H2OGridSearch
        return list(obj.model_ids)
    if getattr(obj, "model_id", None) is not None:
        return obj.model_id
    if isinstance(obj, str):
        return obj
    raise ValueError("Unsupported model_id!")


def make_leaderboard(object, leaderboard_frame=None, sort_metric="AUTO", extra_columns=(), scoring_data="AUTO"):
    import pandas as pd
    from llama_github_io_amd.automl import AutoML
    from llama_github_io_amd.core import dkv
    from llama_github_io_amd.frame import H2OFrame
    if str(scoring_data).lower() not in ("auto", "train", "valid", "xval"):
        raise ValueError('Scoring data has to be set to one of "AUTO", "train", "valid", "xval".')
    ids = _model_ids(object)
    ids = [ids] if isinstance(ids, str) else ids
    models = [dkv.get(i) for i in ids]
    if any(m is None for m in models):
        raise ValueError(f"unknown model ids: {[i for i, m in zip(ids, models) if m is None]}")
    sd = str(scoring_data).lower()
    if leaderboard_frame is None and sd != "auto":
        # rank on the requested metrics: train / valid / xval
        src = {"train": "training_metrics", "valid": "validation_metrics", "xval": "cross_validation_metrics"}[sd]
        shadow = []
        for m in models:
            c = type(m).__new__(type(m))
            c.__dict__.update(m.__dict__)
            c.output = dict(m.output, training_metrics=m.output.get(src) or {})
            shadow.append(c)
        models = shadow
    lb = AutoML.__new__(AutoML)
    lb.models, lb.sort_metric, lb.leaderboard_frame = models, sort_metric, leaderboard_frame
    rows, cols = lb.leaderboard_rows()
    df = pd.DataFrame(rows, columns=cols)
    ex = [extra_columns] if isinstance(extra_columns, str) else list(extra_columns or [])
    if any(str(e).upper() == "ALL" for e in ex):
        ex = ["training_time_ms", "predict_time_per_row_ms", "algo"]
    by_id = {m.key: dkv.get(m.key) for m in models}
    if "training_time_ms" in ex:
        df["training_time_ms"] = [int(by_id[k].output.get("run_time_ms") or 0) for k in df["model_id"]]
    if "predict_time_per_row_ms" in ex:
        if leaderboard_frame is None:
            raise ValueError("predict_time_per_row_ms needs a leaderboard_frame")
        import time
        vals = []
        for k in df["model_id"]:
            t0 = time.perf_counter()
            by_id[k].predict(leaderboard_frame)
            vals.append(1000.0 * (time.perf_counter() - t0) / max(1, leaderboard_frame.nrows))
        df["predict_time_per_row_ms"] = vals
    if "algo" in ex:
        df["algo"] = [by_id[k].algo for k in df["model_id"]]
    return H2OFrame(df)
