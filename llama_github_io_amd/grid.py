"""Hyper-parameter grid search (reference: ``hex/grid/GridSearch.java``, ``HyperSpaceWalker.java``
(Cartesian / RandomDiscrete with max_models, max_runtime_secs, stopping_rounds on the best-so-far
metric), ``hex/grid/Grid.java`` (sorted model table))."""
from __future__ import annotations

import itertools
import json
import math
import os
import shutil
import time

import numpy as np

from .core import dkv
from .core.job import Job
from .models import builder

_SORT_DESC = {"auc", "aucpr", "r2"}


def _metric_of(model, metric, use_valid=True):
    src = None
    for k in (("validation_metrics", "cross_validation_metrics", "training_metrics") if use_valid else ("training_metrics",)):
        if model.output.get(k):
            src = model.output[k]
            break
    if src is None:
        return float("nan")
    key = {"auc": "AUC", "aucpr": "pr_auc", "logloss": "logloss", "mse": "MSE", "rmse": "RMSE", "mae": "mae",
           "r2": "r2", "mean_per_class_error": "mean_per_class_error", "deviance": "mean_residual_deviance",
           "residual_deviance": "mean_residual_deviance", "tot_withinss": "tot_withinss",
           "misclassification": "mean_per_class_error"}.get(metric.lower(), metric)
    v = src.get(key)
    if v is None and key == "mean_residual_deviance":
        v = src.get("MSE")
    return float("nan") if v is None else float(v)


class Grid:
    def __init__(self, grid_id, algo, hyper_params, base_params):
        self.grid_id = grid_id
        self.algo = algo
        self.hyper_params = hyper_params
        self.base_params = base_params
        self.models = []
        self.hyper_values = []
        self.failures = []

    def sorted_models(self, sort_by=None, decreasing=None):
        if not self.models:
            return []
        m0 = self.models[0]
        cat = m0.model_category
        sort_by = sort_by or {"Binomial": "logloss", "Multinomial": "logloss", "Regression": "residual_deviance",
                              "Clustering": "tot_withinss"}.get(cat, "mse")
        if decreasing is None:
            decreasing = sort_by.lower() in _SORT_DESC
        vals = [_metric_of(m, sort_by) for m in self.models]
        order = sorted(range(len(vals)), key=lambda i: (math.isnan(vals[i]), -vals[i] if decreasing else vals[i]))
        return [(self.models[i], self.hyper_values[i], vals[i]) for i in order], sort_by


def walk(hyper_params: dict, criteria: dict | None, seed=None):
    names = list(hyper_params)
    space = [hyper_params[n] if isinstance(hyper_params[n], (list, tuple)) else [hyper_params[n]] for n in names]
    strategy = (criteria or {}).get("strategy", "Cartesian")
    combos = list(itertools.product(*space))
    if strategy.lower() == "randomdiscrete":
        rng = np.random.default_rng(None if seed in (None, -1) else int((criteria or {}).get("seed", seed) or 0))
        rng.shuffle(combos)
    return names, combos


def grid_search(algo, hyper_params, base_params, x, y, training_frame, validation_frame=None, grid_id=None,
                search_criteria=None, parallelism=1, job=None, recovery_dir=None) -> Grid:
    crit = dict(search_criteria or {})
    grid_id = grid_id or dkv.new_key(f"Grid_{algo.upper()}")
    grid = dkv.get(grid_id) if isinstance(dkv.get(grid_id), Grid) else Grid(grid_id, algo, hyper_params, base_params)
    rec = _Recovery(recovery_dir) if recovery_dir else None
    if rec is not None:
        rec.on_start(grid, x, y, training_frame, validation_frame, crit)
    names, combos = walk(hyper_params, crit, crit.get("seed"))
    max_models = int(crit.get("max_models", 0) or 0)
    max_rt = float(crit.get("max_runtime_secs", 0) or 0)
    stop_rounds = int(crit.get("stopping_rounds", 0) or 0)
    stop_metric = crit.get("stopping_metric", "AUTO")
    stop_tol = float(crit.get("stopping_tolerance", 1e-3))
    t0 = time.time()
    best_hist = []
    done = {tuple(map(str, h)) for h in grid.hyper_values}
    for combo in combos:
        if tuple(map(str, combo)) in done:
            continue
        if max_models and len(grid.models) >= max_models:
            break
        if max_rt and time.time() - t0 > max_rt:
            break
        p = dict(base_params)
        p.update(dict(zip(names, combo)))
        mid = f"{grid_id}_model_{len(grid.models) + len(grid.failures) + 1}"
        try:
            m = builder.train(algo, p, x, y, training_frame, validation_frame, job, mid)
        except Exception as e:  # noqa: BLE001 - recorded as a grid failure like GridSearch does
            grid.failures.append(dict(params=dict(zip(names, combo)), error=repr(e)))
            continue
        grid.models.append(m)
        grid.hyper_values.append(list(combo))
        if rec is not None:
            rec.on_model(grid, m, combo)
        if job is not None:
            job.update(1.0 / max(1, len(combos)))
        if stop_rounds > 0:
            metric = stop_metric if stop_metric != "AUTO" else ("logloss" if m.model_category in ("Binomial", "Multinomial") else "deviance")
            v = _metric_of(m, metric)
            larger = metric.lower() in _SORT_DESC
            best = max(best_hist[-1], v) if best_hist and larger else (min(best_hist[-1], v) if best_hist else v)
            best_hist.append(best)
            if len(best_hist) > stop_rounds:
                ref = best_hist[-stop_rounds - 1]
                imp = (best - ref) / abs(ref) if larger else (ref - best) / abs(ref) if ref else 0
                if imp < stop_tol:
                    break
    dkv.put(grid_id, grid)
    if rec is not None:
        rec.on_done()
    return grid


# ================================================================================================
# auto-recovery (reference: hex/faulttolerance/Recovery.java, Recoverable.java, /3/Recovery/resume)
class _Recovery:
    """Snapshot of a running grid in ``recovery_dir``: ``recovery.json`` (grid definition, references),
    the training / validation frames (binary frame save) and every finished model, so an interrupted
    search resumes with :func:`resume` without retraining finished models. Cleaned up on success."""

    META = "recovery.json"

    def __init__(self, path):
        self.path = path
        os.makedirs(path, exist_ok=True)

    def _write(self, meta):
        tmp = os.path.join(self.path, self.META + ".tmp")
        with open(tmp, "w") as f:
            json.dump(meta, f, default=str)
        os.replace(tmp, os.path.join(self.path, self.META))

    def on_start(self, grid, x, y, training_frame, validation_frame, crit):
        from .io.parse import save_frame
        save_frame(training_frame, os.path.join(self.path, "frames", "train"))
        if validation_frame is not None:
            save_frame(validation_frame, os.path.join(self.path, "frames", "valid"))
        self.meta = dict(kind="grid", grid_id=grid.grid_id, algo=grid.algo, hyper_params=grid.hyper_params,
                         base_params={k: v for k, v in grid.base_params.items() if _jsonable(v)}, x=x, y=y,
                         search_criteria=crit, training_frame=training_frame.frame_id,
                         validation_frame=None if validation_frame is None else validation_frame.frame_id,
                         has_valid=validation_frame is not None, models=[])
        for m, hv in zip(grid.models, grid.hyper_values):
            self.on_model(grid, m, hv, write=False)
        self._write(self.meta)

    def on_model(self, grid, model, combo, write=True):
        from .persist import save_model
        path = save_model(model, os.path.join(self.path, "models"), force=True)
        self.meta["models"].append(dict(key=model.key, path=path, hyper=[_jsonable_value(v) for v in combo]))
        if write:
            self._write(self.meta)

    def on_done(self):
        shutil.rmtree(self.path, ignore_errors=True)


def _jsonable(v):
    try:
        json.dumps(v)
        return True
    except TypeError:
        return False


def _jsonable_value(v):
    return v if _jsonable(v) else str(v)


def resume(recovery_dir: str) -> Grid:
    """``h2o.resume`` / ``/3/Recovery/resume``: reload the snapshot and continue the interrupted search."""
    from .io.parse import load_frame
    from .persist import load_model
    with open(os.path.join(recovery_dir, _Recovery.META)) as f:
        meta = json.load(f)
    train = load_frame(meta["training_frame"], os.path.join(recovery_dir, "frames", "train"))
    dkv.put(meta["training_frame"], train)
    valid = None
    if meta.get("has_valid"):
        valid = load_frame(meta["validation_frame"], os.path.join(recovery_dir, "frames", "valid"))
        dkv.put(meta["validation_frame"], valid)
    grid = Grid(meta["grid_id"], meta["algo"], meta["hyper_params"], meta["base_params"])
    for rec in meta["models"]:
        m = load_model(rec["path"])
        dkv.put(m.key, m)
        grid.models.append(m)
        grid.hyper_values.append(rec["hyper"])
    dkv.put(grid.grid_id, grid)
    return grid_search(meta["algo"], meta["hyper_params"], meta["base_params"], meta["x"], meta["y"], train, valid,
                       meta["grid_id"], meta["search_criteria"], recovery_dir=recovery_dir)
