"""AutoML (reference: ``h2o-automl/src/main/java/ai/h2o/automl/AutoML.java``, ``ModelingPlans.java``,
``Leaderboard.java``, ``modeling/*StepsProvider.java``).

Modeling plan (H2O default order, trimmed by ``include_algos``/``exclude_algos``): XGBoost (3
presets), GLM, DRF, GBM (5 presets), DeepLearning, XRT, GBM/XGBoost random grids while budget
remains, then two Stacked Ensembles (best-of-family, all models). Every model gets ``nfolds``
(default 5, Modulo fold assignment so all share folds) CV with kept holdout predictions. Budgets:
``max_models``, ``max_runtime_secs`` (default 3600 when neither is set), ``max_runtime_secs_per_model``.
Leaderboard sort: AUC (binomial), mean_per_class_error (multinomial), mean_residual_deviance
(regression), with the other standard columns.
"""
from __future__ import annotations

import math
import time

import numpy as np

from .core import dkv
from .core.job import Job
from .grid import _metric_of
from .models import builder

_DEFAULT_SORT = {"Binomial": "auc", "Multinomial": "mean_per_class_error", "Regression": "mean_residual_deviance"}
_DESC = {"auc", "aucpr", "r2"}


def _plan(seed):
    s = seed
    return [
        ("xgboost", "XGBoost_1", dict(ntrees=100, max_depth=10, min_rows=5, sample_rate=0.6, col_sample_rate=0.8, col_sample_rate_per_tree=0.8, seed=s)),
        ("xgboost", "XGBoost_2", dict(ntrees=100, max_depth=20, min_rows=10, sample_rate=0.6, col_sample_rate=0.8, col_sample_rate_per_tree=0.8, seed=s)),
        ("xgboost", "XGBoost_3", dict(ntrees=100, max_depth=5, min_rows=3, sample_rate=0.8, col_sample_rate=0.8, col_sample_rate_per_tree=0.8, seed=s)),
        ("glm", "GLM_1", dict(lambda_search=True, seed=s)),
        ("drf", "DRF_1", dict(ntrees=50, seed=s)),
        ("gbm", "GBM_1", dict(ntrees=100, max_depth=6, min_rows=1, sample_rate=0.8, col_sample_rate=0.8, col_sample_rate_per_tree=0.8, seed=s)),
        ("gbm", "GBM_2", dict(ntrees=100, max_depth=7, min_rows=10, sample_rate=0.8, col_sample_rate=0.8, col_sample_rate_per_tree=0.8, seed=s)),
        ("gbm", "GBM_3", dict(ntrees=100, max_depth=8, min_rows=10, sample_rate=0.8, col_sample_rate=0.8, col_sample_rate_per_tree=0.8, seed=s)),
        ("gbm", "GBM_4", dict(ntrees=100, max_depth=10, min_rows=10, sample_rate=0.8, col_sample_rate=0.8, col_sample_rate_per_tree=0.8, seed=s)),
        ("gbm", "GBM_5", dict(ntrees=100, max_depth=15, min_rows=100, sample_rate=0.8, col_sample_rate=0.8, col_sample_rate_per_tree=0.8, seed=s)),
        ("deeplearning", "DeepLearning_1", dict(epochs=10, hidden=[10, 10, 10], seed=s)),
        ("drf", "XRT_1", dict(ntrees=50, histogram_type="Random", seed=s)),
    ]


def _random_grid(algo, rng, seed):
    if algo == "gbm":
        return dict(ntrees=int(rng.choice([50, 100, 200])), max_depth=int(rng.choice([3, 5, 7, 9, 11, 13])),
                    min_rows=float(rng.choice([1, 5, 10, 15, 30, 100])), learn_rate=float(rng.choice([0.01, 0.05, 0.1])),
                    sample_rate=float(rng.choice([0.5, 0.6, 0.7, 0.8, 0.9, 1.0])),
                    col_sample_rate=float(rng.choice([0.4, 0.7, 1.0])), seed=seed)
    return dict(ntrees=int(rng.choice([50, 100, 200])), max_depth=int(rng.choice([5, 10, 15, 20])),
                min_rows=float(rng.choice([0.01, 0.1, 1, 3, 5, 10])), sample_rate=float(rng.choice([0.6, 0.8, 1.0])),
                col_sample_rate=float(rng.choice([0.6, 0.8, 1.0])), reg_lambda=float(rng.choice([0.001, 0.01, 0.1, 1, 10])),
                reg_alpha=float(rng.choice([0.001, 0.01, 0.1, 0.5, 1])), seed=seed)


class AutoML:
    def __init__(self, project_name=None, max_models=None, max_runtime_secs=None, max_runtime_secs_per_model=0,
                 nfolds=5, seed=None, sort_metric="AUTO", include_algos=None, exclude_algos=None,
                 stopping_metric="AUTO", stopping_rounds=3, stopping_tolerance=None, balance_classes=False,
                 keep_cross_validation_predictions=True, keep_cross_validation_models=False, verbosity="warn", **kw):
        self.project_name = project_name or dkv.new_key("AutoML")
        self.max_models = max_models
        self.max_runtime_secs = max_runtime_secs if max_runtime_secs is not None else (0 if max_models else 3600)
        self.per_model = max_runtime_secs_per_model or 0
        self.nfolds = nfolds
        self.seed = seed if seed not in (None, -1) else int(np.random.SeedSequence().entropy % (1 << 31))
        self.sort_metric = sort_metric
        self.include = [a.lower() for a in include_algos] if include_algos else None
        self.exclude = [a.lower() for a in exclude_algos] if exclude_algos else []
        self.stopping = dict(stopping_metric=stopping_metric, stopping_rounds=stopping_rounds,
                             stopping_tolerance=stopping_tolerance)
        self.models = []
        self.event_log = []

    def _allowed(self, algo):
        name = {"gbm": "gbm", "drf": "drf", "xgboost": "xgboost", "glm": "glm", "deeplearning": "deeplearning",
                "stackedensemble": "stackedensemble"}[algo]
        if self.include is not None and name not in self.include:
            return False
        return name not in self.exclude

    def _log(self, msg):
        self.event_log.append(dict(timestamp=time.time(), message=msg))

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, leaderboard_frame=None,
              blending_frame=None, fold_column=None, weights_column=None, job: Job | None = None):
        t0 = time.time()
        common = dict(nfolds=self.nfolds if not fold_column else 0, fold_assignment="Modulo",
                      keep_cross_validation_predictions=True, keep_cross_validation_models=False,
                      fold_column=fold_column, weights_column=weights_column)
        if self.stopping["stopping_rounds"]:
            common.update(stopping_rounds=self.stopping["stopping_rounds"], stopping_metric=self.stopping["stopping_metric"])
        from .parallel import collectives as coll
        # every rank takes rank 0's budget decision (a rank must not start a model the others skip)
        budget = lambda: coll.agree((self.max_runtime_secs <= 0 or time.time() - t0 < self.max_runtime_secs) and
                                    (not self.max_models or len(self.models) < self.max_models))  # noqa: E731
        steps = _plan(self.seed)
        rng = np.random.default_rng(self.seed)
        i = 0
        while budget():
            if i < len(steps):
                algo, name, p = steps[i]
            else:
                if not (self._allowed("gbm") or self._allowed("xgboost")):
                    break
                algo = "gbm" if (i % 2 == 0 and self._allowed("gbm")) or not self._allowed("xgboost") else "xgboost"
                name = f"{dict(gbm='GBM', xgboost='XGBoost')[algo]}_grid_1_model_{i - len(steps) + 1}"
                p = _random_grid(algo, rng, self.seed)
                if i > len(steps) + 200:
                    break
            i += 1
            if not self._allowed(algo):
                continue
            p = dict(p, **common)
            if self.per_model:
                p["max_runtime_secs"] = self.per_model
            elif self.max_runtime_secs > 0:
                p["max_runtime_secs"] = coll.broadcast_object(max(1.0, self.max_runtime_secs - (time.time() - t0)))
            mid = f"{name}_AutoML_{self.project_name}"
            try:
                m = builder.train(algo, p, x, y, training_frame, validation_frame, job, mid)
                self.models.append(m)
                self._log(f"built {mid}")
            except Exception as e:  # noqa: BLE001 - AutoML logs and moves on (EventLog)
                self._log(f"{mid} failed: {e!r}")
        if self._allowed("stackedensemble") and len(self.models) >= 2 and self.models[0].info.response:
            self._ensembles(x, y, training_frame, validation_frame, job)
        self.leaderboard_frame = leaderboard_frame
        dkv.put(self.project_name, self)
        return self

    def _ensembles(self, x, y, fr, valid, job):
        cat = self.models[0].model_category
        metric = self._sort_key(cat)
        best = {}
        for m in self.models:
            if getattr(m, "cv_holdout", None) is None:
                continue
            fam = m.algo if not m.key.startswith("XRT") else "xrt"
            v = _metric_of(m, metric)
            if fam not in best or self._better(v, best[fam][1], metric):
                best[fam] = (m, v)
        for name, ms in (("BestOfFamily", [b[0] for b in best.values()]),
                         ("AllModels", [m for m in self.models if getattr(m, "cv_holdout", None) is not None])):
            if len(ms) < 2:
                continue
            mid = f"StackedEnsemble_{name}_1_AutoML_{self.project_name}"
            try:
                # StackedEnsembleStepsProvider.setMetalearnerParameters: the metalearner is cross-validated
                # with the AutoML nfolds, and its out-of-fold metrics are what the leaderboard ranks
                sp = dict(base_models=[m.key for m in ms], seed=self.seed, metalearner_nfolds=self.nfolds,
                          metalearner_fold_assignment="Modulo", keep_levelone_frame=True)
                if cat in ("Binomial", "Multinomial"):
                    sp["metalearner_transform"] = "Logit"
                se = builder.train("stackedensemble", sp, x, y, fr, valid, job, mid)
                self.models.append(se)
            except Exception as e:  # noqa: BLE001
                self._log(f"{mid} failed: {e!r}")

    def _sort_key(self, cat):
        s = str(self.sort_metric).lower()
        return _DEFAULT_SORT.get(cat, "mse") if s == "auto" else s

    @staticmethod
    def _better(a, b, metric):
        if math.isnan(b):
            return True
        return a > b if metric in _DESC else a < b

    def leaderboard_rows(self):
        if not self.models:
            return [], []
        cat = self.models[0].model_category
        key = self._sort_key(cat)
        cols = {"Binomial": ["auc", "logloss", "aucpr", "mean_per_class_error", "rmse", "mse"],
                "Multinomial": ["mean_per_class_error", "logloss", "rmse", "mse"],
                "Regression": ["mean_residual_deviance", "rmse", "mse", "mae", "rmsle"]}.get(cat, ["mse"])
        if key in cols:
            cols.remove(key)
        cols = [key] + cols
        lb = self.leaderboard_frame
        rows = []
        for m in self.models:
            if lb is not None:
                perf = m.model_performance(lb)
                vals = {c: _metric_of_dict(perf, c) for c in cols}
            else:
                vals = {c: _metric_of(m, c) for c in cols}
            rows.append(dict(model_id=m.key, **vals))
        desc = key in _DESC
        rows.sort(key=lambda r: (math.isnan(r[key]), -r[key] if desc else r[key]))
        return rows, ["model_id"] + cols

    @property
    def leader(self):
        rows, _ = self.leaderboard_rows()
        return dkv.get(rows[0]["model_id"]) if rows else None


def _metric_of_dict(perf, metric):
    key = {"auc": "AUC", "aucpr": "pr_auc", "logloss": "logloss", "mse": "MSE", "rmse": "RMSE", "mae": "mae",
           "rmsle": "rmsle", "mean_per_class_error": "mean_per_class_error",
           "mean_residual_deviance": "mean_residual_deviance"}.get(metric, metric)
    v = perf.get(key) if perf else None
    if v is None and key == "mean_residual_deviance" and perf:
        v = perf.get("MSE")
    return float("nan") if v is None else float(v)


def leaderboard_frame(models, frame=None, sort_metric="AUTO"):
    """``makeLeaderboard`` (h2o-automl ``Leaderboard.java``): rank arbitrary models on a frame (or their
    own training/cross-validation metrics) with the AutoML leaderboard columns."""
    import numpy as np
    import torch
    from .frame import Column, H2OFrame, engine_device
    lb = AutoML.__new__(AutoML)
    lb.models = list(models)
    lb.sort_metric = sort_metric
    lb.leaderboard_frame = frame
    rows, cols = lb.leaderboard_rows()
    out = [Column("model_id", "string", strings=np.array([r["model_id"] for r in rows], dtype=object))]
    for c in cols[1:]:
        out.append(Column(c, "real", torch.tensor([r[c] for r in rows], dtype=torch.float64, device=engine_device())))
    return H2OFrame._from_columns(out)
