"""Model / ModelBuilder base classes (reference: ``hex/ModelBuilder.java``, ``hex/Model.java``,
``hex/ScoreKeeper.java`` early stopping, ``hex/CVModelBuilder.java`` cross-validation).

A model is trained from an :class:`~llama_github_io_amd.frame.H2OFrame` (or raw tensors), keeps a
``DataInfo`` describing how to turn any frame into the model's feature tensor (column order, domains,
categorical level remapping — ``Model.adaptTestForTrain``), and scores on the training device.
"""
from __future__ import annotations

import copy
import math
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import metrics as mm


# ------------------------------------------------------------------------------------------------
@dataclass
class DataInfo:
    x: list                         # predictor names (model order)
    iscat: np.ndarray               # int32 [F]
    domains: list                   # per predictor: list of levels or None
    response: str | None = None
    response_domain: list | None = None
    weights: str | None = None
    offset: str | None = None
    fold: str | None = None

    @property
    def F(self):
        return len(self.x)

    @property
    def nlevels(self):
        return np.array([len(d) if d is not None else 0 for d in self.domains], dtype=np.int32)

    def to_state(self):
        return dict(x=self.x, iscat=self.iscat.tolist(), domains=self.domains, response=self.response,
                    response_domain=self.response_domain, weights=self.weights, offset=self.offset, fold=self.fold)

    @staticmethod
    def from_state(s):
        return DataInfo(s["x"], np.asarray(s["iscat"], dtype=np.int32), s["domains"], s.get("response"),
                        s.get("response_domain"), s.get("weights"), s.get("offset"), s.get("fold"))


def default_device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def model_category(info: DataInfo, distribution: str | None = None) -> str:
    if info.response is None:
        return "Unsupervised"
    if info.response_domain is not None:
        return "Binomial" if len(info.response_domain) == 2 else "Multinomial"
    return "Regression"


# ------------------------------------------------------------------------------------------------
class ScoreKeeper:
    """Early stopping on a moving average of the stopping metric (``hex/ScoreKeeper.java``)."""

    LARGER_IS_BETTER = {"auc", "aucpr", "lift_top_group", "r2"}

    def __init__(self, stopping_rounds=0, stopping_metric="AUTO", stopping_tolerance=1e-3, category="Regression"):
        self.k = int(stopping_rounds)
        m = (stopping_metric or "AUTO").lower()
        if m == "auto":
            m = "logloss" if category in ("Binomial", "Multinomial") else "deviance"
        self.metric = m
        self.tol = float(stopping_tolerance)
        self.values = []

    def value_of(self, metrics: mm.ModelMetrics) -> float:
        m = self.metric
        key = {"logloss": "logloss", "mse": "MSE", "rmse": "RMSE", "mae": "mae", "rmsle": "rmsle", "auc": "AUC",
               "aucpr": "pr_auc", "deviance": "mean_residual_deviance", "misclassification": "mean_per_class_error",
               "mean_per_class_error": "mean_per_class_error", "r2": "r2"}.get(m, m)
        v = metrics.get(key)
        if v is None and key == "mean_residual_deviance":
            v = metrics.get("MSE")
        if v is None and key == "logloss":
            v = metrics.get("MSE")
        return float("nan") if v is None else float(v)

    def add(self, metrics) -> bool:
        """Record a scoring event; return True if training should stop."""
        self.values.append(self.value_of(metrics))
        k = self.k
        if k <= 0 or len(self.values) < 2 * k:
            return False
        v = np.asarray(self.values, dtype=np.float64)
        if np.isnan(v[-k:]).any():
            return False
        larger = self.metric in self.LARGER_IS_BETTER
        ma = np.convolve(v, np.ones(k) / k, mode="valid")
        last = ma[-1]
        ref = ma[:-k].max() if larger else ma[:-k].min()
        if larger:
            return not (last > ref * (1 + self.tol) if ref > 0 else last > ref + abs(ref) * self.tol)
        return not (last < ref * (1 - self.tol) if ref > 0 else last < ref - abs(ref) * self.tol)


# ------------------------------------------------------------------------------------------------
def rows_of(frame):
    """Context for row-wise work on ``frame``'s tensors: frames built inside carry its shard, and for a
    replicated frame under a multi-rank cloud nothing is all-reduced / gathered (every rank has all rows)."""
    import contextlib
    from ..parallel import collectives as coll, dframe
    stack = contextlib.ExitStack()
    sh = getattr(frame, "_shard", None)
    stack.enter_context(dframe.shard_ctx(sh))
    if sh is None and coll.world_active():
        stack.enter_context(coll.replicated())
    return stack


# ------------------------------------------------------------------------------------------------
_FRAME_METHODS = ("predict", "anomaly", "deepfeatures", "transform", "predict_rules", "reconstruct", "transform_frame",
                  "predict_leaf_node_assignment_frame", "staged_predict_proba_frame")


def _with_rows_of(fn):
    import functools

    @functools.wraps(fn)
    def w(self, frame, *a, **k):
        from ..frame import H2OFrame
        if not isinstance(frame, H2OFrame):
            return fn(self, frame, *a, **k)
        with rows_of(frame):
            return fn(self, self._adapt(frame), *a, **k)
    w._rows_of = True
    return w


class Model:
    """Trained model. Subclasses implement ``_predict_tensor(X [F,N] float32) -> [N] or [N,K]``.

    Frame-scoring methods (``predict``, ``anomaly``, ``transform``, ...) run under :func:`rows_of` for
    their input frame in every subclass: scoring is row-local, so a sharded frame is scored on its shard
    and the result frame is sharded the same way."""

    algo = "model"

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        for name in _FRAME_METHODS:
            fn = cls.__dict__.get(name)
            if fn is not None and callable(fn) and not getattr(fn, "_rows_of", False):
                setattr(cls, name, _with_rows_of(fn))

    def __init__(self, key: str, params: dict, info: DataInfo):
        self.key = key
        self.params = dict(params)
        self.info = info
        self.output = {"model_category": model_category(info), "scoring_history": [], "training_metrics": None,
                       "validation_metrics": None, "cross_validation_metrics": None, "variable_importances": None,
                       "run_time_ms": 0}
        self.device = default_device()

    # ---- category helpers
    @property
    def model_category(self) -> str:
        return self.output["model_category"]

    @property
    def nclasses(self) -> int:
        return len(self.info.response_domain) if self.info.response_domain else 1

    # ---- scoring
    def _predict_tensor(self, X: torch.Tensor, offset=None) -> torch.Tensor:
        raise NotImplementedError

    def score_tensor(self, X: torch.Tensor, offset=None) -> torch.Tensor:
        """Returns the prediction matrix: regression [N]; classification [N, K] probabilities."""
        P = self._predict_tensor(X.to(self.device), None if offset is None else offset.to(self.device))
        bal = self.output.get("model_class_distrib") if isinstance(self.output, dict) else None
        if bal and P.dim() == 2 and P.shape[1] == len(bal):
            from .adapt import correct_probabilities        # balance_classes: back to the prior distribution
            P = correct_probabilities(P, self.output["prior_class_distrib"], bal)
        return P

    def _adapt(self, frame):
        """Replay the model's preprocessors (AutoML target encoding: ``Model.Parameters._preprocessors``),
        then the training frame's categorical encoding / interaction columns (models/adapt.py)."""
        for pp in getattr(self, "preprocessors", None) or []:
            frame = pp.transform(frame)
        ad = getattr(self, "adapter", None)
        return ad.apply(frame) if ad else frame

    def predict(self, frame):
        from ..frame import H2OFrame
        frame = self._adapt(frame)
        with rows_of(frame):
            X, offset = frame.model_matrix(self.info, device=self.device)
            P = self.score_tensor(X, offset)
            out = H2OFrame.from_predictions(P, self.model_category, self.info.response_domain,
                                            threshold=self.default_threshold(), names=self.prediction_names(),
                                            labels=self.predict_labels(P))
            cm = getattr(self, "calibration_model", None)
            if cm is not None and P.dim() == 2 and P.shape[1] == 2:
                out = out.cbind(self._calibrated(P))
        return out

    # ---- calibration (CalibrationHelper.OutputWithCalibration)
    def set_calibration_model(self, calibration_model):
        if self.model_category != "Binomial":
            raise ValueError(f"Models of type {self.algo} don't support calibration.")
        self.calibration_model = calibration_model
        self.output["calibration_model"] = getattr(calibration_model, "key", None)
        return "OK"

    def _calibrated(self, P):
        from ..frame import Column, H2OFrame
        cm = self.calibration_model
        if cm.algo == "isotonicregression":
            c1 = cm.score_tensor(P[:, 1:2].T.float().contiguous()).double().reshape(-1)
            c0 = 1 - c1
        else:
            C = cm.score_tensor(P[:, 0:1].T.float().contiguous()).double()
            c0, c1 = C[:, 0], C[:, 1]
        return H2OFrame._from_columns([Column("cal_p0", "real", c0.contiguous()), Column("cal_p1", "real", c1.contiguous())])

    def prediction_names(self):
        """Column names of a multi-column non-classification prediction frame (None = defaults)."""
        return None

    def predict_labels(self, P):
        """Predicted classes when the model's rule is not argmax of the class probabilities (None = argmax)."""
        return None

    def default_threshold(self):
        tm = self.output.get("training_metrics") or {}
        vm = self.output.get("validation_metrics") or {}
        return (vm or tm).get("max_f1_threshold", 0.5) if self.model_category == "Binomial" else None

    def metrics_for(self, X, y, w=None, offset=None):
        P = self.score_tensor(X, offset)
        cat = self.model_category
        if cat in ("Binomial", "Multinomial", "Regression"):
            return mm.make_metrics(cat, y.to(P.device), P, None if w is None else w.to(P.device),
                                   self.info.response_domain, getattr(self, "distribution", None),
                                   labels=self.predict_labels(P))
        return None

    def model_performance(self, test_data=None, train=False, valid=False, xval=False):
        if test_data is None:
            if valid:
                return self.output.get("validation_metrics")
            if xval:
                return self.output.get("cross_validation_metrics")
            return self.output.get("training_metrics")
        test_data = self._adapt(test_data)
        with rows_of(test_data):
            X, offset = test_data.model_matrix(self.info, device=self.device)
            y = test_data.response_tensor(self.info, device=self.device)
            w = test_data.weights_tensor(self.info, device=self.device)
            return self.metrics_for(X, y, w, offset)

    # ---- H2O-python style accessors
    def varimp(self, use_pandas=False):
        vi = self.output.get("variable_importances")
        if vi is None:
            return None
        if use_pandas:
            import pandas as pd
            return pd.DataFrame(vi, columns=["variable", "relative_importance", "scaled_importance", "percentage"])
        return vi

    def scoring_history(self):
        return self.output.get("scoring_history")

    # ---- explanation (explain.py)
    def predict_contributions(self, test_data, output_format="Original", top_n=None, bottom_n=None, compare_abs=False):
        from .. import explain
        return explain.predict_contributions(self, test_data, output_format, top_n, bottom_n, compare_abs)

    def partial_plot(self, data, cols=None, nbins=20, plot=False, targets=None, include_na=False, user_splits=None,
                     **kw):
        from .. import explain
        return explain.partial_plot(self, data, cols, nbins, targets, include_na, user_splits,
                                    weight_column=kw.get("weight_column"), row_index=kw.get("row_index", -1),
                                    col_pairs_2dpdp=kw.get("col_pairs_2dpdp"))

    def h(self, frame, variables):
        from .. import explain
        return explain.h(self, frame, variables)

    def feature_interaction(self, max_interaction_depth=100, max_tree_depth=100, max_deepening=-1):
        """List of tables as in h2o-py: one per interaction depth, the leaf statistics, then one split-value
        histogram per single feature (pandas DataFrames)."""
        import pandas as pd
        from .. import explain
        r = explain.feature_interaction(self, max_interaction_depth, max_tree_depth, max_deepening)
        out = [pd.DataFrame(t) for t in r["tables"]] + [pd.DataFrame(r["leaf_statistics"])]
        out += [pd.DataFrame({"Split Value": list(h), "Count": list(h.values())}) for h in r["split_value_histograms"].values()]
        return out

    def fairness_metrics(self, frame, protected_columns, reference=None, favorable_class=None):
        """Per protected-group metrics + adverse impact ratios (h2o-py ``model.fairness_metrics``)."""
        from ..rapids_more import fairness_metrics
        fav = favorable_class if favorable_class is not None else self.info.response_domain[-1]
        return fairness_metrics(self, frame, protected_columns, reference, fav)

    def explain(self, frame, **kw):
        from .. import explain
        return explain.explain(self, frame, **kw)

    def _m(self, name, train, valid, xval):
        src = "validation_metrics" if valid else ("cross_validation_metrics" if xval else "training_metrics")
        m = self.output.get(src) or {}
        return m.get(name)

    # ---- h2o-py model-level metric delegation (model/models/binomial.py, multinomial.py: _delegate_to_metrics):
    # the training metrics unless train / valid / xval pick others; several picked -> {"train": .., "valid": ..}
    def _delegate(self, method, *args, train=False, valid=False, xval=False, **kw):
        from .. import metrics as _mm
        if not (train or valid or xval):
            train = True
        sel = [(k, src) for k, src, on in (("train", "training_metrics", train), ("valid", "validation_metrics", valid),
                                          ("xval", "cross_validation_metrics", xval)) if on]
        res = {}
        for k, src in sel:
            m = self.output.get(src)
            if m is not None and not isinstance(m, _mm.ModelMetrics):
                m = _mm.ModelMetrics(m)
            res[k] = getattr(m, method)(*args, **kw) if m is not None else None
        return next(iter(res.values())) if len(res) == 1 else res

    def F1(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("F1", thresholds, train=train, valid=valid, xval=xval)

    def F2(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("F2", thresholds, train=train, valid=valid, xval=xval)

    def F0point5(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("F0point5", thresholds, train=train, valid=valid, xval=xval)

    def accuracy(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("accuracy", thresholds, train=train, valid=valid, xval=xval)

    def error(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("error", thresholds, train=train, valid=valid, xval=xval)

    def precision(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("precision", thresholds, train=train, valid=valid, xval=xval)

    def recall(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("recall", thresholds, train=train, valid=valid, xval=xval)

    def sensitivity(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("sensitivity", thresholds, train=train, valid=valid, xval=xval)

    def specificity(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("specificity", thresholds, train=train, valid=valid, xval=xval)

    def tpr(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("tpr", thresholds, train=train, valid=valid, xval=xval)

    def tnr(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("tnr", thresholds, train=train, valid=valid, xval=xval)

    def fpr(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("fpr", thresholds, train=train, valid=valid, xval=xval)

    def fnr(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("fnr", thresholds, train=train, valid=valid, xval=xval)

    def fallout(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("fallout", thresholds, train=train, valid=valid, xval=xval)

    def missrate(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("missrate", thresholds, train=train, valid=valid, xval=xval)

    def mcc(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("mcc", thresholds, train=train, valid=valid, xval=xval)

    def max_per_class_error(self, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("max_per_class_error", thresholds, train=train, valid=valid, xval=xval)

    def mean_per_class_error(self, train=False, valid=False, xval=False):
        return self._m("mean_per_class_error", train, valid, xval)

    def metric(self, metric, thresholds=None, train=False, valid=False, xval=False):
        return self._delegate("metric", metric, thresholds, train=train, valid=valid, xval=xval)

    def find_threshold_by_max_metric(self, metric, train=False, valid=False, xval=False):
        return self._delegate("find_threshold_by_max_metric", metric, train=train, valid=valid, xval=xval)

    def find_idx_by_threshold(self, threshold, train=False, valid=False, xval=False):
        return self._delegate("find_idx_by_threshold", threshold, train=train, valid=valid, xval=xval)

    def confusion_matrix(self, metrics=None, thresholds=None, train=False, valid=False, xval=False):
        if metrics is not None and hasattr(metrics, "model_matrix"):      # h2o-py: confusion_matrix(frame)
            return self.model_performance(metrics).confusion_matrix()
        return self._delegate("confusion_matrix", metrics, thresholds, train=train, valid=valid, xval=xval)

    def roc(self, train=False, valid=False, xval=False):
        return self._delegate("roc", train=train, valid=valid, xval=xval)

    def gains_lift(self, train=False, valid=False, xval=False):
        return self._delegate("gains_lift", train=train, valid=valid, xval=xval)

    def gains_lift_plot(self, type="both", server=False, save_plot_path=None, plot=True):
        return self._delegate("plot", "gainslift", server, save_plot_path, plot)

    def plot(self, timestep="AUTO", metric="AUTO", server=False, save_plot_path=None, **kw):
        """Binomial: the ROC curve of the training metrics (h2o-py plots the scoring history for other models)."""
        return self._delegate("plot", "roc", server, save_plot_path)

    def kolmogorov_smirnov(self, train=False, valid=False, xval=False):
        """max |TPR - FPR| over the threshold table (the gains/lift table's K-S statistic)."""
        def ks(roc):
            if roc is None:
                return None
            f, t = roc
            return max((abs(y - x) for x, y in zip(f, t)), default=None)
        r = self.roc(train=train, valid=valid, xval=xval)
        return {k: ks(v) for k, v in r.items()} if isinstance(r, dict) else ks(r)

    def hit_ratio_table(self, train=False, valid=False, xval=False):
        return self._m("hit_ratio_table", train, valid, xval) or self._m("hit_ratios", train, valid, xval)

    def multinomial_auc_table(self, train=False, valid=False, xval=False):
        return self._m("multinomial_auc_table", train, valid, xval)

    def multinomial_aucpr_table(self, train=False, valid=False, xval=False):
        return self._m("multinomial_aucpr_table", train, valid, xval)

    def auc(self, train=False, valid=False, xval=False): return self._m("AUC", train, valid, xval)
    def aucpr(self, train=False, valid=False, xval=False): return self._m("pr_auc", train, valid, xval)
    def logloss(self, train=False, valid=False, xval=False): return self._m("logloss", train, valid, xval)
    def mse(self, train=False, valid=False, xval=False): return self._m("MSE", train, valid, xval)
    def rmse(self, train=False, valid=False, xval=False): return self._m("RMSE", train, valid, xval)
    def mae(self, train=False, valid=False, xval=False): return self._m("mae", train, valid, xval)
    def r2(self, train=False, valid=False, xval=False): return self._m("r2", train, valid, xval)

    # ---- persistence
    def to_state(self) -> dict:
        st = dict(algo=self.algo, key=self.key, params=_jsonable(self.params), info=self.info.to_state(),
                  output=_jsonable(self.output))
        cm = getattr(self, "calibration_model", None)
        if cm is not None:
            cs = cm.to_state()
            cs["__class__"] = type(cm).__module__ + ":" + type(cm).__name__
            st["calibration"] = cs
        ad = getattr(self, "adapter", None)
        if ad:
            st["adapter"] = ad.to_state()
        pps = getattr(self, "preprocessors", None)
        if pps:
            st["preprocessors"] = [pp.to_state() | {"__class__": type(pp).__module__ + ":" + type(pp).__name__}
                                   for pp in pps]
        return st

    def _restore(self, state):
        self.output = state["output"]
        if state.get("adapter"):
            from .adapt import FrameAdapter
            self.adapter = FrameAdapter.from_state(state["adapter"])
        if state.get("calibration"):
            from ..persist import _from_state
            self.calibration_model = _from_state(dict(state["calibration"]))
        if state.get("preprocessors"):
            from ..persist import _from_state
            self.preprocessors = [_from_state(dict(pp)) for pp in state["preprocessors"]]

    def __repr__(self):
        return f"<{type(self).__name__} key={self.key} category={self.model_category}>"


def _jsonable(o):
    if isinstance(o, dict):
        return {k: _jsonable(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_jsonable(v) for v in o]
    if isinstance(o, np.ndarray):
        return o.tolist()
    if isinstance(o, (np.floating, np.integer)):
        return o.item()
    if isinstance(o, torch.Tensor):
        return o.detach().cpu().tolist()
    return o


def variable_importance(names, gains) -> list:
    g = np.asarray(gains, dtype=np.float64)
    order = np.argsort(-g, kind="stable")
    mx = g.max() if g.size and g.max() > 0 else 1.0
    tot = g.sum() if g.sum() > 0 else 1.0
    return [(names[i], float(g[i]), float(g[i] / mx), float(g[i] / tot)) for i in order]


_key_counter = [0]


def make_key(algo: str) -> str:
    from ..api import cloud            # REST cloud task: the same model key on every rank
    k = cloud.task_key(f"{algo.upper()}_model") if cloud.active() else None
    if k:
        return k
    _key_counter[0] += 1
    return f"{algo.upper()}_model_{int(time.time() * 1000) % 10_000_000}_{_key_counter[0]}"
