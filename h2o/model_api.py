"""The trained-model surface of h2o-py's ``ModelBase`` and its model extensions (reference:
``h2o-py/h2o/model/model_base.py``, ``h2o-py/h2o/model/extensions/*.py``) on the in-process estimators.

Metric accessors follow the reference convention: with one of ``train`` / ``valid`` / ``xval`` (or none:
training) they return the value, with several a dict keyed ``train`` / ``valid`` / ``xval``. Everything is
read from the trained model's output or computed on device by the engine (permutation importance,
feature frequencies, predicted-vs-actual, row-to-tree assignment); plots use matplotlib (headless Agg).
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

_SRC = (("train", "training_metrics"), ("valid", "validation_metrics"), ("xval", "cross_validation_metrics"))


def _pick(model, key, train, valid, xval):
    want = [s for s, on in zip(("train", "valid", "xval"), (train, valid, xval)) if on] or ["train"]
    out = {}
    for s, src in _SRC:
        if s in want:
            m = model.output.get(src) or {}
            out[s] = m.get(key) if hasattr(m, "get") else None
    return out[want[0]] if len(want) == 1 else out


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


class ModelBaseAPI:
    """Mixin of :class:`h2o.estimators.estimator_base.H2OEstimator` (needs ``self._m()``)."""

    # ---- identity / bookkeeping -------------------------------------------------------------------
    @property
    def type(self):
        cat = self._m().model_category
        return {"Binomial": "classifier", "Multinomial": "classifier", "Ordinal": "classifier",
                "Regression": "regressor"}.get(cat, "unsupervised")

    @property
    def default_params(self):
        from llama_github_io_amd.models import builder
        spec = builder.REGISTRY.get(self.algo)
        return dict(spec.defaults) if spec is not None else {}

    @property
    def full_parameters(self):
        d = self.default_params
        act = self._m().params
        return {k: {"default_value": d.get(k), "actual_value": v} for k, v in {**d, **act}.items()}

    @property
    def start_time(self):
        return int(self._m().output.get("start_time") or 0)

    @property
    def end_time(self):
        o = self._m().output
        return int(o.get("end_time") or (o.get("start_time") or 0) + (o.get("run_time_ms") or 0))

    @property
    def run_time(self):
        return int(self._m().output.get("run_time_ms") or 0)

    def join(self):
        """Training is synchronous in process: the model is complete when ``train`` returns."""
        return self

    def detach(self):
        """Drop the local reference to the backend model (the model stays in the DKV)."""
        object.__setattr__(self, "_model", None)

    def have_mojo(self):
        from llama_github_io_amd.mojo import writer
        return getattr(writer, "supports_mojo", lambda m: True)(self._m())

    def have_pojo(self):
        from llama_github_io_amd.mojo import pojo
        return getattr(pojo, "supports_pojo", lambda m: True)(self._m())

    def save_model_details(self, path="", force=False, filename=None):
        """JSON model details (``/3/Models/<id>`` payload) written next to ``path``."""
        import json
        import os
        from llama_github_io_amd.models.base import _jsonable
        m = self._m()
        fn = os.path.join(path or ".", filename or f"{m.key}.json")
        if os.path.exists(fn) and not force:
            raise FileExistsError(fn)
        with open(fn, "w") as f:
            json.dump(dict(model_id=m.key, algo=m.algo, parameters=_jsonable(m.params), output=_jsonable(m.output)), f)
        return fn

    # ---- summaries --------------------------------------------------------------------------------
    def summary(self):
        o = self._m().output
        return o.get("model_summary") or {k: o.get(k) for k in ("ntrees", "epochs", "iterations", "number_of_trees")
                                          if o.get(k) is not None}

    get_summary = summary

    def show_summary(self):
        print(self.summary())

    def show(self, verbose=False, fmt=None):
        m = self._m()
        print(f"Model Details\n=============\n{type(self).__name__} : {m.algo}\nModel Key: {m.key}\n")
        print(self.summary())
        for s, src in _SRC:
            if m.output.get(src):
                print(f"\nModelMetrics ({s}): {m.output[src]!r}")

    def training_model_metrics(self):
        return self._m().output.get("training_metrics")

    def score_history(self):
        import pandas as pd
        return pd.DataFrame(self._m().output.get("scoring_history") or [])

    def scoring_history_plot(self, timestep="AUTO", metric="AUTO", save_plot_path=None, **kw):
        sh = self.score_history()
        plt = _plt()
        fig, ax = plt.subplots()
        cols = [c for c in sh.columns if c.startswith("training_") or c.startswith("validation_")]
        if metric != "AUTO":
            cols = [c for c in cols if c.endswith(str(metric).lower())]
        x = sh.index if timestep == "AUTO" or timestep not in sh.columns else sh[timestep]
        for c in cols[:4]:
            ax.plot(x, sh[c], label=c)
        ax.legend()
        if save_plot_path:
            fig.savefig(save_plot_path)
        return fig

    # ---- metric accessors (train / valid / xval) -------------------------------------------------------
    def gini(self, train=False, valid=False, xval=False):
        return _pick(self._m(), "Gini", train, valid, xval)

    def pr_auc(self, train=False, valid=False, xval=False):
        return _pick(self._m(), "pr_auc", train, valid, xval)

    def mean_residual_deviance(self, train=False, valid=False, xval=False):
        return _pick(self._m(), "mean_residual_deviance", train, valid, xval)

    def rmsle(self, train=False, valid=False, xval=False):
        return _pick(self._m(), "rmsle", train, valid, xval)

    def _glm_stat(self, name, out_key, train, valid, xval):
        m = self._m()
        fn = getattr(type(m), name, None)
        if fn is not None:
            return fn(m, train, valid, xval) if name not in ("null_degrees_of_freedom", "residual_degrees_of_freedom") \
                else fn(m)
        v = _pick(m, out_key, train, valid, xval)
        return m.output.get(out_key) if v is None and not (valid or xval) else v

    def null_deviance(self, train=False, valid=False, xval=False):
        return self._glm_stat("null_deviance", "null_deviance", train, valid, xval)

    def residual_deviance(self, train=False, valid=False, xval=False):
        return self._glm_stat("residual_deviance", "residual_deviance", train, valid, xval)

    def null_degrees_of_freedom(self, train=False, valid=False, xval=False):
        return self._glm_stat("null_degrees_of_freedom", "null_degrees_of_freedom", train, valid, xval)

    def residual_degrees_of_freedom(self, train=False, valid=False, xval=False):
        return self._glm_stat("residual_degrees_of_freedom", "residual_degrees_of_freedom", train, valid, xval)

    def aic(self, train=False, valid=False, xval=False):
        m = self._m()
        v = _pick(m, "AIC", train, valid, xval)
        return m.output.get("aic") if v is None and not (valid or xval) else v

    def loglikelihood(self, train=False, valid=False, xval=False):
        m = self._m()
        v = _pick(m, "loglikelihood", train, valid, xval)
        if v is None and not (valid or xval):
            v = m.output.get("loglikelihood", m.output.get("log_likelihood"))
        return v

    def negative_log_likelihood(self):
        ll = self.loglikelihood()
        return None if ll is None else -ll

    def average_objective(self):
        o = self._m().output
        return o.get("average_objective", o.get("objective"))

    # ---- coefficient family (GLM / GAM / CoxPH / HGLM ...) ----------------------------------------------
    def _coef_out(self, key):
        m = self._m()
        if getattr(m, "glm", None) is not None and key not in m.output:
            m = m.glm
        c = m.output.get(key)
        if c is None:
            raise ValueError(f"{self.algo} models have no {key}")
        return dict(c)

    def coef(self):
        return self._coef_out("coefficients")

    def coef_norm(self):
        return self._coef_out("standardized_coefficients")

    def coef_with_p_values(self):
        import pandas as pd
        o = self._m().output
        if not o.get("p_values"):
            raise ValueError("p-values were not computed: train with compute_p_values=True")
        names = list(o["coefficients"])
        return pd.DataFrame(dict(names=names, coefficients=[o["coefficients"][n] for n in names],
                                 std_error=[o["std_errs"].get(n) for n in names],
                                 z_value=[o["z_values"].get(n) for n in names],
                                 p_value=[o["p_values"].get(n) for n in names],
                                 standardized_coefficients=[o.get("standardized_coefficients", {}).get(n) for n in names]))

    def pprint_coef(self):
        for k, v in sorted(self.coef().items(), key=lambda kv: -abs(kv[1])):
            print(f"{k}: {v}")

    def std_coef_plot(self, num_of_features=None, server=False, save_plot_path=None):
        c = self.coef_norm()
        items = sorted(((k, v) for k, v in c.items() if k != "Intercept"), key=lambda kv: -abs(kv[1]))
        items = items[: num_of_features or len(items)]
        plt = _plt()
        fig, ax = plt.subplots()
        ax.barh([k for k, _ in items][::-1], [abs(v) for _, v in items][::-1],
                color=["tab:blue" if v >= 0 else "tab:orange" for _, v in items][::-1])
        ax.set_title("Standardized Coef. Magnitudes")
        if save_plot_path:
            fig.savefig(save_plot_path)
        return fig

    def get_variable_inflation_factors(self):
        v = self._m().output.get("variable_inflation_factors")
        if v is None:
            raise ValueError("variable inflation factors were not computed: train with generate_variable_inflation_factors=True")
        return dict(v)

    # ---- DeepLearning / PCA internals ---------------------------------------------------------------
    def _dl(self):
        m = self._m()
        if getattr(m, "net", None) is None:
            raise ValueError(f"{self.algo} models have no network")
        return m

    def deepfeatures(self, test_data, layer):
        """Hidden layer ``layer`` (0-based index, or the layer name) of a DeepLearning model on ``test_data``
        (model_base.py deepfeatures: /4/Predictions deep_features_hidden_layer)."""
        if test_data is None:
            raise ValueError("Must specify test data")
        m = self._dl()
        if not str(layer).isdigit():
            names = [f"hidden_{i}" for i in range(len(list(m.net.hidden)))]
            if layer not in names:
                raise ValueError(f"unknown hidden layer {layer!r} (one of {names})")
            layer = names.index(layer)
        return m.deepfeatures(test_data, int(layer))

    def biases(self, vector_id=0):
        from llama_github_io_amd.frame import H2OFrame
        m = self._dl()
        lins = list(m.net.hidden) + [m.net.out]
        return H2OFrame.from_tensor(lins[vector_id].bias.detach().double().reshape(-1, 1), [f"C{1}"])

    def normmul(self):
        ex = self._dl().expander
        return (1.0 / ex.num_sd).cpu().tolist() if getattr(ex, "num_sd", None) is not None else []

    def normsub(self):
        ex = self._dl().expander
        return ex.num_mean.cpu().tolist() if getattr(ex, "num_mean", None) is not None else []

    def respmul(self):
        m = self._dl()
        return [1.0 / float(m.resp_sd)] if m.model_category == "Regression" else []

    def respsub(self):
        m = self._dl()
        return [float(m.resp_mu)] if m.model_category == "Regression" else []

    def catoffsets(self):
        ex = self._dl().expander
        offs = list(getattr(ex, "cat_offsets", []) or [])
        return offs + [getattr(ex, "num_off", 0)]

    def rotation(self):
        m = self._m()
        ev = m.output.get("eigenvectors")
        if ev is None:
            raise ValueError(f"{self.algo} models have no rotation")
        import pandas as pd
        vecs = np.asarray(ev["vectors"] if isinstance(ev, dict) else ev)
        return pd.DataFrame(vecs, index=ev.get("names") if isinstance(ev, dict) else None,
                            columns=[f"pc{i + 1}" for i in range(vecs.shape[1])])

    # ---- trees ------------------------------------------------------------------------------------
    def _forest(self):
        m = self._m()
        fr = getattr(m, "forest", None)
        if fr is None:
            raise ValueError(f"{self.algo} models have no trees")
        return m, fr

    @property
    def ntrees_actual(self):
        m = self._m()
        if getattr(m, "forest", None) is not None:
            return int(m.output.get("ntrees") or len(m.forest.trees) // max(1, m.forest.K))
        return int(m.output.get("ntrees") or 0)

    def feature_frequencies(self, test_data):
        """Per row and feature: how many tree nodes on the row's prediction paths split on the feature
        (``Model.FeatureFrequencies``)."""
        from llama_github_io_amd.frame import H2OFrame
        m, fr = self._forest()
        frame = m._adapt(test_data)
        X, _ = frame.model_matrix(m.info, device=m.device)
        Xh = X.double().cpu().numpy()
        N, F = Xh.shape[1], Xh.shape[0]
        cnt = np.zeros((N, F))
        for tree in fr.trees:
            node = np.zeros(N, dtype=np.int64)
            for _ in range(256):
                feat = tree.feat[node]
                inner = feat >= 0
                if not inner.any():
                    break
                rows = np.nonzero(inner)[0]
                f = feat[rows]
                np.add.at(cnt, (rows, f), 1)
                x = Xh[f, rows]
                go_left = np.where(np.isnan(x), tree.na_left[node[rows]] != 0, x < tree.thr[node[rows]])
                if tree.is_cat is not None and tree.is_cat.any():
                    catm = tree.is_cat[node[rows]] != 0
                    for i in np.nonzero(catm)[0]:
                        nd = node[rows[i]]
                        bits = tree.cat_bits[nd]
                        v = x[i]
                        if not np.isnan(v) and bits is not None:
                            b = int(v)
                            go_left[i] = b < len(bits) * 32 and bool((int(bits[b >> 5]) >> (b & 31)) & 1)
                node[rows] = np.where(go_left, tree.left[node[rows]], tree.right[node[rows]])
        return H2OFrame.from_tensor(torch.as_tensor(cnt), list(m.info.x))

    def row_to_tree_assignment(self, original_training_data):
        """0/1 per (row, tree): the row was sampled into the tree's training set (the engine's row sampler
        is a function of the global row index and seed, so the assignment is recomputed exactly)."""
        from llama_github_io_amd.frame import H2OFrame
        from llama_github_io_amd.models.shared_tree import resolve_seed
        from llama_github_io_amd.parallel import collectives as coll
        m, fr = self._forest()
        rate = float(m.params.get("sample_rate", 1.0) or 1.0)
        seed = resolve_seed(m.params.get("seed", -1))
        N = original_training_data.nrows
        ntrees = self.ntrees_actual
        cols = [torch.ones(N, dtype=torch.float64) if rate >= 1.0 else
                (coll.row_uniform(seed, 1000 + t, 0, N, "cpu") < rate).double() for t in range(ntrees)]
        out = H2OFrame.from_tensor(torch.stack([torch.arange(N, dtype=torch.float64)] + cols, 1),
                                   ["row_id"] + [f"tree_{t + 1}" for t in range(ntrees)])
        return out

    # ---- cross-validation ---------------------------------------------------------------------------
    def is_cross_validated(self):
        return bool(self._m().output.get("cross_validation_models") or self._m().output.get("cross_validation_metrics"))

    def xval_keys(self):
        return list(self._m().output.get("cross_validation_models") or [])

    def get_xval_models(self, key=None):
        from llama_github_io_amd.core import dkv
        keys = self.xval_keys()
        if key is not None:
            return dkv.get(key) if key in keys else None
        return [dkv.get(k) for k in keys]

    @property
    def xvals(self):
        return self.get_xval_models()

    def cross_validation_fold_assignment(self):
        from llama_github_io_amd.core import dkv
        k = self._m().output.get("cross_validation_fold_assignment_frame_id")
        return dkv.get(k) if k else None

    def cross_validation_predictions(self):
        """Per fold model: its predictions on the training rows, zero outside its holdout fold."""
        from llama_github_io_amd.core import dkv
        m = self._m()
        ho = dkv.get(m.output.get("cross_validation_holdout_predictions_frame_id") or "")
        fa = self.cross_validation_fold_assignment()
        if ho is None or fa is None:
            raise ValueError("train with keep_cross_validation_predictions=True and "
                             "keep_cross_validation_fold_assignment=True")
        fold = fa._col(0).data.long()
        out = []
        from llama_github_io_amd.frame import Column, H2OFrame
        for i in range(len(self.xval_keys())):
            mask = (fold == i).to(fold.device)
            cols = []
            for c in ho._cols.values():
                if c.type == "enum":
                    cols.append(Column(c.name, c.type, torch.where(mask, c.data, torch.zeros_like(c.data)), c.domain))
                else:
                    cols.append(Column(c.name, c.type, torch.where(mask, c.data, torch.zeros_like(c.data))))
            out.append(H2OFrame._from_columns(cols))
        return out

    # ---- explanations ---------------------------------------------------------------------------------
    def varimp_plot(self, num_of_features=None, server=False, save_plot_path=None):
        vi = self._m().varimp()
        if not vi:
            raise ValueError(f"{self.algo} model has no variable importances")
        rows = [(r[0], r[2]) if isinstance(r, (list, tuple)) else (r["variable"], r["scaled_importance"]) for r in vi]
        rows = rows[: num_of_features or 10]
        plt = _plt()
        fig, ax = plt.subplots()
        ax.barh([r[0] for r in rows][::-1], [r[1] for r in rows][::-1])
        ax.set_title("Variable Importance: " + self.algo)
        if save_plot_path:
            fig.savefig(save_plot_path)
        return fig

    def permutation_importance(self, frame, metric="AUTO", n_samples=10000, n_repeats=1, features=None, seed=-1,
                               use_pandas=False):
        from llama_github_io_amd.rapids import _permutation_varimp
        fr = frame
        if n_samples and 0 < n_samples < frame.nrows:
            fr = frame.split_frame([n_samples / frame.nrows], seed=seed if seed >= 0 else 1)[0]
        out = _permutation_varimp(self._m(), fr, str(metric).upper() if metric != "AUTO" else "AUTO", n_repeats, seed)
        if features is not None:
            df = out.as_data_frame()
            df = df[df["Variable"].isin(list(features))]
            return df if use_pandas else df
        return out.as_data_frame() if use_pandas else out

    def permutation_importance_plot(self, frame, metric="AUTO", n_samples=10000, n_repeats=1, features=None,
                                    seed=-1, num_of_features=10, save_plot_path=None):
        df = self.permutation_importance(frame, metric, n_samples, n_repeats, features, seed, use_pandas=True)
        df = df.head(num_of_features)
        plt = _plt()
        fig, ax = plt.subplots()
        ax.barh(list(df["Variable"])[::-1], list(df["Scaled Importance"])[::-1])
        ax.set_title("Permutation Variable Importance")
        if save_plot_path:
            fig.savefig(save_plot_path)
        return fig

    def predicted_vs_actual_by_variable(self, frame, predicted, variable):
        """Per level of a categorical ``variable``: mean actual response and mean prediction
        (``PredictedVsActualByVariable``)."""
        import pandas as pd
        m = self._m()
        col = frame._col(variable)
        if col.type != "enum":
            raise ValueError("variable must be categorical")
        y = frame.response_tensor(m.info, device=m.device).double().cpu()
        p = predicted._col(predicted.names[-1] if m.model_category == "Binomial" else predicted.names[0]).as_float().double().cpu()
        codes = col.data.double().cpu()
        rows = []
        for k, lvl in enumerate(col.domain):
            sel = codes == k
            n = int(sel.sum())
            rows.append(dict(level=lvl, actual=float(y[sel].mean()) if n else math.nan,
                             predict=float(p[sel].mean()) if n else math.nan, count=n))
        return pd.DataFrame(rows)

    # ---- calibration / fairness ------------------------------------------------------------------------
    def calibrate(self, calibration_model):
        return self._m().set_calibration_model(getattr(calibration_model, "_model", calibration_model))

    def _fair(self, frame, protected_columns, reference=None, favorable_class=None):
        return self._m().fairness_metrics(frame, protected_columns, reference, favorable_class)

    def inspect_model_fairness(self, frame, protected_columns, reference, favorable_class, metrics=("auc", "aucpr",
                               "f1", "p.value", "selectedRatio", "total"), figsize=None, render=False):
        """Fairness report (h2o-py ``inspect_model_fairness``): the fairness metrics tables plus, when
        ``render``, the ROC / PR / PDP figures."""
        res = self._fair(frame, protected_columns, reference, favorable_class)
        if render:
            res["figures"] = [self.fair_roc_plot(frame, protected_columns, reference, favorable_class),
                              self.fair_pr_plot(frame, protected_columns, reference, favorable_class)]
        return res

    def _group_curves(self, frame, protected_columns, kind):
        m = self._m()
        if m.model_category != "Binomial":
            raise ValueError("Model has to be a binomial model!")
        pcs = [protected_columns] if isinstance(protected_columns, str) else list(protected_columns)
        pred = m.predict(frame)
        p1 = pred._col(pred.names[-1]).as_float().double().cpu().numpy()
        y = frame.response_tensor(m.info, device=m.device).double().cpu().numpy()
        keys = [tuple(frame._col(c).domain[int(v)] if frame._col(c).domain else v
                      for c, v in zip(pcs, vals)) for vals in zip(*[frame._col(c).as_float().cpu().numpy() for c in pcs])]
        curves = {}
        for g in sorted(set(keys), key=str):
            sel = np.array([k == g for k in keys])
            ps, ys = p1[sel], y[sel]
            order = np.argsort(-ps, kind="stable")
            tp = np.cumsum(ys[order] == 1)
            fp = np.cumsum(ys[order] == 0)
            P, Nn = max(tp[-1], 1), max(fp[-1], 1)
            curves[g] = (fp / Nn, tp / P) if kind == "roc" else (tp / P, tp / np.maximum(tp + fp, 1))
        return curves

    def fair_roc_plot(self, frame, protected_columns, reference, favorable_class, figsize=None, save_plot_path=None):
        plt = _plt()
        fig, ax = plt.subplots(figsize=figsize)
        for g, (x, yv) in self._group_curves(frame, protected_columns, "roc").items():
            ax.plot(x, yv, label=str(g))
        ax.set_xlabel("False Positive Rate")
        ax.set_ylabel("True Positive Rate")
        ax.legend()
        if save_plot_path:
            fig.savefig(save_plot_path)
        return fig

    def fair_pr_plot(self, frame, protected_columns, reference, favorable_class, figsize=None, save_plot_path=None):
        plt = _plt()
        fig, ax = plt.subplots(figsize=figsize)
        for g, (x, yv) in self._group_curves(frame, protected_columns, "pr").items():
            ax.plot(x, yv, label=str(g))
        ax.set_xlabel("Recall")
        ax.set_ylabel("Precision")
        ax.legend()
        if save_plot_path:
            fig.savefig(save_plot_path)
        return fig

    def fair_pd_plot(self, frame, column, protected_columns, figsize=None, autoscale=True, save_plot_path=None):
        """Partial dependence of ``column`` per protected group."""
        from llama_github_io_amd import explain
        m = self._m()
        pcs = [protected_columns] if isinstance(protected_columns, str) else list(protected_columns)
        plt = _plt()
        fig, ax = plt.subplots(figsize=figsize)
        col = frame._col(pcs[0])
        for k, lvl in enumerate(col.domain or []):
            sub = frame[frame[pcs[0]] == lvl]
            if sub.nrows == 0:
                continue
            pd_ = explain.partial_plot(m, sub, [column])[0]
            xs = pd_[column] if column in pd_ else pd_.iloc[:, 0]
            ax.plot(list(xs), list(pd_["mean_response"]), label=str(lvl))
        ax.set_xlabel(column)
        ax.legend()
        if save_plot_path:
            fig.savefig(save_plot_path)
        return fig

    def fair_shap_plot(self, frame, column, protected_columns, autoscale=True, figsize=None, jitter=0.35, alpha=1,
                       save_plot_path=None):
        """SHAP contribution of ``column`` against its value, coloured by protected group."""
        m = self._m()
        contrib = m.predict_contributions(frame)
        cvals = contrib._col(column).as_float().cpu().numpy()
        xv = frame._col(column).as_float().cpu().numpy()
        pcs = [protected_columns] if isinstance(protected_columns, str) else list(protected_columns)
        grp = frame._col(pcs[0])
        plt = _plt()
        fig, ax = plt.subplots(figsize=figsize)
        codes = grp.as_float().cpu().numpy()
        for k, lvl in enumerate(grp.domain or []):
            sel = codes == k
            ax.scatter(xv[sel], cvals[sel], s=4, alpha=alpha, label=str(lvl))
        ax.set_xlabel(column)
        ax.set_ylabel("SHAP contribution")
        ax.legend()
        if save_plot_path:
            fig.savefig(save_plot_path)
        return fig
