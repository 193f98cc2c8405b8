"""Model explanation functions of h2o-py (``h2o-py/h2o/explanation/_explain.py``), computed on this engine.

Data first: every function builds the pandas table the reference plots (through the engine's TreeSHAP,
partial dependence, scoring history and metrics), then draws it with matplotlib if available.
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd


class Explanation:
    """One explanation: ``data`` (pandas) + a lazily drawn matplotlib figure."""

    def __init__(self, kind, data, draw=None, **meta):
        self.kind, self.data, self._draw, self.meta = kind, data, draw, meta
        self._fig = None

    def figure(self):
        if self._fig is None and self._draw is not None:
            try:
                import matplotlib
                matplotlib.use("Agg", force=False)
                import matplotlib.pyplot as plt
            except ImportError:      # pragma: no cover - matplotlib is optional
                return None
            self._fig = self._draw(plt)
        return self._fig

    def save(self, path):
        fig = self.figure()
        if fig is not None:
            fig.savefig(path)
        return path

    def __repr__(self):
        return f"<Explanation {self.kind}: {type(self.data).__name__}{getattr(self.data, 'shape', '')}>"


# ------------------------------------------------------------------------------------------------ helpers
def _model(m):
    return getattr(m, "_model", m)


def _models(models):
    """Models of an AutoML run, a leaderboard frame, a grid, a list, or a single model."""
    from llama_github_io_amd.core import dkv
    if hasattr(models, "leaderboard"):
        lb = models.leaderboard
        ids = lb.as_data_frame()["model_id"].tolist() if hasattr(lb, "as_data_frame") else [r["model_id"] for r in lb]
        return [_model(dkv.get(i)) for i in ids if dkv.get(i) is not None]
    if hasattr(models, "as_data_frame") and "model_id" in getattr(models, "names", []):
        return [_model(dkv.get(i)) for i in models.as_data_frame()["model_id"].tolist() if dkv.get(i) is not None]
    if hasattr(models, "models") and not callable(getattr(models, "models")):
        return [_model(m) for m in models.models]
    if isinstance(models, (list, tuple)):
        return [_model(m) for m in models]
    return [_model(models)]


def _varimp_dict(m):
    vi = m.varimp() or []
    out = {}
    xs = set(m.info.x)
    for r in vi:
        name, rel = r[0], float(r[1])
        if name not in xs and "." in name and name.split(".", 1)[0] in xs:
            name = name.split(".", 1)[0]          # one-hot expanded level -> its column (summed)
        out[name] = out.get(name, 0.0) + rel
    mx = max(out.values()) if out else 1.0
    return {k: (v / mx if mx > 0 else 0.0) for k, v in out.items()}


def _is_tree(m):
    return getattr(m, "forest", None) is not None and m.model_category in ("Binomial", "Regression")


def _predict_col(m, frame):
    p = m.predict(frame).as_data_frame()
    return p.iloc[:, 0]


# ------------------------------------------------------------------------------------------------ varimp
def varimp(models, num_of_features=20, cluster=True, use_pandas=True):
    """Scaled variable importance of each model (rows: variables, columns: models)."""
    ms = [m for m in _models(models) if m.varimp()]
    tab = pd.DataFrame({m.key: pd.Series(_varimp_dict(m)) for m in ms}).fillna(0.0)
    if tab.empty:
        return tab if use_pandas else tab.to_numpy()
    tab = tab.loc[tab.mean(1).sort_values(ascending=False).index]
    if num_of_features:
        tab = tab.iloc[:num_of_features]
    if cluster and tab.shape[1] > 2:
        order = np.argsort(np.argsort(-tab.to_numpy(), 0).mean(0))
        tab = tab.iloc[:, order]
    return tab if use_pandas else tab.to_numpy()


def varimp_heatmap(models, top_n=None, num_of_features=20, figsize=(16, 9), cluster=True, colormap="RdYlBu_r",
                   save_plot_path=None):
    ms = _models(models)
    if top_n:
        ms = ms[:top_n]
    tab = varimp(ms, num_of_features, cluster)

    def draw(plt):
        fig, ax = plt.subplots(figsize=figsize)
        im = ax.imshow(tab.to_numpy(), cmap=colormap, aspect="auto")
        ax.set_yticks(range(tab.shape[0]), tab.index)
        ax.set_xticks(range(tab.shape[1]), tab.columns, rotation=45, ha="right")
        fig.colorbar(im)
        ax.set_title("Variable Importance Heatmap")
        return fig
    e = Explanation("varimp_heatmap", tab, draw)
    if save_plot_path:
        e.save(save_plot_path)
    return e


# ------------------------------------------------------------------------------------------------ model correlation
def model_correlation(models, frame, cluster_models=True, use_pandas=True):
    """Prediction similarity between models: Pearson correlation of predictions (regression) or the
    fraction of rows with the same predicted class (classification)."""
    ms = _models(models)
    preds = {m.key: _predict_col(m, frame) for m in ms}
    keys = list(preds)
    n = len(keys)
    M = np.ones((n, n))
    for i in range(n):
        for j in range(i + 1, n):
            a, b = preds[keys[i]], preds[keys[j]]
            if a.dtype == object or str(a.dtype) == "category":
                v = float((a.astype(str) == b.astype(str)).mean())
            else:
                v = float(np.corrcoef(a.to_numpy(float), b.to_numpy(float))[0, 1])
            M[i, j] = M[j, i] = v
    tab = pd.DataFrame(M, index=keys, columns=keys)
    if cluster_models and n > 2:
        order = np.argsort(-M.mean(0))
        tab = tab.iloc[order, order]
    return tab if use_pandas else tab.to_numpy()


def model_correlation_heatmap(models, frame, top_n=None, cluster_models=True, triangular=True, figsize=(13, 13),
                              colormap="RdYlBu_r", save_plot_path=None):
    ms = _models(models)
    if top_n:
        ms = ms[:top_n]
    tab = model_correlation(ms, frame, cluster_models)

    def draw(plt):
        fig, ax = plt.subplots(figsize=figsize)
        M = tab.to_numpy().copy()
        if triangular:
            M[np.triu_indices_from(M, 1)] = np.nan
        im = ax.imshow(M, cmap=colormap, vmin=min(0.0, np.nanmin(M)), vmax=1.0)
        ax.set_xticks(range(len(tab)), tab.columns, rotation=45, ha="right")
        ax.set_yticks(range(len(tab)), tab.index)
        fig.colorbar(im)
        ax.set_title("Model Correlation")
        return fig
    e = Explanation("model_correlation_heatmap", tab, draw)
    if save_plot_path:
        e.save(save_plot_path)
    return e


# ------------------------------------------------------------------------------------------------ SHAP
def _contributions(m, frame, rows=None):
    sub = frame if rows is None else frame._rows(__import__("torch").as_tensor(rows))
    return m.predict_contributions(sub).as_data_frame()


def shap_summary_plot(model, frame, columns=None, top_n_features=20, samples=1000, colorize_factors=True, alpha=1,
                      colormap=None, figsize=(12, 12), jitter=0.35, save_plot_path=None):
    """TreeSHAP contributions of up to ``samples`` rows, long format (feature, contribution, normalized
    feature value), features ordered by mean |contribution|."""
    m = _model(model)
    n = frame.nrows
    rng = np.random.default_rng(42)
    rows = np.sort(rng.choice(n, min(samples, n), replace=False)) if n > samples else np.arange(n)
    c = _contributions(m, frame, rows)
    feats = [f for f in c.columns if f != "BiasTerm"]
    if columns:
        feats = [f for f in feats if f in columns]
    order = c[feats].abs().mean().sort_values(ascending=False).index[:top_n_features].tolist()
    X = frame.as_data_frame().iloc[rows]
    recs = []
    for f in order:
        xv = pd.to_numeric(X[f], errors="coerce") if f in X else pd.Series(np.nan, index=X.index)
        lo, hi = xv.min(), xv.max()
        nv = (xv - lo) / (hi - lo) if hi > lo else xv * 0
        for r, (cv, v) in enumerate(zip(c[f].to_numpy(), nv.to_numpy())):
            recs.append(dict(feature=f, row=int(rows[r]), contribution=float(cv), normalized_value=float(v)))
    tab = pd.DataFrame(recs)

    def draw(plt):
        fig, ax = plt.subplots(figsize=figsize)
        for i, f in enumerate(order):
            d = tab[tab.feature == f]
            y = len(order) - 1 - i + rng.uniform(-jitter, jitter, len(d))
            ax.scatter(d.contribution, y, c=d.normalized_value, cmap=colormap or "RdBu_r", alpha=alpha, s=6)
        ax.set_yticks(range(len(order)), order[::-1])
        ax.set_xlabel("SHAP value")
        ax.set_title(f"SHAP Summary plot for \"{m.key}\"")
        return fig
    e = Explanation("shap_summary", tab, draw)
    if save_plot_path:
        e.save(save_plot_path)
    return e


def shap_explain_row_plot(model, frame, row_index, columns=None, top_n_features=10, figsize=(16, 9),
                          plot_type="barplot", contribution_type="both", save_plot_path=None):
    m = _model(model)
    c = _contributions(m, frame, [int(row_index)]).iloc[0]
    bias = float(c.get("BiasTerm", 0.0))
    c = c.drop(labels=["BiasTerm"], errors="ignore")
    if columns:
        c = c[[f for f in c.index if f in columns]]
    if contribution_type == "positive":
        c = c[c > 0]
    elif contribution_type == "negative":
        c = c[c < 0]
    c = c.reindex(c.abs().sort_values(ascending=False).index)[:top_n_features]
    tab = pd.DataFrame({"feature": c.index, "contribution": c.to_numpy()})
    tab.attrs["bias"] = bias

    def draw(plt):
        fig, ax = plt.subplots(figsize=figsize)
        ax.barh(tab.feature[::-1], tab.contribution[::-1], color=["tab:red" if v > 0 else "tab:blue" for v in tab.contribution[::-1]])
        ax.set_title(f"SHAP explanation for \"{m.key}\" on row {row_index}")
        return fig
    e = Explanation("shap_explain_row", tab, draw, bias=bias)
    if save_plot_path:
        e.save(save_plot_path)
    return e


# ------------------------------------------------------------------------------------------------ PD / ICE
def _pd_table(m, frame, column, row_index=None, target=None, max_levels=30):
    from llama_github_io_amd import explain as ex
    targets = [target] if target is not None and m.model_category == "Multinomial" else None
    if m.model_category == "Multinomial" and targets is None:
        targets = [m.info.response_domain[0]]
    r = ex.partial_plot(m, frame, [column], nbins=20, targets=targets, row_index=-1 if row_index is None else row_index)
    rows = next(iter(r.values()))
    tab = pd.DataFrame(rows)
    return tab.iloc[:max_levels] if frame.type(column) == "enum" else tab


def pd_plot(model, frame, column, row_index=None, target=None, max_levels=30, figsize=(16, 9), colormap="Dark2",
            save_plot_path=None, binary_response_scale="response", **kw):
    m = _model(model)
    tab = _pd_table(m, frame, column, row_index, target, max_levels)
    if binary_response_scale == "logodds" and m.model_category == "Binomial":
        p = tab.mean_response.clip(1e-12, 1 - 1e-12)
        tab = tab.assign(mean_response=np.log(p / (1 - p)))

    def draw(plt):
        fig, ax = plt.subplots(figsize=figsize)
        ax.plot(range(len(tab)) if tab.value.dtype == object else tab.value, tab.mean_response)
        ax.set_xlabel(column)
        ax.set_ylabel("Mean Response")
        ax.set_title(f"Partial Dependence plot for \"{column}\"")
        return fig
    e = Explanation("pd_plot", tab, draw)
    if save_plot_path:
        e.save(save_plot_path)
    return e


def pd_multi_plot(models, frame, column, best_of_family=True, row_index=None, target=None, max_levels=30,
                  figsize=(16, 9), colormap="Dark2", markers=None, save_plot_path=None, **kw):
    ms = _models(models)
    if best_of_family:
        seen, keep = set(), []
        for m in ms:
            if m.algo not in seen:
                seen.add(m.algo)
                keep.append(m)
        ms = keep
    parts = []
    for m in ms:
        t = _pd_table(m, frame, column, row_index, target, max_levels)
        parts.append(t.assign(model_id=m.key))
    tab = pd.concat(parts, ignore_index=True) if parts else pd.DataFrame()

    def draw(plt):
        fig, ax = plt.subplots(figsize=figsize)
        for k, d in tab.groupby("model_id"):
            ax.plot(range(len(d)) if d.value.dtype == object else d.value, d.mean_response, label=k)
        ax.legend()
        ax.set_title(f"Partial Dependence plot for \"{column}\"")
        return fig
    e = Explanation("pd_multi_plot", tab, draw)
    if save_plot_path:
        e.save(save_plot_path)
    return e


def ice_plot(model, frame, column, target=None, max_levels=30, figsize=(16, 9), colormap="plasma",
             save_plot_path=None, show_pdp=True, binary_response_scale="response", centered=False, **kw):
    """ICE curves of the rows at the 0, 10, ..., 100th percentiles of the prediction (as the reference)."""
    m = _model(model)
    pred = _predict_col(m, frame) if m.model_category == "Regression" else m.predict(frame).as_data_frame().iloc[:, -1]
    pv = pred.to_numpy(float)
    order = np.argsort(pv, kind="stable")
    picks = sorted({int(order[min(len(order) - 1, int(round(q / 100 * (len(order) - 1))))]) for q in range(0, 101, 10)})
    parts = []
    for r in picks:
        t = _pd_table(m, frame, column, r, target, max_levels)
        if centered:
            t = t.assign(mean_response=t.mean_response - t.mean_response.iloc[0])
        pct = float((pv <= pv[r]).mean() * 100)
        parts.append(t.assign(row=r, percentile=round(pct)))
    tab = pd.concat(parts, ignore_index=True)
    pdp = _pd_table(m, frame, column, None, target, max_levels) if show_pdp else None

    def draw(plt):
        fig, ax = plt.subplots(figsize=figsize)
        for r, d in tab.groupby("row"):
            ax.plot(range(len(d)) if d.value.dtype == object else d.value, d.mean_response, alpha=0.7,
                    label=f"{int(d.percentile.iloc[0])}th percentile")
        if pdp is not None:
            ax.plot(range(len(pdp)) if pdp.value.dtype == object else pdp.value, pdp.mean_response, "k--",
                    label="Partial Dependence")
        ax.legend()
        ax.set_title(f"Individual Conditional Expectation for \"{column}\"")
        return fig
    e = Explanation("ice_plot", tab, draw, pdp=pdp)
    if save_plot_path:
        e.save(save_plot_path)
    return e


# ------------------------------------------------------------------------------------------------ residuals / learning curve
def residual_analysis_plot(model, frame, figsize=(16, 9), save_plot_path=None):
    m = _model(model)
    if m.model_category != "Regression":
        raise ValueError("residual analysis is available for regression models")
    y = pd.to_numeric(frame.as_data_frame()[m.info.response], errors="coerce").to_numpy(float)
    f = _predict_col(m, frame).to_numpy(float)
    tab = pd.DataFrame({"fitted": f, "residual": y - f})

    def draw(plt):
        fig, ax = plt.subplots(figsize=figsize)
        ax.scatter(tab.fitted, tab.residual, s=4, alpha=0.5)
        ax.axhline(0, color="k", lw=1)
        ax.set_xlabel("Fitted")
        ax.set_ylabel("Residuals")
        ax.set_title(f"Residual Analysis for \"{m.key}\"")
        return fig
    e = Explanation("residual_analysis", tab, draw)
    if save_plot_path:
        e.save(save_plot_path)
    return e


_LC_DEFAULT = {"Binomial": "logloss", "Multinomial": "logloss", "Regression": "deviance", "Ordinal": "logloss"}


def learning_curve_plot(model, metric="AUTO", cv_ribbon=None, cv_lines=None, figsize=(16, 9), colormap=None,
                        save_plot_path=None):
    """Scoring history of the model (training / validation metric per iteration, tree or epoch)."""
    m = _model(model)
    sh = m.output.get("scoring_history") or []
    tab = pd.DataFrame(sh if isinstance(sh, list) else [])
    met = (_LC_DEFAULT.get(m.model_category, "rmse") if str(metric).upper() == "AUTO" else str(metric)).lower()
    cols = [c for c in tab.columns if met in c.lower()]
    xcol = next((c for c in ("number_of_trees", "epochs", "iterations", "iteration", "lambda") if c in tab.columns), None)

    def draw(plt):
        fig, ax = plt.subplots(figsize=figsize)
        xs = tab[xcol] if xcol else range(len(tab))
        for c in cols:
            ax.plot(xs, tab[c], label=c)
        ax.set_xlabel(xcol or "scoring event")
        ax.set_ylabel(met)
        ax.legend()
        ax.set_title(f"Learning Curve for \"{m.key}\"")
        return fig
    e = Explanation("learning_curve", tab, draw, metric=met, columns=cols)
    if save_plot_path:
        e.save(save_plot_path)
    return e


# ------------------------------------------------------------------------------------------------ pareto front
def pareto_front(frame, x_metric=None, y_metric=None, optimum="top left", title=None, color_col="algo",
                 figsize=(16, 9), colormap="Dark2"):
    """Rows of a leaderboard-like table not dominated in (x_metric, y_metric) for the given optimum corner."""
    df = frame.as_data_frame() if hasattr(frame, "as_data_frame") else pd.DataFrame(frame)
    num = [c for c in df.columns if pd.api.types.is_numeric_dtype(df[c])]
    x_metric = x_metric or ("predict_time_per_row_ms" if "predict_time_per_row_ms" in df else num[-1])
    y_metric = y_metric or num[0]
    sx = -1 if "left" in optimum else 1     # want small x for "left"
    sy = 1 if "top" in optimum else -1      # want large y for "top"
    xs, ys = df[x_metric].to_numpy(float) * sx, df[y_metric].to_numpy(float) * sy
    keep = []
    for i in range(len(df)):
        dominated = np.any((xs >= xs[i]) & (ys >= ys[i]) & ((xs > xs[i]) | (ys > ys[i])))
        if not dominated:
            keep.append(i)
    front = df.iloc[keep].sort_values(x_metric)

    def draw(plt):
        fig, ax = plt.subplots(figsize=figsize)
        ax.scatter(df[x_metric], df[y_metric], alpha=0.5)
        ax.plot(front[x_metric], front[y_metric], "r-o")
        ax.set_xlabel(x_metric)
        ax.set_ylabel(y_metric)
        ax.set_title(title or "Pareto Front")
        return fig
    return Explanation("pareto_front", front, draw, x_metric=x_metric, y_metric=y_metric)


# ------------------------------------------------------------------------------------------------ fairness
def disparate_analysis(models, frame, protected_columns, reference, favorable_class, air_metric="selectedRatio",
                       alpha=0.05):
    """Per model: performance plus the min/max adverse impact ratio over the protected groups."""
    rows = []
    for m in _models(models):
        fm = m.fairness_metrics(frame, protected_columns, reference, favorable_class)
        ov = fm.get("overview") if isinstance(fm, dict) else None
        ovdf = pd.DataFrame(ov) if ov is not None else pd.DataFrame()
        col = f"AIR_{air_metric}"
        air = ovdf[col] if col in ovdf else pd.Series(dtype=float)
        tm = m.output.get("training_metrics") or {}
        rows.append(dict(model_id=m.key, auc=tm.get("AUC"), logloss=tm.get("logloss"),
                         air_min=float(air.min()) if len(air) else float("nan"),
                         air_max=float(air.max()) if len(air) else float("nan"),
                         cair=float((air - 1).abs().mean()) if len(air) else float("nan")))
    return pd.DataFrame(rows)


# ------------------------------------------------------------------------------------------------ bundles
_SINGLE = ("residual_analysis", "learning_curve", "varimp", "shap_summary", "pdp", "ice")
_MULTI = ("leaderboard", "varimp_heatmap", "model_correlation_heatmap", "pdp")


def _want(name, include, exclude):
    inc = [include] if isinstance(include, str) else list(include)
    exc = [exclude] if isinstance(exclude, str) else list(exclude)
    return ("ALL" in inc or name in inc) and name not in exc


def explain(models, frame, columns=None, top_n_features=5, include_explanations="ALL", exclude_explanations=(),
            plot_overrides=None, figsize=(16, 9), render=False, qualitative_colormap="Dark2",
            sequential_colormap="RdYlBu_r", background_frame=None):
    """H2OExplanation of one model or a group of models: a dict of :class:`Explanation` sections."""
    ms = _models(models)
    out = {}
    if len(ms) == 1:
        m = ms[0]
        vi = m.varimp() or []
        cols = list(columns) if columns else [r[0] for r in vi[:top_n_features]]
        if _want("residual_analysis", include_explanations, exclude_explanations) and m.model_category == "Regression":
            out["residual_analysis"] = residual_analysis_plot(m, frame)
        if _want("learning_curve", include_explanations, exclude_explanations) and m.output.get("scoring_history"):
            out["learning_curve"] = learning_curve_plot(m)
        if _want("varimp", include_explanations, exclude_explanations) and vi:
            out["varimp"] = Explanation("varimp", pd.DataFrame(vi, columns=["variable", "relative_importance",
                                                                              "scaled_importance", "percentage"]))
        if _want("shap_summary", include_explanations, exclude_explanations) and _is_tree(m):
            out["shap_summary"] = shap_summary_plot(m, frame)
        if _want("pdp", include_explanations, exclude_explanations):
            out["pdp"] = {c: pd_plot(m, frame, c) for c in cols}
        if _want("ice", include_explanations, exclude_explanations) and m.model_category in ("Regression", "Binomial"):
            out["ice"] = {c: ice_plot(m, frame, c) for c in cols}
        return out
    if _want("leaderboard", include_explanations, exclude_explanations):
        out["leaderboard"] = Explanation("leaderboard", pd.DataFrame(
            [dict(model_id=m.key, **{k: v for k, v in (m.output.get("training_metrics") or {}).items()
                                      if isinstance(v, (int, float))}) for m in ms]))
    if _want("varimp_heatmap", include_explanations, exclude_explanations):
        out["varimp_heatmap"] = varimp_heatmap(ms)
    if _want("model_correlation_heatmap", include_explanations, exclude_explanations):
        out["model_correlation_heatmap"] = model_correlation_heatmap(ms, frame)
    if _want("pdp", include_explanations, exclude_explanations):
        vt = varimp(ms, num_of_features=top_n_features)
        cols = list(columns) if columns else list(vt.index)
        out["pdp"] = {c: pd_multi_plot(ms, frame, c) for c in cols}
    return out


def explain_row(models, frame, row_index, columns=None, top_n_features=5, include_explanations="ALL",
                exclude_explanations=(), plot_overrides=None, qualitative_colormap="Dark2",
                figsize=(16, 9), render=False, background_frame=None):
    ms = _models(models)
    out = {}
    m = ms[0]
    vi = m.varimp() or []
    cols = list(columns) if columns else [r[0] for r in vi[:top_n_features]]
    if len(ms) == 1:
        if _want("shap_explain_row", include_explanations, exclude_explanations) and _is_tree(m):
            out["shap_explain_row"] = shap_explain_row_plot(m, frame, row_index)
        if _want("ice", include_explanations, exclude_explanations):
            out["ice"] = {c: pd_plot(m, frame, c, row_index=row_index) for c in cols}
        return out
    if _want("ice", include_explanations, exclude_explanations):
        out["ice"] = {c: pd_multi_plot(ms, frame, c, row_index=row_index) for c in cols}
    return out


def register_explain_methods():
    """Attach the per-model explanation methods to the estimator classes (``model.shap_summary_plot(...)``)."""
    from h2o.estimators.estimator_base import H2OEstimator
    for name, fn in (("shap_summary_plot", shap_summary_plot), ("shap_explain_row_plot", shap_explain_row_plot),
                     ("pd_plot", pd_plot), ("ice_plot", ice_plot), ("residual_analysis_plot", residual_analysis_plot),
                     ("learning_curve_plot", learning_curve_plot), ("explain_row", explain_row)):
        setattr(H2OEstimator, name, fn)
    H2OEstimator.explain = lambda self, frame, **kw: explain(self, frame, **kw)
