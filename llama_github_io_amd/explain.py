"""Model explanation (reference: ``hex/genmodel/algos/tree/TreeSHAP.java`` + ``SharedTreeModel.
scoreContributions`` (predict_contributions), ``hex/PartialDependence.java`` (partial_plot),
``hex/tree/FriedmanPopescusH.java`` (h statistic), ``hex/FeatureInteractions*.java``).

* ``predict_contributions``: exact path-dependent TreeSHAP in the native runtime (``csrc/treeshap.cpp``,
  one thread per row range) over the flat forest; output columns = features + ``BiasTerm`` in the
  link (margin) space, summing to the raw prediction (GBM adds init_f, DRF averages trees).
* ``partial_plot``: for each grid value of a column (quantiles / levels) the column is overwritten on
  device and the whole frame re-scored (one forest-kernel launch per grid point): mean, sd, std err.
* ``h``: Friedman–Popescu H² from centred partial dependences on the training rows.
* ``feature_interaction``: gain / cover / split counts of feature pairs along tree paths.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from .frame import Column, H2OFrame


def _rt():
    from .ops import _native
    lib = _native.rt()
    if not getattr(lib, "_shap_bound", False):
        c = ctypes
        lib.h2o_treeshap.argtypes = [c.c_void_p, c.c_longlong, c.c_int, c.c_int, c.c_int] + [c.c_void_p] * 14 + [c.c_int]
        lib.h2o_treeshap.restype = c.c_int
        lib._shap_bound = True
    return lib


def tree_shap(forest, X: torch.Tensor, nthreads: int = 0) -> np.ndarray:
    """X [F, N] -> contributions [N, K, F+1] (float64, margin space, per-tree sums)."""
    fl = forest.flatten()
    cover = np.concatenate([t.cover.astype(np.float64) for t in forest.trees]) if forest.trees else np.zeros(1)
    depth = np.array([t.depth() for t in forest.trees], dtype=np.int32)
    Xr = np.ascontiguousarray(X.detach().float().cpu().numpy().T)
    N, F = Xr.shape
    K = forest.K
    out = np.zeros((N, K, F + 1), dtype=np.float64)
    arrs = [fl["roots"], fl["cls"], depth, fl["feat"], fl["thr"], fl["left"], fl["right"], fl["na_left"], fl["cat_off"],
            fl["cat_bits"], fl["cat_nbits"], fl["value"], cover]
    arrs = [np.ascontiguousarray(a) for a in arrs]
    _rt().h2o_treeshap(Xr.ctypes.data, N, F, K, len(forest.trees), *[a.ctypes.data for a in arrs], out.ctypes.data,
                       int(nthreads))
    return out


def predict_contributions(model, frame, output_format="Original", top_n=None, bottom_n=None, compare_abs=False):
    m = getattr(model, "_model", model)
    if not hasattr(m, "forest") or m.forest is None:
        raise NotImplementedError("predict_contributions is available for tree models (GBM, DRF, XGBoost)")
    X, _ = frame.model_matrix(m.info, device=torch.device("cpu"))
    phi = tree_shap(m.forest, X)
    if m.model_category == "Multinomial":
        raise NotImplementedError("contributions for multinomial models are not supported (as in H2O)")
    c = phi[:, 0, :]
    if m.algo == "drf":
        c = c / max(1, m.ntrees_built())
        if m.model_category == "Binomial" and not m.output.get("double_trees"):
            pass
    init = getattr(m, "init_f", 0.0)
    init = init[0] if isinstance(init, (list, tuple)) else init
    c[:, -1] += float(init or 0.0)
    names = list(m.info.x) + ["BiasTerm"]
    cols = [Column(n, "real", torch.as_tensor(c[:, i])) for i, n in enumerate(names)]
    return H2OFrame._from_columns(cols)


def partial_plot(model, frame, cols, nbins=20, targets=None, include_na=False, user_splits=None, weight_column=None):
    m = getattr(model, "_model", model)
    out = {}
    for col in ([cols] if isinstance(cols, str) else cols):
        j = m.info.x.index(col)
        X, off = frame.model_matrix(m.info, device=m.device)
        if m.info.iscat[j]:
            grid = list(range(len(m.info.domains[j])))
            labels = list(m.info.domains[j])
        else:
            if user_splits and col in user_splits:
                grid = [float(v) for v in user_splits[col]]
            else:
                v = X[j][~torch.isnan(X[j])].double()
                grid = torch.unique(torch.quantile(v[: 1 << 20], torch.linspace(0, 1, nbins, dtype=torch.float64,
                                                                                   device=v.device))).tolist()
            labels = grid
        if include_na:
            grid = grid + [float("nan")]
            labels = labels + ["NA"]
        rows = []
        for g, lab in zip(grid, labels):
            Xg = X.clone()
            Xg[j] = float(g)
            P = m.score_tensor(Xg, off)
            r = P[:, -1] if P.dim() == 2 and m.model_category == "Binomial" else (P if P.dim() == 1 else P[:, 0])
            r = r.double()
            rows.append(dict(value=lab, mean_response=float(r.mean()), stddev_response=float(r.std()),
                             std_error_mean_response=float(r.std() / math.sqrt(max(r.numel(), 1)))))
        out[col] = rows
    return out


def _pd_rows(m, X, off, cols, jidx):
    """Partial dependence of the columns ``cols`` evaluated AT each training row's own values."""
    N = X.shape[1]
    res = torch.zeros(N, dtype=torch.float64, device=X.device)
    vals = X[jidx].T  # [N, len]
    for i in range(N):
        Xg = X.clone()
        for k, j in enumerate(jidx):
            Xg[j] = vals[i, k]
        P = m.score_tensor(Xg, off)
        r = P[:, -1] if P.dim() == 2 else P
        res[i] = r.double().mean()
    return res - res.mean()


def h(model, frame, variables, max_rows=200):
    """Friedman–Popescu H² for the given variables (sample of ``max_rows`` rows, like the reference)."""
    m = getattr(model, "_model", model)
    X, off = frame.model_matrix(m.info, device=m.device)
    if X.shape[1] > max_rows:
        X = X[:, :max_rows]
        off = None if off is None else off[:max_rows]
    jidx = [m.info.x.index(v) for v in variables]
    f_joint = _pd_rows(m, X, off, variables, jidx)
    f_single = [_pd_rows(m, X, off, [v], [j]) for v, j in zip(variables, jidx)]
    num = ((f_joint - sum(f_single)) ** 2).sum()
    den = (f_joint ** 2).sum()
    return float(num / den) if den > 0 else float("nan")


def feature_interaction(model, max_interaction_depth=100, max_tree_depth=100, max_deepening=-1):
    m = getattr(model, "_model", model)
    names = m.info.x
    stats = {}
    for t in m.forest.trees:
        def walk(n, path, depth):
            if t.feat[n] < 0 or depth > max_tree_depth:
                return
            f = names[int(t.feat[n])]
            p2 = path + [f]
            key = "|".join(sorted(set(p2[-(max_interaction_depth + 1):])))
            s = stats.setdefault(key, dict(interaction=key, gain=0.0, fscore=0, cover=0.0, depth=len(set(p2))))
            s["gain"] += float(max(t.gain[n], 0))
            s["fscore"] += 1
            s["cover"] += float(t.cover[n])
            walk(int(t.left[n]), p2, depth + 1)
            walk(int(t.right[n]), p2, depth + 1)
        walk(0, [], 0)
    return sorted(stats.values(), key=lambda s: -s["gain"])


def explain(model, frame, columns=None, top_n_features=5):
    """Compact explanation bundle (the plotting-free part of ``h2o.explain``)."""
    m = getattr(model, "_model", model)
    vi = m.varimp() or []
    cols = columns or [r[0] for r in vi[:top_n_features]]
    res = dict(varimp=vi, pdp=partial_plot(m, frame, cols))
    if hasattr(m, "forest") and m.forest is not None and m.model_category in ("Binomial", "Regression"):
        sub = frame._rows(torch.arange(min(frame.nrows, 1000)))
        c = predict_contributions(m, sub).as_data_frame()
        res["shap_summary"] = c.abs().mean().sort_values(ascending=False).to_dict()
    return res
