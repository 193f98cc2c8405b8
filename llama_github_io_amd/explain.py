"""Model explanation (reference: ``hex/genmodel/algos/tree/TreeSHAP.java`` + ``SharedTreeModel.
scoreContributions`` (predict_contributions), ``hex/PartialDependence.java`` (partial_plot),
``hex/tree/FriedmanPopescusH.java`` (h statistic), ``hex/FeatureInteractions*.java``).

* ``predict_contributions``: exact path-dependent TreeSHAP in the native runtime (``csrc/treeshap.cpp``,
  one thread per row range) over the flat forest; output columns = features + ``BiasTerm`` in the
  link (margin) space, summing to the raw prediction (GBM adds init_f, DRF averages trees).
* ``partial_plot``: for each grid value of a column (equally spaced over [min, max] / levels) the
  column is overwritten on device and the whole frame re-scored (one forest-kernel launch per grid
  point): mean, sd, std err; 2-D pairs, multinomial targets, ICE rows, weights.
* ``h``: Friedman–Popescu H² from centred partial dependences on the training rows.
* ``feature_interaction``: xgbfi statistics of split-feature paths (gain, F-score, weighted F-score,
  expected gain, ranks), leaf statistics and split-value histograms.
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


def _pdp_grid(col, nbins, user_splits, include_na):
    """PartialDependence.extractColValues: categorical -> every level; numeric -> ``nbins`` equally
    spaced values over [min, max] (unit steps for an integer column with fewer distinct values)."""
    if col.type == "enum":
        vals = [float(i) for i in range(len(col.domain))]
        labels = list(col.domain)
    elif user_splits is not None:
        vals = [float(v) for v in user_splits]
        labels = list(vals)
    else:
        v = col.as_float().double()
        v = v[~torch.isnan(v)]
        lo, hi = (float(v.min()), float(v.max())) if v.numel() else (0.0, 0.0)
        nb = int(nbins)
        if col.type == "int" and hi - lo + 1 < nb:
            nb = int(hi - lo + 1)
        delta = 0.0 if nb <= 1 else (hi - lo) / (nb - 1)
        vals = [lo + j * delta for j in range(max(nb, 1))]
        labels = list(vals)
    if include_na:
        vals.append(float("nan"))
        labels.append(".missing(NA)" if col.type == "enum" else float("nan"))
    return vals, labels


def partial_plot(model, frame, cols=None, nbins=20, targets=None, include_na=False, user_splits=None,
                 weight_column=None, row_index=-1, col_pairs_2dpdp=None):
    """Partial dependence (reference ``hex/PartialDependence.java``): for each grid value the column
    (or column pair) is overwritten on device for every row and the frame re-scored; mean, weighted
    standard deviation and standard error of the response. ``targets`` picks classes of a multinomial
    model (one table per column and class), ``row_index`` >= 0 gives an ICE curve of that row.
    Returns ``{name: [row dicts]}`` with name = column, ``"a|b"`` for pairs, ``"col|class"`` with targets."""
    m = getattr(model, "_model", model)
    cols = [] if cols is None else ([cols] if isinstance(cols, str) else list(cols))
    X, off = frame.model_matrix(m.info, device=m.device)
    w = None
    if weight_column is not None and weight_column != -1:
        wn = frame.names[weight_column] if isinstance(weight_column, int) else weight_column
        w = frame._col(wn).as_float().double().to(X.device)
    if row_index is not None and int(row_index) >= 0:
        X = X[:, int(row_index):int(row_index) + 1]
        off = None if off is None else off[int(row_index):int(row_index) + 1]
        w = None if w is None else w[int(row_index):int(row_index) + 1]
    dom = m.info.response_domain
    if m.model_category == "Multinomial":
        if not targets:
            raise ValueError("targets are required for a multinomial model's partial dependence")
        tidx = [(t, dom.index(t)) for t in targets]
    else:
        tidx = [(None, 1 if m.model_category == "Binomial" else 0)]
    user_splits = user_splits or {}

    def response(Xg, k):
        P = m.score_tensor(Xg, off)
        if P.dim() == 1:
            return P.double()
        return P[:, k].double() if m.model_category in ("Binomial", "Multinomial") else P[:, 0].double()

    def stats(r):
        if w is None:
            mu = float(r.mean())
            sd = float(r.std()) if r.numel() > 1 else 0.0
            return mu, sd, sd / math.sqrt(max(r.numel(), 1))
        ws = float(w.sum())
        mu = float((w * r).sum() / ws)
        sd = math.sqrt(float((w * (r - mu) ** 2).sum()) / max(ws - 1.0, 1e-300))
        return mu, sd, sd / math.sqrt(max(ws, 1e-300))

    out = {}
    jobs = [(c,) for c in cols] + [tuple(pr) for pr in (col_pairs_2dpdp or [])]
    for cc in jobs:
        js = [m.info.x.index(c) for c in cc]
        grids = [_pdp_grid(frame._col(c), nbins, user_splits.get(c), include_na) for c in cc]
        for tname, k in tidx:
            rows = []
            if len(cc) == 1:
                combos = [((v,), (lab,)) for v, lab in zip(*grids[0])]
            else:
                combos = [((v1, v2), (l1, l2)) for v1, l1 in zip(*grids[0]) for v2, l2 in zip(*grids[1])]
            for vals, labs in combos:
                Xg = X.clone()
                for j, v in zip(js, vals):
                    Xg[j] = float(v)
                mu, sd, se = stats(response(Xg, k))
                row = dict(value=labs[0], mean_response=mu, stddev_response=sd, std_error_mean_response=se)
                if len(cc) == 2:
                    row["value2"] = labs[1]
                rows.append(row)
            key = "|".join(cc) + (f"|{tname}" if tname is not None else "")
            out[key] = rows
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


class _FI:
    __slots__ = ("name", "depth", "gain", "cover", "fscore", "wfscore", "expected_gain", "tree_index", "tree_depth",
                 "has_leaf", "leaf_vl", "leaf_cl", "leaf_vr", "leaf_cr", "split_hist")

    def __init__(self, name, depth, gain, cover, proba, tree_depth, tree_index, split_value=None):
        self.name, self.depth, self.gain, self.cover = name, depth, gain, cover
        self.fscore, self.wfscore, self.expected_gain = 1.0, proba, gain * proba
        self.tree_index, self.tree_depth = float(tree_index), float(tree_depth)
        self.has_leaf, self.leaf_vl, self.leaf_cl, self.leaf_vr, self.leaf_cr = False, 0.0, 0.0, 0.0, 0.0
        self.split_hist = {}
        if depth == 0 and split_value is not None:
            self.split_hist[split_value] = 1


def feature_interaction(model, max_interaction_depth=100, max_tree_depth=100, max_deepening=-1):
    """xgbfi-style feature interactions (reference ``hex/FeatureInteractions.java``
    ``collectFeatureInteractions``): every path of split features (up to ``max_interaction_depth``+1
    features) accumulates gain, cover, an F-score, the path-probability weighted F-score and the
    expected gain; leaf statistics and split-value histograms of single features. Returns
    ``{"tables": [per-depth row dicts], "leaf_statistics": [...], "split_value_histograms": {name: {v: n}}}``;
    the legacy list view (``[{interaction, gain, fscore, cover, depth}]``) is under ``"flat"``."""
    m = getattr(model, "_model", model)
    names = m.info.x
    fis: dict = {}
    for ti, t in enumerate(m.forest.trees):
        memo: set = set()

        def split_value(n):
            return None if t.is_cat[n] else float(t.thr[n])

        def collect(n, path, cur_gain, cur_cover, proba, depth, deepening):
            if t.feat[n] < 0 or depth == max_tree_depth:
                return
            path = path + [n]
            cur_gain += float(max(t.gain[n], 0.0))
            cur_cover += float(t.cover[n])
            L, R = int(t.left[n]), int(t.right[n])
            cw = float(t.cover[n]) or 1.0
            ppl, ppr = proba * float(t.cover[L]) / cw, proba * float(t.cover[R]) / cw
            order = sorted(path, key=lambda q: names[int(t.feat[q])])
            name = "|".join(names[int(t.feat[q])] for q in order)
            if depth < max_deepening or max_deepening < 0:
                collect(L, [], 0.0, 0.0, ppl, depth + 1, deepening + 1)
                collect(R, [], 0.0, 0.0, ppr, depth + 1, deepening + 1)
            key = "-".join(str(q) for q in sorted(path))
            fi = fis.get(name)
            if fi is None:
                fis[name] = _FI(name, len(path) - 1, cur_gain, cur_cover, proba, depth, ti, split_value(path[0]))
                memo.add(key)
            else:
                if key in memo:
                    return
                memo.add(key)
                fi.gain += cur_gain
                fi.cover += cur_cover
                fi.fscore += 1
                fi.wfscore += proba
                fi.expected_gain += cur_gain * proba
                fi.tree_depth += depth
                fi.tree_index += ti
                if len(path) == 1 and split_value(path[0]) is not None:
                    sv = split_value(path[0])
                    fi.split_hist[sv] = fi.split_hist.get(sv, 0) + 1
            if len(path) - 1 == max_interaction_depth:
                return
            fi = fis[name]
            if t.feat[L] < 0 and deepening == 0:
                fi.leaf_vl += float(t.value[L])
                fi.leaf_cl += float(t.cover[L])
                fi.has_leaf = True
            if t.feat[R] < 0 and deepening == 0:
                fi.leaf_vr += float(t.value[R])
                fi.leaf_cr += float(t.cover[R])
                fi.has_leaf = True
            # the reference passes the running gain as the cover here as well
            collect(L, path, cur_gain, cur_gain, ppl, depth + 1, deepening)
            collect(R, path, cur_gain, cur_gain, ppr, depth + 1, deepening)

        if t.n_nodes:
            collect(0, [], 0.0, 0.0, 1.0, 0, 0)
    tables = []
    maxd = max((f.depth for f in fis.values()), default=-1)
    for d in range(maxd + 1):
        lst = [f for f in fis.values() if f.depth == d]

        def rank(key):
            srt = sorted(lst, key=lambda f: -key(f))
            return {f.name: i + 1 for i, f in enumerate(srt)}
        rk = [rank(lambda f: f.gain), rank(lambda f: f.fscore), rank(lambda f: f.wfscore),
              rank(lambda f: f.wfscore / f.fscore), rank(lambda f: f.gain / f.fscore), rank(lambda f: f.expected_gain)]
        rows = []
        for f in lst:
            r = [x[f.name] for x in rk]
            rows.append({"Interaction": f.name, "Gain": f.gain, "FScore": f.fscore, "wFScore": f.wfscore,
                         "Average wFScore": f.wfscore / f.fscore, "Average Gain": f.gain / f.fscore,
                         "Expected Gain": f.expected_gain, "Gain Rank": r[0], "FScore Rank": r[1],
                         "wFScore Rank": r[2], "Avg wFScore Rank": r[3], "Avg Gain Rank": r[4],
                         "Expected Gain Rank": r[5], "Average Rank": sum(r) / 6.0,
                         "Average Tree Index": f.tree_index / f.fscore, "Average Tree Depth": f.tree_depth / f.fscore})
        tables.append(rows)
    leaf = [{"Interaction": f.name, "Sum Leaf Values Left": f.leaf_vl, "Sum Leaf Values Right": f.leaf_vr,
             "Sum Leaf Covers Left": f.leaf_cl, "Sum Leaf Covers Right": f.leaf_cr} for f in fis.values() if f.has_leaf]
    hists = {f.name: dict(sorted(f.split_hist.items())) for f in fis.values() if f.depth == 0}
    flat = sorted(({"interaction": f.name, "gain": f.gain, "fscore": f.fscore, "cover": f.cover, "depth": f.depth + 1}
                   for f in fis.values()), key=lambda r: -r["gain"])
    return {"tables": tables, "leaf_statistics": leaf, "split_value_histograms": hists, "flat": flat}


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
