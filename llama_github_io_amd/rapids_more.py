"""The remaining Rapids primitives: lambdas (``{x . body}``) and the ops that take them (``ddply``,
``apply`` with a function), time-series iSAX, grouped permutation, fairness metrics, calibration /
tree-weight / rule model ops, and the small testing/internal hooks.

References: ``water/rapids/ast/AstFunction.java`` (lambdas), ``ast/prims/mungers/AstDdply.java``,
``AstGroupedPermute.java``, ``ast/prims/timeseries/AstIsax.java``, ``ast/prims/models/AstFairnessMetrics.java``,
``AstTestJavaScoring.java``, ``AstSegmentModelsAsFrame.java``, ``ast/prims/internal/AstRunTool.java``,
``ast/prims/testing/AstSetReadForbidden.java``, ``h2o-algos/.../rapids/prims/{AstPredictedVsActualByVar,
AstSetCalibrationModel, tree/AstTreeUpdateWeights, rulefit/AstPredictRule, word2vec/AstWord2VecToFrame,
isotonic/AstPoolAdjacentViolators}.java``.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .core import dkv
from .frame import Column, H2OFrame, engine_device

READ_FORBIDDEN: set = set()


class RapidsFunction:
    """A Rapids lambda bound to the session: calling it binds the parameters (frames / numbers) in a new
    scope and evaluates the body; 1x1 frame results come back as floats."""

    def __init__(self, sess, params, body):
        self.sess, self.params, self.body = sess, params, body

    def __call__(self, *args):
        vals = [_to_value(a) for a in args]
        self.sess.scopes.append(dict(zip(self.params, vals)))
        try:
            r = self.sess.eval_node(self.body)
        finally:
            self.sess.scopes.pop()
        return _scalar(r)


def _to_value(a):
    if isinstance(a, torch.Tensor):
        t = a.double().reshape(-1)
        return H2OFrame._from_columns([Column("C1", "real", t.to(engine_device()))])
    return a


def _scalar(r):
    if isinstance(r, H2OFrame) and r.nrows == 1 and r.ncols == 1:
        return float(r._col(0).as_float()[0])
    if isinstance(r, list) and len(r) == 1:
        return r[0]
    return r


def as_function(sess, f):
    """A Rapids function argument: a lambda, or the name of a primitive (``mean``, ``sum``, ...)."""
    if callable(f):
        return f
    if isinstance(f, str) and f in sess.prims:
        prim = sess.prims[f]
        return lambda *a: _scalar(prim(*[_to_value(x) for x in a]))
    raise TypeError(f"expected a function, got {f!r}")


# ------------------------------------------------------------------------------------------------ mungers
def ddply(sess, fr: H2OFrame, groupby, fun):
    """Split rows by the group columns, apply ``fun`` to each group's sub-frame, one result row per group
    (group keys + ``ddply_C1..``)."""
    from .rapids import _idx_list
    fn = as_function(sess, fun)
    gcols = [fr.names[i] for i in _idx_list(groupby, fr.ncols)]
    keys = torch.stack([fr._col(c).as_float() for c in gcols], 1).cpu().numpy()
    ukeys, inv = np.unique(np.nan_to_num(keys, nan=-np.inf), axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    rows = []
    for g in range(len(ukeys)):
        idx = torch.as_tensor(np.nonzero(inv == g)[0], device=fr._col(0).as_float().device)
        r = fn(H2OFrame._from_columns([fr._col(n).take(idx) for n in fr.names]))
        if isinstance(r, H2OFrame):
            if r.nrows != 1:
                raise ValueError(f"ddply must return a 1-row (many column) frame, found {r.nrows}")
            r = [float(v) for v in r.as_tensor(dtype=torch.float64)[0].tolist()]
        rows.append(list(np.atleast_1d(np.asarray(r, dtype=np.float64))))
    width = max(len(r) for r in rows) if rows else 1
    dev = engine_device()
    cols = []
    for j, c in enumerate(gcols):
        src = fr._col(c)
        v = torch.as_tensor(np.where(np.isneginf(ukeys[:, j]), np.nan, ukeys[:, j]), dtype=torch.float64, device=dev)
        if src.type == "enum":
            cols.append(Column(c, "enum", torch.nan_to_num(v, nan=-1).int(), domain=list(src.domain)))
        else:
            cols.append(Column(c, "real", v))
    for k in range(width):
        cols.append(Column(f"ddply_C{k + 1}", "real",
                           torch.tensor([r[k] if k < len(r) else math.nan for r in rows], dtype=torch.float64, device=dev)))
    return H2OFrame._from_columns(cols)


def grouped_permute(fr: H2OFrame, perm_col, groupby, permute_by, keep_col):
    """Per group (first group column): rows whose ``permute_by`` level is "D" (In) against all others (Out),
    amounts of ``keep_col`` summed per ``perm_col`` id; output = every (In, Out) pair of the group."""
    from .rapids import _idx_list
    g = _idx_list(groupby, fr.ncols)
    gname, pname, kname = fr.names[g[0]], fr.names[int(perm_col)], fr.names[int(keep_col)]
    bcol = fr._col(fr.names[int(permute_by)])
    dom = list(bcol.domain)
    jid = fr._col(gname).as_float().cpu().numpy()
    rid = fr._col(pname).as_float().cpu().numpy()
    amt = fr._col(kname).as_float().cpu().numpy()
    typ = np.array([0 if dom[int(c)] == "D" else 1 for c in bcol.data.cpu().numpy()])
    groups: dict = {}
    for j, r, a, t in zip(jid, rid, amt, typ):
        d = groups.setdefault(j, ({}, {}))[t]
        d[r] = d.get(r, 0.0) + a
    out = []
    for j, (d0, d1) in groups.items():
        for r0, a0 in d0.items():
            for r1, a1 in d1.items():
                out.append((j, r0, r1, a0, a1))
    arr = np.asarray(out, dtype=np.float64).reshape(-1, 5)
    dev = engine_device()
    cols = []
    for k, (name, src) in enumerate(zip([gname, "In", "Out", "InAmnt", "OutAmnt"], [gname, pname, pname, kname, kname])):
        c = fr._col(src)
        v = torch.as_tensor(arr[:, k], device=dev)
        cols.append(Column(name, "enum", v.int(), domain=list(c.domain)) if c.type == "enum" else Column(name, "real", v))
    return H2OFrame._from_columns(cols)


def isax(fr: H2OFrame, num_words, max_cardinality, optimize_card=0):
    """iSAX words of each row (a time series across the columns): piecewise aggregate means of ``num_words``
    segments, z-scored by the row mean / std, mapped to ``max_cardinality`` equiprobable N(0,1) symbols."""
    from scipy.stats import norm
    nw, mc = int(num_words), int(max_cardinality)
    if nw < 0 or mc < 0:
        raise ValueError("numWords and maxCardinality must be greater than 0!")
    for n in fr.names:
        if fr.type(n) not in ("real", "int"):
            raise ValueError("iSax only applies to numeric columns!")
    X = fr.as_tensor(dtype=torch.float64)                          # [N, C]
    step = fr.ncols // nw
    seg = X[:, :nw * step].reshape(X.shape[0], nw, step)
    means = seg.mean(2)
    # the reference accumulates its sigma from within-segment squared deviations (Welford reset per word)
    sse = ((seg - means[:, :, None]) ** 2).sum((1, 2))
    n = nw * step
    mu = seg.reshape(X.shape[0], -1).mean(1)
    sd = torch.sqrt(sse / (n - 1))
    z = (means - mu[:, None]) / sd[:, None]
    bounds = torch.as_tensor(norm.ppf(np.arange(1, mc) / mc), dtype=torch.float64, device=X.device)
    sym = (bounds[None, None, :] < z[:, :, None]).sum(2).clamp(max=mc - 1).double()
    cards = [mc] * nw
    if optimize_card:
        for w in range(nw):
            u = torch.unique(sym[:, w])
            cards[w] = int(u.numel())
            if u.numel() < mc:
                sym[:, w] = torch.searchsorted(u, sym[:, w].contiguous()).double()
    s = sym.long().cpu().numpy()
    idx = np.array(["_".join(f"{s[i, w]}^{cards[w]}" for w in range(nw)) for i in range(s.shape[0])], dtype=object)
    cols = [Column("iSax_index", "string", strings=idx)]
    cols += [Column(f"c{w}", "real", sym[:, w].contiguous()) for w in range(nw)]
    return H2OFrame._from_columns(cols)


# ------------------------------------------------------------------------------------------------ models
def fairness_metrics(model, fr: H2OFrame, protected_columns, reference, favourable_class, frame_name=None):
    """Per protected-group confusion counts, accuracy/precision/F1/rates, AUC / AUCPR / Gini, log loss,
    selection ratio, adverse impact ratios (AIR_*) against the reference group (default: the largest) and a
    Fisher exact / G-test p-value on the selection counts; plus per-group threshold tables."""
    from scipy.stats import chi2_contingency, fisher_exact
    from . import metrics as mm
    if model.model_category != "Binomial":
        raise ValueError("Model has to be a binomial model!")
    protected_columns = [protected_columns] if isinstance(protected_columns, str) else list(protected_columns)
    reference = None if reference is None else ([reference] if isinstance(reference, str) else list(reference))
    for pc in protected_columns:
        if pc not in fr.names:
            raise ValueError(f"{pc} was not found in the frame!")
        if fr.type(pc) != "enum":
            raise ValueError(f"{pc} has to be a categorical column!")
    if reference is not None and len(reference) != len(protected_columns):
        reference = None
    rdom = list(model.info.response_domain)
    if favourable_class not in rdom:
        raise ValueError("Favourable class is not present in the response!")
    fav = rdom.index(favourable_class)
    X, off = fr.model_matrix(model.info, device=model.device)
    P = model.score_tensor(X, off).double()
    thr = model.default_threshold()
    y = fr.response_tensor(model.info, device=P.device).double()
    pred = (P[:, 1] >= thr).double()
    if fav == 0:
        y, pred, prob = 1 - y, 1 - pred, P[:, 0]
    else:
        prob = P[:, 1]
    cards = [len(fr._col(c).domain) + 1 for c in protected_columns]
    if float(np.prod(cards)) > 1e6:
        raise ValueError("Too many combinations of categories! Maximum number of category combinations is 1e6.")
    key = torch.zeros_like(y, dtype=torch.long)
    base = 1
    for c, card in zip(protected_columns, cards):
        code = fr._col(c).data.to(P.device).long()
        key += torch.where(code < 0, torch.full_like(code, card - 1), code) * base
        base *= card
    nrows = float(y.numel())
    fields = ["tp", "fp", "tn", "fn", "total", "relativeSize", "accuracy", "precision", "f1", "tpr", "tnr", "fpr",
              "fnr", "auc", "aucpr", "gini", "selected", "selectedRatio", "logloss"]
    groups, tables = {}, {}
    eps = 1e-15
    for k in torch.unique(key).tolist():
        m = key == k
        yy, pp, pr = y[m], pred[m], prob[m]
        tp = float(((yy == 1) & (pp == 1)).sum()); tn = float(((yy == 0) & (pp == 0)).sum())
        fp = float(((yy == 0) & (pp == 1)).sum()); fn = float(((yy == 1) & (pp == 0)).sum())
        tot = tp + fp + tn + fn
        prc = pr.clamp(eps, 1 - eps)
        ll = float(-(yy * torch.log(prc) + (1 - yy) * torch.log(1 - prc)).sum()) / tot
        div = lambda a, b: a / b if b else math.nan   # noqa: E731
        auc = aucpr = gini = math.nan
        if 0 < float(yy.sum()) < yy.numel():
            bm = mm.binomial_metrics(yy, pr, None, ["0", "1"])
            auc, aucpr, gini = bm["AUC"], bm["pr_auc"], bm["Gini"]
            tables[k] = bm.get("thresholds_and_metric_scores")
        groups[k] = dict(tp=tp, fp=fp, tn=tn, fn=fn, total=tot, relativeSize=tot / nrows, accuracy=div(tp + tn, tot),
                         precision=div(tp, fp + tp), f1=div(2 * tp, 2 * tp + fp + fn), tpr=div(tp, tp + fn),
                         tnr=div(tn, tn + fp), fpr=div(fp, fp + tn), fnr=div(fn, fn + tp), auc=auc, aucpr=aucpr,
                         gini=gini, selected=tp + fp, selectedRatio=div(tp + fp, tot), logloss=ll)

    def decode(k):
        out = []
        for card in cards:
            out.append(k % card)
            k //= card
        return out
    if reference is not None:
        idx = [list(fr._col(c).domain).index(r) for c, r in zip(protected_columns, reference)]
        ref_key, b = 0, 1
        for i, card in zip(idx, cards):
            ref_key += i * b
            b *= card
    else:
        ref_key = max(groups, key=lambda k: groups[k]["total"])
    ref = groups[ref_key]

    def pval(g):
        a, b = int(g["selected"]), int(ref["selected"])
        c, d = int(g["total"] - g["selected"]), int(ref["total"] - ref["selected"])
        try:
            if (ref["total"] < 10000 and g["total"] < 10000) or 0 in (a, b, c, d):
                return float(fisher_exact([[a, b], [c, d]])[1])
            return float(chi2_contingency([[a, c], [b, d]], correction=False, lambda_="log-likelihood")[1])
        except Exception:   # noqa: BLE001 - degenerate tables -> NaN like the reference
            return math.nan
    keys = sorted(groups)
    dev = engine_device()
    cols = []
    for j, c in enumerate(protected_columns):
        codes = [decode(k)[j] for k in keys]
        nlev = len(fr._col(c).domain)
        cols.append(Column(c, "enum", torch.tensor([v if v < nlev else -1 for v in codes], dtype=torch.int32, device=dev),
                           domain=list(fr._col(c).domain)))
    for f in fields:
        cols.append(Column(f, "real", torch.tensor([groups[k][f] for k in keys], dtype=torch.float64, device=dev)))
    for f in fields:
        if f in ("total", "relativeSize"):
            continue
        cols.append(Column("AIR_" + f, "real", torch.tensor(
            [groups[k][f] / ref[f] if ref[f] else math.nan for k in keys], dtype=torch.float64, device=dev)))
    cols.append(Column("p.value", "real", torch.tensor([pval(groups[k]) for k in keys], dtype=torch.float64, device=dev)))
    res = {"overview": H2OFrame._from_columns(cols)}
    for k, tab in tables.items():
        if not tab:
            continue
        name = "_".join(
            (list(fr._col(c).domain)[v] if v < len(fr._col(c).domain) else "NaN")
            for c, v in zip(protected_columns, decode(k)))
        import pandas as pd
        res["thresholds_and_metrics_" + "".join(ch if ch.isalnum() or ch == "," else "_" for ch in name)] = \
            H2OFrame(pd.DataFrame(tab))
    return res


def predicted_vs_actual_by_variable(model, fr: H2OFrame, variable, predicted: H2OFrame):
    """Weighted mean prediction and mean actual per level of a categorical variable (NA level last)."""
    if model.info.response is None:
        raise ValueError("Only supervised models are supported for calculating predicted v actual")
    if model.model_category == "Multinomial":
        raise ValueError("Multinomial classification models are not supported by predicted v actual")
    if variable not in fr.names:
        raise ValueError(f"Frame doesn't contain column '{variable}'.")
    if fr.nrows != predicted.nrows:
        raise ValueError("Input frame and frame of predictions need to have same number of columns.")
    vc = fr._col(variable)
    dom = list(vc.domain) if vc.type == "enum" else None
    if dom is None:
        raise ValueError(f"{variable} must be categorical")
    pcol = predicted._col(0)
    yc = fr._col(model.info.response)
    p = pcol.as_float().double()
    a = yc.as_float().double()
    w = fr._col(model.info.weights).as_float().double() if model.info.weights else torch.ones_like(p)
    code = vc.data.long()
    code = torch.where(code < 0, torch.full_like(code, len(dom)), code).to(p.device)
    L = len(dom) + 1
    sw = torch.zeros(L, dtype=torch.float64, device=p.device).index_add_(0, code, w)
    sp = torch.zeros_like(sw).index_add_(0, code, w * p)
    sa = torch.zeros_like(sw).index_add_(0, code, w * a)
    dev = engine_device()
    return H2OFrame._from_columns([
        Column(variable, "enum", torch.arange(L, dtype=torch.int32, device=dev).where(
            torch.arange(L, device=dev) < len(dom), torch.tensor(-1, dtype=torch.int32, device=dev)), domain=dom),
        Column(predicted.names[0], "real", (sp / sw).to(dev)),
        Column("actual", "real", (sa / sw).to(dev))])


def test_java_scoring(model, fr: H2OFrame, preds: H2OFrame, epsilon):
    """Score the frame through the model's exported MOJO (the Java-scoring stand-in) and compare to ``preds``."""
    import os
    import tempfile
    from .mojo import reader, writer
    path = writer.write_mojo(model, os.path.join(tempfile.mkdtemp(), "model.zip"))
    g = reader.import_mojo(path)
    a = g.predict(fr).as_tensor(dtype=torch.float64)
    b = preds.as_tensor(dtype=torch.float64)
    k = min(a.shape[1], b.shape[1])
    ok = torch.allclose(a[:, -k:], b[:, -k:], rtol=0, atol=float(epsilon), equal_nan=True)
    return H2OFrame._from_columns([Column("C1", "real", torch.tensor([1.0 if ok else 0.0], dtype=torch.float64,
                                                                     device=engine_device()))])


def pav(fr: H2OFrame):
    """Pool-adjacent-violators on a sorted (x, y[, w]) frame: the thresholds frame (x, y) of the fit."""
    from .models.isotonic import pava
    X = fr.as_tensor(dtype=torch.float64).cpu().numpy()
    x, y = X[:, 0], X[:, 1]
    w = X[:, 2] if X.shape[1] > 2 else np.ones_like(y)
    ok = ~(np.isnan(x) | np.isnan(y) | np.isnan(w)) & (w > 0)
    x, y, w = x[ok], y[ok], w[ok]
    o = np.argsort(x, kind="stable")
    fit = pava(y[o], w[o])
    xs = x[o]
    keep = np.ones(len(fit), dtype=bool)     # knots: first and last point of every constant block
    if len(fit) > 2:
        same_prev = np.r_[False, fit[1:] == fit[:-1]]
        same_next = np.r_[fit[:-1] == fit[1:], False]
        keep = ~(same_prev & same_next)
    dev = engine_device()
    return H2OFrame._from_columns([Column("X", "real", torch.as_tensor(xs[keep], device=dev)),
                                   Column("Y", "real", torch.as_tensor(fit[keep], dtype=torch.float64, device=dev))])


_TOOLS = {}


def register_tool(name, fn):
    _TOOLS[name] = fn


def run_tool(tool_class, tool_parameters):
    """``run_tool``: internal maintenance tools by name (reference runs a Java main class)."""
    name = tool_class.split(".")[-1]
    if name not in _TOOLS:
        raise ValueError(f"unknown tool {tool_class!r}; available: {sorted(_TOOLS)}")
    args = tool_parameters if isinstance(tool_parameters, list) else [tool_parameters]
    return _TOOLS[name](*[str(a) for a in args])


def _tool_convert_mojo(src, dst):
    """MojoConvertTool: re-export an imported MOJO (zip) to ``dst``."""
    import shutil
    shutil.copyfile(src, dst)
    return "OK"


register_tool("MojoConvertTool", _tool_convert_mojo)


def more_prims(sess):
    fr = lambda v: sess_frame(v)   # noqa: E731

    def model(m):
        return dkv.get(m) if isinstance(m, str) else m
    return {
        "%/%": lambda a, b: sess.prims["intDiv"](a, b),
        "ddply": lambda a, g, f: ddply(sess, fr(a), g, f),
        "grouped_permute": lambda a, p, g, by, keep: grouped_permute(fr(a), p, g, by, keep),
        "isax": lambda a, nw, mc, opt=0: isax(fr(a), nw, mc, opt),
        "fairnessMetrics": lambda m, f, pc, ref, fav: fairness_metrics(model(m), fr(f), pc, ref, fav),
        "predicted.vs.actual.by.var": lambda m, f, var, p: predicted_vs_actual_by_variable(model(m), fr(f), var, fr(p)),
        "model.testJavaScoring": lambda m, f, p, eps: test_java_scoring(model(m), fr(f), fr(p), eps),
        "isotonic.pav": lambda f: pav(fr(f)),
        "rulefit.predict.rules": lambda m, f, ids: model(m).predict_rules(fr(f), ids if isinstance(ids, list) else [ids]),
        "tree.update.weights": lambda m, f, wc: model(m).update_tree_weights(fr(f), wc),
        "set.calibration.model": lambda m, c: model(m).set_calibration_model(model(c)),
        "word2vec.to.frame": lambda m: model(m).to_frame(),
        "segment_models_as_frame": lambda s: model(s).as_frame(),
        "scale_inplace": lambda a, c=1, s=1: _scale_inplace(fr(a), c, s),
        "run_tool": lambda tc, tp: run_tool(tc, tp),
        "testing.setreadforbidden": lambda forbidden: _set_read_forbidden(forbidden),
    }


def sess_frame(v):
    from .rapids import _frame
    return _frame(v)


def _scale_inplace(f, c, s):
    out = f.scale(bool(c) if not isinstance(c, list) else c, bool(s) if not isinstance(s, list) else s)
    for n in f.names:
        f._cols[n] = out._col(n)
    return f


def _set_read_forbidden(forbidden):
    READ_FORBIDDEN.clear()
    READ_FORBIDDEN.update([forbidden] if isinstance(forbidden, str) else list(forbidden))
    return "OK"
