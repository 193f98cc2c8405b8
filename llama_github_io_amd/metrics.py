"""Model metrics (reference: ``hex/ModelMetricsBinomial.java``, ``ModelMetricsMultinomial.java``,
``ModelMetricsRegression.java``, ``ModelMetricsClustering.java``, ``AUC2.java``, ``GainsLift.java``,
``ConfusionMatrix.java``).

All metric builders take torch tensors (any device) and reduce on device; the summary is a plain
python object with H2O's metric names (``auc``, ``aucpr``, ``logloss``, ``mse``, ``rmse``, ``mae``,
``rmsle``, ``mean_residual_deviance``, ``r2``, ``mean_per_class_error``, ``hit_ratio_table``,
``thresholds_and_metric_scores``, ``gains_lift_table``, ...).
"""
from __future__ import annotations

import math

import numpy as np
import torch

THRESHOLD_CRITERIA = ("f1", "f2", "f0point5", "accuracy", "precision", "recall", "specificity",
                      "absolute_mcc", "min_per_class_accuracy", "mean_per_class_accuracy")


def _sharded_rows(*row_args):
    """Metrics of row-sharded predictions: all-gather the per-row arguments named in ``row_args``
    (rank order) and compute once on the full rows — exact, and bit-identical to the single-process
    metrics (the reference merges fixed-bin AUC2 histograms instead; the gathered predictions are a
    few bytes per row, small next to training traffic)."""
    import functools
    import inspect

    def deco(fn):
        sig = inspect.signature(fn)

        @functools.wraps(fn)
        def w(*args, **kwargs):
            from .parallel import collectives as coll
            if not coll.is_dist():
                return fn(*args, **kwargs)
            b = sig.bind(*args, **kwargs)
            b.apply_defaults()
            for name in row_args:
                t = b.arguments.get(name)
                if isinstance(t, torch.Tensor):
                    dev = t.device
                    g = coll.all_gather_cat(t.contiguous().cpu() if coll.comm_device().type == "cpu" else t.contiguous(), 0)
                    b.arguments[name] = g.to(dev)
            with coll.replicated():
                return fn(*b.args, **b.kwargs)
        return w
    return deco


class ModelMetrics(dict):
    """dict with attribute access; ``model_category`` names the family."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    # H2O-python style accessors
    def auc(self): return self.get("AUC")
    def aucpr(self): return self.get("pr_auc")
    def logloss(self): return self.get("logloss")
    def mse(self): return self.get("MSE")
    def rmse(self): return self.get("RMSE")
    def mae(self): return self.get("mae")
    def r2(self): return self.get("r2")
    def mean_residual_deviance(self): return self.get("mean_residual_deviance")
    def mean_per_class_error(self): return self.get("mean_per_class_error")
    def gini(self): return self.get("Gini")

    def __repr__(self):
        keys = [k for k in ("model_category", "MSE", "RMSE", "mae", "r2", "logloss", "AUC", "pr_auc",
                            "mean_per_class_error", "mean_residual_deviance", "tot_withinss", "betweenss")
                if k in self]
        return "ModelMetrics(" + ", ".join(f"{k}={self[k]}" for k in keys) + ")"


def _w(w, n, device):
    return torch.ones(n, dtype=torch.float64, device=device) if w is None else w.double()


@_sharded_rows("y", "pred", "w")
def regression_metrics(y, pred, w=None, distribution=None) -> ModelMetrics:
    y, pred = y.double(), pred.double()
    w = _w(w, y.numel(), y.device)
    ok = ~torch.isnan(y) & (w > 0)
    y, pred, w = y[ok], pred[ok], w[ok]
    sw = w.sum()
    err = y - pred
    mse = (w * err * err).sum() / sw
    mae = (w * err.abs()).sum() / sw
    ybar = (w * y).sum() / sw
    var = (w * (y - ybar) ** 2).sum() / sw
    r2 = 1 - mse / var if var > 0 else torch.tensor(float("nan"))
    rmsle = float("nan")
    if bool((y > -1).all()) and bool((pred > -1).all()):
        rmsle = math.sqrt(float((w * (torch.log1p(pred) - torch.log1p(y)) ** 2).sum() / sw))
    mrd = float(mse)
    if distribution is not None and distribution.name not in ("gaussian",):
        f = distribution.link_fn(torch.clamp(pred, min=1e-300)) if distribution.link == "log" else pred
        try:
            mrd = float(distribution.deviance(w, y, f).sum() / sw)
        except Exception:  # noqa: BLE001
            mrd = float(mse)
    return ModelMetrics(model_category="Regression", MSE=float(mse), RMSE=math.sqrt(float(mse)), mae=float(mae),
                        rmsle=rmsle, r2=float(r2), mean_residual_deviance=mrd, nobs=int(y.numel()))


def _auc_from_sorted(pos, neg):
    """pos/neg: weights per distinct threshold sorted by descending score. Trapezoid ROC + PR AUC."""
    tp = torch.cumsum(pos, 0)
    fp = torch.cumsum(neg, 0)
    P, Nn = tp[-1], fp[-1]
    if P <= 0 or Nn <= 0:
        return float("nan"), float("nan"), tp, fp
    tpr = torch.cat([torch.zeros(1, dtype=tp.dtype, device=tp.device), tp / P])
    fpr = torch.cat([torch.zeros(1, dtype=fp.dtype, device=fp.device), fp / Nn])
    auc = torch.trapz(tpr, fpr)
    prec = tp / (tp + fp)
    rec = tp / P
    rec0 = torch.cat([torch.zeros(1, dtype=rec.dtype, device=rec.device), rec])
    prec0 = torch.cat([prec[:1], prec])
    aucpr = torch.trapz(prec0, rec0)
    return float(auc), float(aucpr), tp, fp


@_sharded_rows("y", "p1", "w")
def binomial_metrics(y, p1, w=None, domain=("0", "1"), nbins_thresholds: int = 400) -> ModelMetrics:
    """y in {0,1}; p1 = P(class 1)."""
    y, p1 = y.double(), p1.double()
    w = _w(w, y.numel(), y.device)
    ok = ~torch.isnan(y) & (w > 0)
    y, p1, w = y[ok], p1[ok], w[ok]
    sw = w.sum()
    pc = torch.clamp(p1, 1e-15, 1 - 1e-15)
    logloss = float(-(w * (y * torch.log(pc) + (1 - y) * torch.log(1 - pc))).sum() / sw)
    mse = float((w * (y - p1) ** 2).sum() / sw)
    # exact ROC over distinct scores
    order = torch.argsort(p1, descending=True)
    ps, ys, ws = p1[order], y[order], w[order]
    pos, neg, uniq = _group_sorted(ps, ws * ys, ws * (1 - ys))
    auc, aucpr, tp, fp = _auc_from_sorted(pos, neg)
    # thresholds table (H2O keeps <= 400 bins)
    thr_tab = _threshold_table(uniq, tp, fp, nbins_thresholds)
    ybar = float((w * y).sum() / sw)
    var = ybar * (1 - ybar)
    r2 = 1 - mse / var if var > 0 else float("nan")
    mm = ModelMetrics(model_category="Binomial", MSE=mse, RMSE=math.sqrt(mse), logloss=logloss, AUC=auc,
                      pr_auc=aucpr, Gini=2 * auc - 1 if auc == auc else float("nan"), r2=r2, nobs=int(y.numel()),
                      domain=list(domain), thresholds_and_metric_scores=thr_tab)
    if thr_tab:
        best = max(thr_tab, key=lambda r: r["f1"])
        mm["max_f1_threshold"] = best["threshold"]
        mm["cm"] = dict(threshold=best["threshold"], table=[[best["tns"], best["fps"]], [best["fns"], best["tps"]]])
        mm["mean_per_class_error"] = 1 - best["mean_per_class_accuracy"]
        mm["max_criteria_and_metric_scores"] = {c: max(thr_tab, key=lambda r: r[c])[c] for c in THRESHOLD_CRITERIA}
    mm["gains_lift_table"] = gains_lift(y, p1, w)
    return mm


def _group_sorted(keys_sorted, a, b):
    """Per distinct key of an already-sorted key vector: sums of a and b (segmented by cumsum)."""
    uniq, counts = torch.unique_consecutive(keys_sorted, return_counts=True)
    ends = torch.cumsum(counts, 0) - 1
    ca, cb = torch.cumsum(a, 0)[ends], torch.cumsum(b, 0)[ends]
    za = torch.zeros(1, dtype=ca.dtype, device=ca.device)
    return torch.diff(ca, prepend=za), torch.diff(cb, prepend=za), uniq


def _threshold_table(uniq, tp, fp, nb):
    n = uniq.numel()
    if n == 0:
        return []
    P, Nn = float(tp[-1]), float(fp[-1])
    # float64 lattice: a float32 linspace rounds n - 1 up to n past 2^24 distinct scores (one element out of
    # bounds: the HSA 0x1016 memory fault of the 100M-row XGBoost run)
    idx = torch.linspace(0, n - 1, steps=min(n, nb), dtype=torch.float64, device=uniq.device).round().long().unique()
    idx = idx.clamp_(0, n - 1)
    th = uniq[idx].cpu().numpy()
    tps = tp[idx].cpu().numpy(); fps = fp[idx].cpu().numpy()
    rows = []
    for t, a, b in zip(th, tps, fps):
        fn, tn = P - a, Nn - b
        prec = a / (a + b) if a + b > 0 else 1.0
        rec = a / P if P > 0 else 0.0
        spec = tn / Nn if Nn > 0 else 0.0
        f = lambda beta: (1 + beta ** 2) * prec * rec / (beta ** 2 * prec + rec) if (beta ** 2 * prec + rec) > 0 else 0.0
        den = math.sqrt(max((a + b) * (a + fn) * (tn + b) * (tn + fn), 1e-300))
        mcc = (a * tn - b * fn) / den
        rows.append(dict(threshold=float(t), f1=f(1.0), f2=f(2.0), f0point5=f(0.5), accuracy=(a + tn) / (P + Nn),
                         precision=prec, recall=rec, specificity=spec, absolute_mcc=abs(mcc),
                         min_per_class_accuracy=min(rec, spec), mean_per_class_accuracy=(rec + spec) / 2,
                         tns=tn, fns=fn, fps=b, tps=a))
    return rows


def gains_lift(y, p1, w, groups: int = 16):
    order = torch.argsort(p1, descending=True)
    ys, ws = y[order], w[order]
    cw = torch.cumsum(ws, 0)
    tot = float(cw[-1]) if cw.numel() else 0.0
    tot_pos = float((ws * ys).sum())
    if tot <= 0 or tot_pos <= 0:
        return []
    out = []
    cpos = torch.cumsum(ws * ys, 0)
    for g in range(1, groups + 1):
        frac = g / groups
        k = int(torch.searchsorted(cw, torch.tensor(frac * tot, dtype=cw.dtype, device=cw.device)).clamp(max=cw.numel() - 1))
        cum_rate = float(cpos[k] / cw[k])
        out.append(dict(group=g, cumulative_data_fraction=float(cw[k] / tot), cumulative_capture_rate=float(cpos[k]) / tot_pos,
                        cumulative_lift=cum_rate / (tot_pos / tot), cumulative_response_rate=cum_rate))
    return out


@_sharded_rows("y", "probs", "w")
def multinomial_metrics(y, probs, w=None, domain=None, hit_k: int = 10) -> ModelMetrics:
    """y: class index; probs [N, K]."""
    y = y.long() if not torch.is_floating_point(y) else torch.nan_to_num(y, nan=-1).long()
    w = _w(w, y.numel(), y.device)
    ok = (y >= 0) & (w > 0)
    y, probs, w = y[ok], probs[ok].double(), w[ok]
    K = probs.shape[1]
    sw = w.sum()
    py = torch.clamp(probs.gather(1, y[:, None]).squeeze(1), 1e-15, 1.0)
    logloss = float(-(w * torch.log(py)).sum() / sw)
    onehot = torch.nn.functional.one_hot(y, K).double()
    mse = float((w * ((onehot - probs) ** 2).sum(1)).sum() / sw)
    pred = probs.argmax(1)
    from .ops.segment import segment_sum
    cm = segment_sum(y * K + pred, w, K * K).view(K, K)
    per_class_err = 1 - torch.diag(cm) / cm.sum(1).clamp(min=1e-300)
    rank = (probs > py[:, None]).sum(1)
    hits = [float((w * (rank < k).double()).sum() / sw) for k in range(1, min(hit_k, K) + 1)]
    auc = multinomial_auc(y, probs, w) if K <= 50 else float("nan")
    return ModelMetrics(model_category="Multinomial", MSE=mse, RMSE=math.sqrt(mse), logloss=logloss,
                        mean_per_class_error=float(per_class_err.mean()), cm=dict(table=cm.cpu().tolist()),
                        hit_ratio_table=hits, nobs=int(y.numel()), domain=domain, AUC=auc)


def multinomial_auc(y, probs, w):
    """Macro one-vs-rest AUC (H2O ``MultinomialAucType.MACRO_OVR``)."""
    K = probs.shape[1]
    aucs = []
    for k in range(K):
        yk = (y == k).double()
        if yk.sum() == 0 or yk.sum() == yk.numel():
            continue
        order = torch.argsort(probs[:, k], descending=True)
        ps = probs[order, k]
        pos, neg, _ = _group_sorted(ps, (w * yk)[order], (w * (1 - yk))[order])
        aucs.append(_auc_from_sorted(pos, neg)[0])
    return float(np.mean(aucs)) if aucs else float("nan")


def clustering_metrics(X, centers, assign, w=None, chunk: int = 1 << 20) -> ModelMetrics:
    """X [N, F] (standardised space), centers [K, F], assign [N].

    fp64 sums over row chunks (no [N, F] fp64 temporaries); row-sharded frames merge per-rank partial
    sums (sizes, within-SS, column sums, then total SS about the global mean) with all-reduces instead of
    gathering rows (``hex/ModelMetricsClustering.java`` IndependentMetricBuilder.reduce)."""
    from .ops.segment import segment_sum
    from .parallel import collectives as coll
    C = centers.double().to(X.device)
    K, N = C.shape[0], X.shape[0]
    w = _w(w, N, X.device)
    within = torch.zeros(K, dtype=torch.float64, device=X.device)
    size = torch.zeros(K, dtype=torch.float64, device=X.device)
    sx = torch.zeros(X.shape[1] + 1, dtype=torch.float64, device=X.device)
    for i in range(0, N, chunk):
        xb, ab, wb = X[i:i + chunk].double(), assign[i:i + chunk].long(), w[i:i + chunk]
        d = ((xb - C[ab]) ** 2).sum(1)
        within += segment_sum(ab, wb * d, K)
        size += segment_sum(ab, wb, K)
        sx[:-1] += (wb[:, None] * xb).sum(0)
        sx[-1] += wb.sum()
    dist = coll.is_dist()
    if dist:
        for t in (within, size, sx):
            coll.all_reduce_(t)
    mu = sx[:-1] / sx[-1]
    totss = torch.zeros(1, dtype=torch.float64, device=X.device)
    for i in range(0, N, chunk):
        xb, wb = X[i:i + chunk].double(), w[i:i + chunk]
        totss += (wb * ((xb - mu) ** 2).sum(1)).sum()
    if dist:
        coll.all_reduce_(totss)
    totss = float(totss)
    tw = float(within.sum())
    n = int(coll.all_reduce_scalar(N)) if dist else N
    return ModelMetrics(model_category="Clustering", tot_withinss=tw, totss=totss, betweenss=totss - tw,
                        withinss=within.cpu().tolist(), size=size.cpu().tolist(), nobs=n)


@_sharded_rows("score", "w")
def anomaly_metrics(score, w=None) -> ModelMetrics:
    s = score.double()
    return ModelMetrics(model_category="AnomalyDetection", mean_score=float(s.mean()), nobs=int(s.numel()))


@_sharded_rows("err")
def autoencoder_metrics(err) -> ModelMetrics:
    e = err.double()
    return ModelMetrics(model_category="AutoEncoder", MSE=float(e.mean()), RMSE=math.sqrt(float(e.mean())), nobs=int(e.numel()))


@_sharded_rows("y", "preds", "w")
def make_metrics(category: str, y, preds, w=None, domain=None, distribution=None) -> ModelMetrics:
    """preds: regression -> [N] mean; binomial -> [N] p1 or [N,2]; multinomial -> [N,K] probs."""
    if category == "Binomial":
        p1 = preds[:, -1] if preds.dim() == 2 else preds
        return binomial_metrics(y, p1, w, domain or ("0", "1"))
    if category == "Multinomial":
        return multinomial_metrics(y, preds, w, domain)
    return regression_metrics(y, preds.reshape(-1), w, distribution)
