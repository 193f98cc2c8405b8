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
import os

import numpy as np
import torch

THRESHOLD_CRITERIA = ("f1", "f2", "f0point5", "accuracy", "precision", "recall", "specificity",
                      "absolute_mcc", "min_per_class_accuracy", "mean_per_class_accuracy")


def _dist() -> bool:
    from .parallel import collectives as coll
    return coll.is_dist()


def _allreduce(t: torch.Tensor, op=None) -> torch.Tensor:
    """All-reduce a small statistics tensor (staged through the collective device)."""
    from .parallel import collectives as coll
    dev = coll.comm_device()
    h = t.to(dev)
    coll.all_reduce_(h, op)
    return h.to(t.device)


# Score lattice of the binomial metrics: 2^18 equal bins over [0, 1] (AUC2.java keeps 400 merging bins; a
# finer FIXED lattice merges across row shards by plain summation and keeps the AUC within ~1e-6 of the
# exact one). Every bin carries (positive weight, negative weight, max score): the threshold table, the
# gains/lift groups and — for row-sharded frames — the ROC/PR curves come from these merged histograms.
SCORE_BINS = 1 << 18
# single-process frames of at least this many rows take ROC / PR AUC from the lattice too (no 10M-row sort)
LATTICE_AUC_ROWS = int(os.environ.get("H2O_LATTICE_AUC_ROWS", 1 << 21))


def _score_hist(p, pos_w, neg_w, nb: int = SCORE_BINS, y=None, w=None):
    """[3, nb] float64 (pos, neg, max score; -inf = empty) of scores p in [0, 1], merged over row shards. With
    y / w given on a GPU: one HIP pass (csrc/metrics_kernels.hip) instead of three torch reductions."""
    if y is not None and p.is_cuda and os.environ.get("H2O_METRICS_HIP", "1") != "0":
        from .ops import _native as nat
        h = torch.zeros(3, nb, dtype=torch.float64, device=p.device)
        pd, yd = p.double().contiguous(), y.double().contiguous()
        wd = None if w is None else w.double().contiguous()
        nat.call("h2o_score_hist", pd.data_ptr(), yd.data_ptr(), 0 if wd is None else wd.data_ptr(), pd.numel(), nb,
                 h[0].data_ptr(), h[1].data_ptr(), h[2].data_ptr(), nat.stream_ptr(p.device))
        mx = h[2].view(torch.int64).view(torch.float64)
        h[2] = torch.where((h[0] + h[1]) > 0, mx, torch.full_like(mx, float("-inf")))
    else:
        from .ops.segment import segment_sum
        if pos_w is None:
            wd = torch.ones_like(p, dtype=torch.float64) if w is None else w.double()
            pos_w, neg_w = wd * y, wd * (1 - y)
        b = torch.clamp((p * nb).long(), 0, nb - 1)
        h = torch.empty(3, nb, dtype=torch.float64, device=p.device)
        h[0] = segment_sum(b, pos_w, nb)
        h[1] = segment_sum(b, neg_w, nb)
        h[2] = torch.full((nb,), float("-inf"), dtype=torch.float64, device=p.device).scatter_reduce(
            0, b, p.double(), reduce="amax", include_self=True)
    if _dist():
        from torch.distributed import ReduceOp
        h[:2] = _allreduce(h[:2].contiguous())
        h[2] = _allreduce(h[2].contiguous(), ReduceOp.MAX)
    return h


def _hist_curve(h):
    """Non-empty bins in descending score order: (pos, neg, representative score = the bin's max)."""
    nz = torch.nonzero((h[0] + h[1]) > 0).squeeze(1).flip(0)
    return h[0, nz], h[1, nz], h[2, nz]


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

    # ---- h2o-py model metrics surface (h2o-py/h2o/model/metrics/*.py): thresholds, confusion matrices, ROC,
    # gains / lift, deviance / likelihood, clustering and survival / uplift scalars
    _ALIASES = dict(fallout="fpr", missrate="fnr", recall="tpr", sensitivity="tpr", specificity="tnr")
    MAXIMIZING = ("absolute_mcc", "accuracy", "precision", "f0point5", "f1", "f2", "mean_per_class_accuracy",
                  "min_per_class_accuracy", "tns", "fns", "fps", "tps", "tnr", "fnr", "fpr", "tpr",
                  "fallout", "missrate", "recall", "sensitivity", "specificity")

    def _thr_rows(self):
        rows = self.get("thresholds_and_metric_scores") or []
        out = []
        for r in rows:
            r = dict(r)
            P, N = r["tps"] + r["fns"], r["tns"] + r["fps"]
            r.setdefault("tpr", r["tps"] / P if P > 0 else 0.0)
            r.setdefault("fnr", r["fns"] / P if P > 0 else 0.0)
            r.setdefault("tnr", r["tns"] / N if N > 0 else 0.0)
            r.setdefault("fpr", r["fps"] / N if N > 0 else 0.0)
            out.append(r)
        return out

    def find_threshold_by_max_metric(self, metric):
        m = self._ALIASES.get(metric, metric)
        rows = self._thr_rows()
        if not rows:
            raise ValueError("no threshold table (binomial metrics only)")
        return max(rows, key=lambda r: r[m])["threshold"]

    def find_idx_by_threshold(self, threshold):
        rows = self._thr_rows()
        th = [r["threshold"] for r in rows]
        if threshold in th:
            return th.index(threshold)
        return min(range(len(th)), key=lambda i: abs(th[i] - threshold))

    def metric(self, metric, thresholds=None):
        """[[threshold, value], ...] with ``.value`` (scalar for None / one threshold), as h2o-py's metric()."""
        if metric not in self.MAXIMIZING:
            raise ValueError("The only allowable metrics are " + ", ".join(self.MAXIMIZING))
        m = self._ALIASES.get(metric, metric)
        rows = self._thr_rows()
        scalar = thresholds is None or isinstance(thresholds, (int, float))
        if thresholds is None:
            ts = [self.find_threshold_by_max_metric(m)]
        elif thresholds == "all":
            ts = [r["threshold"] for r in rows]
        elif isinstance(thresholds, (int, float)):
            ts = [thresholds]
        else:
            ts = list(thresholds)
        out = _MetricList([t, rows[self.find_idx_by_threshold(t)][m]] for t in ts)
        out.value = out[0][1] if scalar else [r[1] for r in out]
        return out

    def F1(self, thresholds=None): return self.metric("f1", thresholds)
    def F2(self, thresholds=None): return self.metric("f2", thresholds)
    def F0point5(self, thresholds=None): return self.metric("f0point5", thresholds)
    def accuracy(self, thresholds=None): return self.metric("accuracy", thresholds)
    def precision(self, thresholds=None): return self.metric("precision", thresholds)
    def recall(self, thresholds=None): return self.metric("tpr", thresholds)
    def sensitivity(self, thresholds=None): return self.metric("tpr", thresholds)
    def tpr(self, thresholds=None): return self.metric("tpr", thresholds)
    def tnr(self, thresholds=None): return self.metric("tnr", thresholds)
    def specificity(self, thresholds=None): return self.metric("tnr", thresholds)
    def fpr(self, thresholds=None): return self.metric("fpr", thresholds)
    def fallout(self, thresholds=None): return self.metric("fpr", thresholds)
    def fnr(self, thresholds=None): return self.metric("fnr", thresholds)
    def missrate(self, thresholds=None): return self.metric("fnr", thresholds)
    def mcc(self, thresholds=None): return self.metric("absolute_mcc", thresholds)

    def error(self, thresholds=None):
        acc = self.metric("accuracy", thresholds)
        out = _MetricList([t, 1 - v] for t, v in acc)
        out.value = [1 - v for v in acc.value] if isinstance(acc.value, list) else 1 - acc.value
        return out

    def max_per_class_error(self, thresholds=None):
        acc = self.metric("min_per_class_accuracy", thresholds)
        out = _MetricList([t, 1 - v] for t, v in acc)
        out.value = [1 - v for v in acc.value] if isinstance(acc.value, list) else 1 - acc.value
        return out

    @property
    def thresholds(self):
        return [r["threshold"] for r in self._thr_rows()]

    @property
    def fprs(self):
        return [r["fpr"] for r in self._thr_rows()]

    @property
    def tprs(self):
        return [r["tpr"] for r in self._thr_rows()]

    def roc(self):
        """(false positive rates, true positive rates) over the threshold table."""
        return self.fprs, self.tprs

    def confusion_matrix(self, metrics=None, thresholds=None):
        """Binomial: ConfusionMatrix at the threshold maximizing ``metrics`` (default f1) or at ``thresholds``;
        multinomial / ordinal: the model's confusion matrix."""
        if not self.get("thresholds_and_metric_scores"):
            cm = self.get("cm")
            if cm is None:
                return None
            dom = list(self.get("domain") or range(len(cm["table"])))
            return ConfusionMatrix(cm["table"], dom, "Confusion Matrix: Row labels: Actual class; Column labels: "
                                                      "Predicted class")
        if metrics is None and thresholds is None:
            metrics = ["f1"]
        ml = metrics if isinstance(metrics, list) else ([] if metrics is None else [metrics])
        tl = thresholds if isinstance(thresholds, list) else ([] if thresholds is None else [thresholds])
        if not all(m.lower() in self.MAXIMIZING for m in ml):
            raise ValueError("The only allowable metrics are " + ", ".join(self.MAXIMIZING))
        rows = self._thr_rows()
        items = [(t, None) for t in tl] + [(self.find_threshold_by_max_metric(m.lower()), m) for m in ml]
        out = []
        for t, m in items:
            r = rows[self.find_idx_by_threshold(t)]
            hdr = (f"Confusion Matrix (Act/Pred) for max {m} @ threshold = {r['threshold']}" if m else
                   f"Confusion Matrix (Act/Pred) @ threshold = {r['threshold']}")
            out.append(ConfusionMatrix([[r["tns"], r["fps"]], [r["fns"], r["tps"]]],
                                       list(self.get("domain") or ["0", "1"]), hdr))
        return out[0] if len(out) == 1 else out

    def gains_lift(self):
        import pandas as pd
        gl = self.get("gains_lift_table")
        return pd.DataFrame(gl) if gl else None

    def plot(self, type="roc", server=False, save_plot_path=None, plot=True):
        """ROC ('roc'), precision-recall ('pr') or gains/lift ('gainslift') curve; a matplotlib figure."""
        import matplotlib
        matplotlib.use("Agg", force=False)
        import matplotlib.pyplot as plt
        fig, ax = plt.subplots()
        if type == "roc":
            ax.plot(self.fprs, self.tprs)
            ax.set_xlabel("False Positive Rate")
            ax.set_ylabel("True Positive Rate")
            ax.set_title(f"ROC Curve (AUC = {self.get('AUC')})")
        elif type == "pr":
            rows = self._thr_rows()
            ax.plot([r["tpr"] for r in rows], [r["precision"] for r in rows])
            ax.set_xlabel("Recall")
            ax.set_ylabel("Precision")
        else:
            gl = self.gains_lift()
            ax.plot(gl["cumulative_data_fraction"], gl["cumulative_lift"])
            ax.set_xlabel("Cumulative data fraction")
            ax.set_ylabel("Cumulative lift")
        if save_plot_path:
            fig.savefig(save_plot_path)
        return fig

    def n(self): return self.get("nobs")
    def residual_deviance(self): return self.get("residual_deviance")
    def residual_degrees_of_freedom(self): return self.get("residual_degrees_of_freedom")
    def null_deviance(self): return self.get("null_deviance")
    def null_degrees_of_freedom(self): return self.get("null_degrees_of_freedom")
    def aic(self): return self.get("AIC", self.get("aic"))
    def loglikelihood(self): return self.get("loglikelihood")
    def hglm_metric(self, metric_string): return self.get(metric_string)
    def custom_metric_name(self): return self.get("custom_metric_name")
    def custom_metric_value(self): return self.get("custom_metric_value")
    def tot_withinss(self): return self.get("tot_withinss")
    def totss(self): return self.get("totss")
    def betweenss(self): return self.get("betweenss")
    def num_err(self): return self.get("numerr", self.get("num_err"))
    def cat_err(self): return self.get("caterr", self.get("cat_err"))
    def concordance(self): return self.get("concordance")
    def concordant(self): return self.get("concordant")
    def tied_y(self): return self.get("tied_y")
    def mean_score(self): return self.get("mean_score")
    def mean_normalized_score(self): return self.get("mean_normalized_score")
    def auuc(self, metric=None): return self.get("AUUC")
    def auuc_normalized(self, metric=None): return self.get("auuc_normalized")
    def qini(self): return self.get("qini")
    def aecu(self, metric="qini"): return (self.get("aecu_table") or {}).get(metric, self.get("aecu"))
    def auuc_table(self): return self.get("auuc_table")
    def aecu_table(self): return self.get("aecu_table")
    def uplift(self, metric="AUTO"): return (self.get("auuc_table") or {}).get("uplift")
    def uplift_normalized(self, metric="AUTO"): return (self.get("auuc_table") or {}).get("uplift_normalized")
    def uplift_random(self, metric="AUTO"): return (self.get("auuc_table") or {}).get("uplift_random")
    def multinomial_auc_table(self): return self.get("multinomial_auc_table")
    def multinomial_aucpr_table(self): return self.get("multinomial_aucpr_table")

    def show(self, verbosity=None, fmt=None):
        print(repr(self))

    def __repr__(self):
        keys = [k for k in ("model_category", "MSE", "RMSE", "mae", "r2", "logloss", "AUC", "pr_auc",
                            "mean_per_class_error", "mean_residual_deviance", "tot_withinss", "betweenss")
                if k in self]
        return "ModelMetrics(" + ", ".join(f"{k}={self[k]}" for k in keys) + ")"


class _MetricList(list):
    """[[threshold, value], ...] with a ``value`` attribute (h2o-py metrics' List)."""
    value = None


class ConfusionMatrix:
    """h2o-py ConfusionMatrix: ``table`` (pandas, with the per-row Error and Rate columns) and ``to_list()``."""

    def __init__(self, cm, domains, table_header=""):
        import pandas as pd
        self._cm = [[float(v) for v in r] for r in cm]
        self.domains = [str(d) for d in domains]
        self.table_header = table_header
        rows = []
        for i, r in enumerate(self._cm):
            tot = sum(r)
            err = tot - r[i]
            rows.append(r + [err / tot if tot else 0.0, f"({int(err)}.0/{int(tot)}.0)"])
        tot_err = sum(sum(r) - r[i] for i, r in enumerate(self._cm))
        tot = sum(sum(r) for r in self._cm)
        rows.append([sum(r[j] for r in self._cm) for j in range(len(self._cm))] +
                    [tot_err / tot if tot else 0.0, f"({int(tot_err)}.0/{int(tot)}.0)"])
        self.table = pd.DataFrame(rows, index=self.domains + ["Total"], columns=self.domains + ["Error", "Rate"])

    def to_list(self):
        return [[int(v) for v in r] for r in self._cm]

    def __repr__(self):
        return f"{self.table_header}\n{self.table}"


def _w(w, n, device):
    return torch.ones(n, dtype=torch.float64, device=device) if w is None else w.double()


def regression_metrics(y, pred, w=None, distribution=None) -> ModelMetrics:
    """Weighted sums only (ModelMetricsRegression.MetricBuilderRegression): row shards merge by all-reduce."""
    y, pred = y.double(), pred.double()
    w = _w(w, y.numel(), y.device)
    ok = ~torch.isnan(y) & (w > 0)
    y, pred, w = y[ok], pred[ok], w[ok]
    err = y - pred
    dev_sum = torch.zeros((), dtype=torch.float64, device=y.device)
    dev_ok = 1.0
    if distribution is not None and distribution.name not in ("gaussian",):
        f = distribution.link_fn(torch.clamp(pred, min=1e-300)) if distribution.link == "log" else pred
        try:
            dev_sum = distribution.deviance(w, y, f).sum().double()
        except Exception:  # noqa: BLE001
            dev_ok = 0.0
    log_ok = bool((y > -1).all()) and bool((pred > -1).all())
    lerr = (w * (torch.log1p(pred) - torch.log1p(y)) ** 2).sum() if log_ok else torch.zeros((), dtype=torch.float64,
                                                                                              device=y.device)
    v = torch.stack([w.sum(), (w * err * err).sum(), (w * err.abs()).sum(), (w * y).sum(), lerr, dev_sum,
                     torch.tensor(float(y.numel()), dtype=torch.float64, device=y.device),
                     torch.tensor(0.0 if log_ok else 1.0, dtype=torch.float64, device=y.device),
                     torch.tensor(1.0 - dev_ok, dtype=torch.float64, device=y.device)])
    if _dist():
        v = _allreduce(v)
    sw, se, sa, sy, sl, sd, n, nlog, ndev = v.tolist()
    if sw <= 0:
        sw = float("nan")
    ybar = sy / sw
    var_t = (w * (y - ybar) ** 2).sum().reshape(1)
    var = float(_allreduce(var_t) if _dist() else var_t) / sw
    mse, mae = se / sw, sa / sw
    r2 = 1 - mse / var if var > 0 else float("nan")
    rmsle = math.sqrt(sl / sw) if nlog == 0 and sw == sw else float("nan")
    mrd = mse
    if distribution is not None and distribution.name not in ("gaussian",) and ndev == 0:
        mrd = sd / sw
    return ModelMetrics(model_category="Regression", MSE=mse, RMSE=math.sqrt(mse), mae=mae,
                        rmsle=rmsle, r2=r2, mean_residual_deviance=mrd, nobs=int(n))


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


def binomial_metrics(y, p1, w=None, domain=("0", "1"), nbins_thresholds: int = 400) -> ModelMetrics:
    """y in {0,1}; p1 = P(class 1). Single process: exact ROC/PR AUC over the distinct scores. Row-sharded:
    ROC/PR from the merged score-lattice histogram (no row is gathered). Threshold table and gains/lift
    come from the lattice in both cases, so they are identical however the rows are split."""
    y, p1 = y.double(), p1.double()
    w = _w(w, y.numel(), y.device)
    ok = ~torch.isnan(y) & (w > 0)
    lattice = _dist() or y.numel() >= LATTICE_AUC_ROWS
    if lattice:
        # excluded rows keep their slot with weight 0 (every sum below and the score lattice ignore them): no
        # compaction pass (nonzero + three gathers) over a 10M-row frame
        w = torch.where(ok, w, 0.0)
        y = torch.where(ok, y, 0.0)
        p1 = torch.where(ok, p1, 0.0)
        nobs = ok.sum().double()
    else:
        y, p1, w = y[ok], p1[ok], w[ok]
        nobs = torch.tensor(float(y.numel()), dtype=torch.float64, device=y.device)
    pc = torch.clamp(p1, 1e-15, 1 - 1e-15)
    v = torch.stack([w.sum(), -(w * (y * torch.log(pc) + (1 - y) * torch.log(1 - pc))).sum(), (w * (y - p1) ** 2).sum(),
                     (w * y).sum(), nobs])
    if _dist():
        v = _allreduce(v)
    sw, sll, sse, sy, n = v.tolist()
    if sw <= 0:
        sw = float("nan")
    logloss, mse = sll / sw, sse / sw
    h = _score_hist(p1, None, None, y=y, w=w)
    hpos, hneg, huniq = _hist_curve(h)
    if lattice:
        # from the 2^18-bin lattice (within ~1e-6 of the exact value; H2O's AUC2 itself bins into 400): large
        # frames skip the full sort of the scores
        auc, aucpr, _, _ = _auc_from_sorted(hpos, hneg)
    else:
        order = torch.argsort(p1, descending=True)
        ps, ys, ws = p1[order], y[order], w[order]
        pos, neg, _ = _group_sorted(ps, ws * ys, ws * (1 - ys))
        auc, aucpr, _, _ = _auc_from_sorted(pos, neg)
    # thresholds table (H2O keeps <= 400 bins) over the lattice's non-empty bins
    thr_tab = _threshold_table(huniq, torch.cumsum(hpos, 0), torch.cumsum(hneg, 0), nbins_thresholds) \
        if hpos.numel() else []
    ybar = sy / sw
    var = ybar * (1 - ybar)
    r2 = 1 - mse / var if var > 0 else float("nan")
    mm = ModelMetrics(model_category="Binomial", MSE=mse, RMSE=math.sqrt(mse), logloss=logloss, AUC=auc,
                      pr_auc=aucpr, Gini=2 * auc - 1 if auc == auc else float("nan"), r2=r2, nobs=int(n),
                      domain=list(domain), thresholds_and_metric_scores=thr_tab)
    if thr_tab:
        best = max(thr_tab, key=lambda r: r["f1"])
        mm["max_f1_threshold"] = best["threshold"]
        mm["cm"] = dict(threshold=best["threshold"], table=[[best["tns"], best["fps"]], [best["fns"], best["tps"]]])
        mm["mean_per_class_error"] = 1 - best["mean_per_class_accuracy"]
        mm["max_criteria_and_metric_scores"] = {c: max(thr_tab, key=lambda r: r[c])[c] for c in THRESHOLD_CRITERIA}
    mm["gains_lift_table"] = _gains_lift_hist(hpos, hneg)
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
    th, a, b = torch.stack([uniq[idx].double(), tp[idx].double(), fp[idx].double()]).cpu().numpy()   # one copy
    # whole-table numpy (the per-row Python loop was ~1 ms of host time per scoring event)
    fn, tn = P - a, Nn - b
    ab = a + b
    z = np.zeros_like(a)
    with np.errstate(divide="ignore", invalid="ignore"):
        prec = np.where(ab > 0, a / np.where(ab > 0, ab, 1.0), 1.0)
        rec = a / P if P > 0 else z
        spec = tn / Nn if Nn > 0 else z

        def f(beta):
            d = beta ** 2 * prec + rec
            return np.where(d > 0, (1 + beta ** 2) * prec * rec / np.where(d > 0, d, 1.0), 0.0)

        den = np.sqrt(np.maximum(ab * (a + fn) * (tn + b) * (tn + fn), 1e-300))
        mcc = (a * tn - b * fn) / den
        acc = (a + tn) / (P + Nn)
    cols = dict(threshold=th, f1=f(1.0), f2=f(2.0), f0point5=f(0.5), accuracy=acc, precision=prec, recall=rec,
                specificity=spec, absolute_mcc=np.abs(mcc), min_per_class_accuracy=np.minimum(rec, spec),
                mean_per_class_accuracy=(rec + spec) / 2, tns=tn, fns=fn, fps=b, tps=a)
    keys = list(cols)
    return [dict(zip(keys, vals)) for vals in zip(*(np.asarray(cols[k], dtype=np.float64).tolist() for k in keys))]


def _gains_lift_hist(pos, neg, groups: int = 16):
    """Gains/lift table (GainsLift.java, 16 groups) from the score-lattice curve (descending bins)."""
    ws = pos + neg
    if ws.numel() == 0:
        return []
    # the two cumulative curves come to the host once (the group loop was ~50 device syncs per scoring event)
    cw = torch.cumsum(ws, 0).cpu().numpy()
    cpos = torch.cumsum(pos, 0).cpu().numpy()
    tot, tot_pos = float(cw[-1]), float(cpos[-1])
    if tot <= 0 or tot_pos <= 0:
        return []
    out = []
    for g in range(1, groups + 1):
        k = min(int(np.searchsorted(cw, g / groups * tot, side="left")), cw.size - 1)
        cum_rate = float(cpos[k] / cw[k])
        out.append(dict(group=g, cumulative_data_fraction=float(cw[k] / tot), cumulative_capture_rate=float(cpos[k]) / tot_pos,
                        cumulative_lift=cum_rate / (tot_pos / tot), cumulative_response_rate=cum_rate))
    return out


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


def multinomial_metrics(y, probs, w=None, domain=None, hit_k: int = 10, labels=None) -> ModelMetrics:
    """y: class index; probs [N, K]. Sums, the confusion matrix and hit counts merge by all-reduce.
    ``labels`` [N]: the model's predicted classes when they are not argmax(probs) (ordinal GLM)."""
    y = y.long() if not torch.is_floating_point(y) else torch.nan_to_num(y, nan=-1).long()
    w = _w(w, y.numel(), y.device)
    ok = (y >= 0) & (w > 0)
    y, probs, w = y[ok], probs[ok].double(), w[ok]
    K = probs.shape[1]
    py = torch.clamp(probs.gather(1, y[:, None]).squeeze(1), 1e-15, 1.0)
    onehot = torch.nn.functional.one_hot(y, K).double()
    pred = probs.argmax(1) if labels is None else labels.to(probs.device)[ok].long()
    from .ops.segment import segment_sum
    cm = segment_sum(y * K + pred, w, K * K)
    rank = (probs > py[:, None]).sum(1)
    hk = min(hit_k, K)
    hits = torch.stack([(w * (rank < k).double()).sum() for k in range(1, hk + 1)])
    v = torch.cat([torch.stack([w.sum(), -(w * torch.log(py)).sum(), (w * ((onehot - probs) ** 2).sum(1)).sum(),
                                torch.tensor(float(y.numel()), dtype=torch.float64, device=y.device)]), hits, cm])
    if _dist():
        v = _allreduce(v)
    sw, sll, sse, n = v[:4].tolist()
    if sw <= 0:
        sw = float("nan")
    hits = (v[4:4 + hk] / sw).tolist()
    cm = v[4 + hk:].view(K, K)
    per_class_err = 1 - torch.diag(cm) / cm.sum(1).clamp(min=1e-300)
    auc = multinomial_auc(y, probs, w) if K <= 50 else float("nan")
    mse = sse / sw
    return ModelMetrics(model_category="Multinomial", MSE=mse, RMSE=math.sqrt(mse), logloss=sll / sw,
                        mean_per_class_error=float(per_class_err.mean()), cm=dict(table=cm.cpu().tolist()),
                        hit_ratio_table=hits, nobs=int(n), domain=domain, AUC=auc)


def multinomial_auc(y, probs, w):
    """Macro one-vs-rest AUC (H2O ``MultinomialAucType.MACRO_OVR``): exact per class in one process; from
    merged per-class score-lattice histograms when the rows are sharded."""
    K = probs.shape[1]
    dist = _dist()
    if dist:
        # every rank must take the same per-class skip decision: global class totals first
        tot = _allreduce(torch.stack([torch.stack([(w * (y == k).double()).sum(), w.sum()]) for k in range(K)]))
    nb = max(1 << 12, min(1 << 16, (1 << 19) // max(K, 1)))
    aucs = []
    for k in range(K):
        yk = (y == k).double()
        if dist:
            pk, wt = float(tot[k, 0]), float(tot[k, 1])
            if pk == 0 or pk == wt:
                continue
            h = _score_hist(probs[:, k], w * yk, w * (1 - yk), nb)
            pos, neg, _ = _hist_curve(h)
            aucs.append(_auc_from_sorted(pos, neg)[0])
            continue
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


def _sum_count(x: torch.Tensor):
    v = torch.stack([x.double().sum(), torch.tensor(float(x.numel()), dtype=torch.float64, device=x.device)])
    if _dist():
        v = _allreduce(v)
    return float(v[0]), int(v[1])


def anomaly_metrics(score, w=None) -> ModelMetrics:
    s, n = _sum_count(score)
    return ModelMetrics(model_category="AnomalyDetection", mean_score=s / max(n, 1), nobs=n)


def autoencoder_metrics(err) -> ModelMetrics:
    s, n = _sum_count(err)
    return ModelMetrics(model_category="AutoEncoder", MSE=s / max(n, 1), RMSE=math.sqrt(s / max(n, 1)), nobs=n)


def make_metrics(category: str, y, preds, w=None, domain=None, distribution=None, labels=None) -> ModelMetrics:
    """preds: regression -> [N] mean; binomial -> [N] p1 or [N,2]; multinomial -> [N,K] probs (``labels``: the
    predicted classes when they are not the argmax)."""
    if category == "Binomial":
        p1 = preds[:, -1] if preds.dim() == 2 else preds
        return binomial_metrics(y, p1, w, domain or ("0", "1"))
    if category == "Multinomial":
        return multinomial_metrics(y, preds, w, domain, labels=labels)
    return regression_metrics(y, preds.reshape(-1), w, distribution)
