"""Quantiles (reference: ``hex/quantile/Quantile.java``, ``QuantileModel.java``: probs,
``combine_method`` INTERPOLATE / AVERAGE / LOW / HIGH, ``weights_column``).

H2O computes exact quantiles by iterative histogram refinement over the distributed column. In one
process the column fits in HBM, so a single device sort gives the exact order statistics; a row-sharded
column runs the refinement (``parallel/order_stats.py``: <= 6 passes, one small all-reduce each) and
gets the same values without gathering rows. With weights the quantile is taken on the cumulative
weight (rows with weight w count w times).
"""
from __future__ import annotations

import math

import torch

from .base import DataInfo, Model, make_key


def weighted_quantiles(v: torch.Tensor, probs, method: str = "interpolate", w: torch.Tensor | None = None):
    method = str(method).lower()
    v = v.double()
    ok = ~torch.isnan(v)
    if w is not None:
        w = w.double().to(v.device)
        ok &= ~torch.isnan(w) & (w > 0)
    x = v[ok]
    p = torch.as_tensor(probs, dtype=torch.float64, device=v.device)
    from ..parallel import collectives as coll
    if coll.is_dist():
        return _dist_quantiles(x, p, method, None if w is None else w[ok])
    if x.numel() == 0:
        return torch.full((p.numel(),), float("nan"), dtype=torch.float64, device=v.device)
    if w is None:
        xs, _ = torch.sort(x)
        n = xs.numel()
        pos = p * (n - 1)                     # H2O: index = p * (n - 1)
        lo = torch.floor(pos).long().clamp(0, n - 1)
        hi = torch.ceil(pos).long().clamp(0, n - 1)
        a, b = xs[lo], xs[hi]
        if method == "low":
            return a
        if method == "high":
            return b
        if method == "average":
            return torch.where(lo == hi, a, (a + b) / 2)
        return a + (pos - lo.double()) * (b - a)
    ws = w[ok]
    order = torch.argsort(x)
    xs, ws = x[order], ws[order]
    cw = torch.cumsum(ws, 0)
    total = cw[-1]
    pos = p * (total - 1)                     # weighted rank (rows weighted w count w times)
    lo = torch.searchsorted(cw, (torch.floor(pos) + 1).contiguous()).clamp(max=xs.numel() - 1)
    hi = torch.searchsorted(cw, (torch.ceil(pos) + 1).contiguous()).clamp(max=xs.numel() - 1)
    a, b = xs[lo], xs[hi]
    if method == "low":
        return a
    if method == "high":
        return b
    if method == "average":
        return torch.where(lo == hi, a, (a + b) / 2)
    return a + (pos - torch.floor(pos)) * (b - a)


def _dist_quantiles(x, p, method, ws):
    """Row-sharded ``weighted_quantiles``: the same rank arithmetic, order statistics by refinement."""
    from ..parallel import collectives as coll
    from ..parallel.order_stats import order_statistics
    tot = torch.tensor([float(x.numel()), float(ws.sum()) if ws is not None else 0.0], dtype=torch.float64)
    tot = coll.all_reduce_(tot.to(coll.comm_device())).cpu()
    n = tot[0].item()
    if n == 0:
        return torch.full((p.numel(),), float("nan"), dtype=torch.float64, device=x.device)
    pc = p.cpu()
    if ws is None:
        pos = pc * (n - 1)
        lo = torch.floor(pos).clamp(0, n - 1)
        hi = torch.ceil(pos).clamp(0, n - 1)
        tl, th = (lo + 1).tolist(), (hi + 1).tolist()
    else:
        total = tot[1].item()
        pos = pc * (total - 1)
        tl, th = (torch.floor(pos) + 1).tolist(), (torch.ceil(pos) + 1).tolist()
        lo = torch.floor(pos)
    vals = order_statistics(x, tl + th, ws)
    a = torch.tensor(vals[: len(tl)], dtype=torch.float64)
    b = torch.tensor(vals[len(tl):], dtype=torch.float64)
    if method == "low":
        out = a
    elif method == "high":
        out = b
    elif method == "average":
        out = torch.where(a == b, a, (a + b) / 2)
    else:
        out = a + (pos - lo) * (b - a)
    return out.to(x.device)


class QuantileModel(Model):
    algo = "quantile"

    def _predict_tensor(self, X, offset=None):
        raise NotImplementedError("the quantile model has no predict; read output['quantiles']")


class QuantileTrainer:
    def __init__(self, params):
        p = dict(probs=[0.001, 0.01, 0.1, 0.25, 0.333, 0.5, 0.667, 0.75, 0.9, 0.99, 0.999], combine_method="interpolate")
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        m = QuantileModel(model_key or make_key("quantile"), self.p, info)
        m.device = X.device
        m.output["model_category"] = "Unsupervised"
        m.output["quantiles"] = {info.x[j]: weighted_quantiles(X[j], self.p["probs"], self.p["combine_method"], w).cpu().tolist()
                                 for j in range(info.F) if not info.iscat[j]}
        return m
