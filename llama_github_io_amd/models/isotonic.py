"""Isotonic regression (reference: ``hex/isotonic/IsotonicRegression.java``, ``PoolAdjacentViolators``).

Weighted pool-adjacent-violators on the rows sorted by the single predictor (device sort, host
PAVA over unique x — linear time), thresholds kept as (x, y) knots; scoring interpolates linearly
between knots on device; ``out_of_bounds`` = NA (default) or clip.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .base import DataInfo, Model, make_key


def pava(y, w):
    """Weighted PAVA; returns fitted block values per input position (non-decreasing)."""
    vals, wts, counts = [], [], []
    for yi, wi in zip(y, w):
        vals.append(yi); wts.append(wi); counts.append(1)
        while len(vals) > 1 and vals[-2] > vals[-1]:
            v2, w2, c2 = vals.pop(), wts.pop(), counts.pop()
            v1, w1, c1 = vals.pop(), wts.pop(), counts.pop()
            ww = w1 + w2
            vals.append((v1 * w1 + v2 * w2) / ww if ww > 0 else v1); wts.append(ww); counts.append(c1 + c2)
    return np.repeat(vals, counts)


class IsotonicModel(Model):
    algo = "isotonicregression"

    def _predict_tensor(self, X, offset=None):
        x = X[0].double().to(self.device)
        tx = torch.as_tensor(self.thresholds_x, dtype=torch.float64, device=x.device)
        ty = torch.as_tensor(self.thresholds_y, dtype=torch.float64, device=x.device)
        clip = str(self.params.get("out_of_bounds", "NA")).lower() == "clip"
        xc = x.clamp(tx[0], tx[-1]) if clip else x
        i = torch.searchsorted(tx, xc.contiguous(), right=True).clamp(1, len(tx) - 1)
        x0, x1, y0, y1 = tx[i - 1], tx[i], ty[i - 1], ty[i]
        t = torch.where(x1 > x0, (xc - x0) / (x1 - x0), torch.zeros_like(xc))
        out = y0 + t * (y1 - y0)
        out = torch.where(xc == tx[-1], ty[-1], out)
        if not clip:
            out = torch.where((x < tx[0]) | (x > tx[-1]) | torch.isnan(x), torch.full_like(out, float("nan")), out)
        return out.float()

    def to_state(self):
        s = super().to_state()
        s["tx"], s["ty"] = list(self.thresholds_x), list(self.thresholds_y)
        return s

    def _restore(self, s):
        super()._restore(s)
        self.thresholds_x, self.thresholds_y = s["tx"], s["ty"]


class IsotonicTrainer:
    def __init__(self, params):
        p = dict(out_of_bounds="NA", custom_metric_func=None)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        if info.F != 1:
            raise ValueError("isotonic regression takes exactly one predictor column")
        t0 = time.time()
        x = X[0].double()
        N = x.numel()
        w = torch.ones(N, dtype=torch.float64, device=x.device) if w is None else w.double()
        ok = ~torch.isnan(x) & ~torch.isnan(y) & (w > 0)
        x, yy, w = x[ok], y.double()[ok], w[ok]
        ux, inv = torch.unique(x, return_inverse=True)
        sw = torch.zeros_like(ux).index_add_(0, inv, w)
        swy = torch.zeros_like(ux).index_add_(0, inv, w * yy)
        yb = (swy / sw).cpu().numpy()
        fit = pava(yb, sw.cpu().numpy())
        uxn = ux.cpu().numpy()
        # keep only knots where the fitted step function changes (+ ends)
        keep = np.ones(len(fit), dtype=bool)
        if len(fit) > 2:
            keep[1:-1] = ~((fit[1:-1] == fit[:-2]) & (fit[1:-1] == fit[2:]))
        model = IsotonicModel(model_key or make_key("isotonic"), self.p, info)
        model.device = X.device
        model.thresholds_x = uxn[keep].tolist()
        model.thresholds_y = fit[keep].tolist()
        model.output["thresholds_x"] = model.thresholds_x
        model.output["thresholds_y"] = model.thresholds_y
        model.output["training_metrics"] = model.metrics_for(X, y, None)
        if valid is not None:
            Xv, yv, wv, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv, ov)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
