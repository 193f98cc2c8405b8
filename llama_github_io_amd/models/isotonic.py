"""Isotonic regression (reference: ``hex/isotonic/IsotonicRegression.java``, ``PoolAdjacentViolators``).

Weighted pool-adjacent-violators on the rows sorted by the single predictor, thresholds kept as (x, y)
knots; scoring interpolates linearly between knots on device; ``out_of_bounds`` = NA (default) or clip.

Row-sharded training follows the reference's two-stage driver
(``hex/isotonic/PoolAdjacentViolatorsDriver.java`` runPAV: sort, PAV per chunk, PAV again over the chunk
results) without moving rows to one place: each rank folds its rows to (x, sum w, sum w*y) per distinct x,
exact order-statistic splitters cut the x axis into one contiguous range per rank, one all-to-all sends each
distinct x to its range's owner, every rank pools its range (valid: a range is a contiguous run of the
sorted axis), and a final PAV over the ranks' pooled blocks — the model-sized summary the reference also
collects into one chunk — gives the same fit on every rank.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from ..parallel import collectives as coll
from ..parallel.order_stats import order_statistics
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


def pava_blocks(y, w, xlo, xhi):
    """Weighted PAV over ordered blocks (value, weight, first x, last x): the pooled blocks, as arrays."""
    v, ww, lo, hi = [], [], [], []
    for yi, wi, a, b in zip(y, w, xlo, xhi):
        v.append(yi); ww.append(wi); lo.append(a); hi.append(b)
        while len(v) > 1 and v[-2] > v[-1]:
            v2, w2, h2 = v.pop(), ww.pop(), hi.pop()
            lo.pop()
            s = ww[-1] + w2
            v[-1] = (v[-1] * ww[-1] + v2 * w2) / s if s > 0 else v[-1]
            ww[-1], hi[-1] = s, h2
    return np.array(v), np.array(ww), np.array(lo), np.array(hi)


def _fold(x, w, wy):
    """Rows -> (sorted distinct x, sum w, sum w*y)."""
    ux, inv = torch.unique(x, return_inverse=True)
    return (ux, torch.zeros_like(ux).index_add_(0, inv, w), torch.zeros_like(ux).index_add_(0, inv, wy))


def _owned_range(ux, sw, swy):
    """Send each distinct x to the rank owning its range of the global x axis (splitters = exact order
    statistics of the distinct-x entries, so ranges hold about equally many); returns this rank's entries."""
    W = coll.world()
    n = torch.tensor([float(ux.numel())], dtype=torch.float64)
    M = int(coll.all_reduce_(n.to(coll.comm_device())).item())
    targets = [k * M // W + 1 for k in range(1, W)]
    spl = order_statistics(ux, targets) if M else []
    spl = torch.tensor([s for s in spl], dtype=torch.float64, device=ux.device)
    dest = torch.searchsorted(spl, ux.contiguous(), right=True) if len(spl) else torch.zeros_like(ux, dtype=torch.long)
    got = coll.exchange_rows(torch.stack([ux, sw, swy], 1), dest)
    return _fold(got[:, 0], got[:, 1], got[:, 2])


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
        ux, sw, swy = _fold(x, w, w * yy)
        if coll.is_dist():
            ux, sw, swy = _owned_range(ux, sw, swy)
        uxn = ux.cpu().numpy()
        blk = np.stack(pava_blocks((swy / sw).cpu().numpy(), sw.cpu().numpy(), uxn, uxn), 1) \
            if len(uxn) else np.zeros((0, 4))
        if coll.is_dist():
            # ranks own consecutive x ranges, so rank order is x order; the blocks are the compressed PAV
            # summary (model-sized), the final pass pools across the range boundaries
            blk = coll.all_gather_cat(torch.from_numpy(np.ascontiguousarray(blk)).to(coll.comm_device()),
                                      bounded=True).cpu().numpy()
            blk = np.stack(pava_blocks(blk[:, 0], blk[:, 1], blk[:, 2], blk[:, 3]), 1)
        if not len(blk):
            raise ValueError("isotonic regression needs at least one row with a non-NA x, y and weight > 0")
        # knots where the fitted step function changes: the first and last x of each run of equal values
        v, lo, hi = blk[:, 0], blk[:, 2], blk[:, 3]
        start = np.r_[True, v[1:] != v[:-1]]
        end = np.r_[v[1:] != v[:-1], True]
        kx, ky = [], []
        for i in range(len(v)):
            if start[i]:
                kx.append(lo[i]); ky.append(v[i])
            if end[i]:
                j = i
                if hi[j] != kx[-1]:
                    kx.append(hi[j]); ky.append(v[j])
        model = IsotonicModel(model_key or make_key("isotonic"), self.p, info)
        model.device = X.device
        model.thresholds_x = [float(a) for a in kx]
        model.thresholds_y = [float(a) for a in ky]
        model.output["thresholds_x"] = model.thresholds_x
        model.output["thresholds_y"] = model.thresholds_y
        model.output["training_metrics"] = model.metrics_for(X, y, None)
        if valid is not None:
            Xv, yv, wv, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv, ov)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
