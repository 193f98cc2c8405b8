"""Generalized Additive Models (reference: ``hex/gam/GAM.java``, ``GAMModel.java``,
``hex/gam/MatrixFrameUtils/GamUtils.java`` (spline bases and penalty matrices)).

Each ``gam_columns`` entry is replaced by a cubic B-spline basis (``num_knots`` knots at quantiles,
sum-to-zero centered like H2O's identifiability constraint) with a second-difference smoothness
penalty ``scale·DᵀD`` on its coefficients; the penalized GLM (all families) is then fitted by the
IRLSM solver with the penalty added to the device Gram. ``keep_gam_cols`` exposes the basis
columns; scoring rebuilds the basis from the stored knots.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .base import DataInfo, Model, make_key

GAM_DEFAULTS = dict(gam_columns=None, num_knots=None, scale=None, bs=None, knot_ids=None, keep_gam_cols=False,
                    standardize=False, family="AUTO", lambda_=0.0, alpha=0.0, seed=-1)


def bspline_basis(x, knots, degree=3):
    """Cox–de Boor B-spline basis for 1-D tensor x; knots include boundaries (clamped)."""
    t = torch.cat([knots[:1].repeat(degree), knots, knots[-1:].repeat(degree)])
    xc = x.clamp(float(knots[0]), float(knots[-1]))
    nb = len(t) - 1
    B = ((xc[:, None] >= t[None, :-1]) & (xc[:, None] < t[None, 1:])).double()
    last = (xc == t[-1])
    if last.any():
        idx = int(torch.nonzero(t[:-1] < t[1:]).flatten()[-1])
        B[last, :] = 0
        B[last, idx] = 1
    for k in range(1, degree + 1):
        n = nb - k
        left_den = t[k:k + n] - t[:n]
        right_den = t[k + 1:k + 1 + n] - t[1:1 + n]
        a = torch.where(left_den > 0, (xc[:, None] - t[None, :n]) / left_den.clamp(min=1e-300)[None, :], torch.zeros(1, dtype=torch.float64, device=x.device))
        b = torch.where(right_den > 0, (t[None, k + 1:k + 1 + n] - xc[:, None]) / right_den.clamp(min=1e-300)[None, :], torch.zeros(1, dtype=torch.float64, device=x.device))
        B = a * B[:, :n] + b * B[:, 1:n + 1]
    return B


class GAMModel(Model):
    algo = "gam"

    def _expand(self, X):
        rows = []
        for j in range(len(self.base_x)):
            rows.append(X[self.col_index[self.base_x[j]]])
        out = [X[self.col_index[n]].double() for n in self.lin_x]
        for g in self.gams:
            x = X[self.col_index[g["col"]]].double()
            B = bspline_basis(torch.nan_to_num(x, nan=g["mean"]), torch.as_tensor(g["knots"], dtype=torch.float64, device=X.device))
            B = B - torch.as_tensor(g["center"], dtype=torch.float64, device=X.device)[None, :]
            out += [B[:, i] for i in range(B.shape[1])]
        return torch.stack(out, 0).float()

    def _predict_tensor(self, X, offset=None):
        return self.glm._predict_tensor(self._expand(X.to(self.device)), offset)

    def coef(self):
        return self.glm.output["coefficients"]


class GAMTrainer:
    def __init__(self, params):
        p = dict(GAM_DEFAULTS)
        if "lambda" in params:
            params = dict(params)
            params["lambda_"] = params.pop("lambda")
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from .glm import GLMTrainer
        t0 = time.time()
        p = self.p
        gcols = p["gam_columns"]
        if not gcols:
            raise ValueError("GAM needs gam_columns")
        gcols = [g if isinstance(g, str) else g[0] for g in gcols]
        nk = p["num_knots"] or [10] * len(gcols)
        sc = p["scale"] or [0.001] * len(gcols)
        col_index = {n: j for j, n in enumerate(info.x)}
        lin = [n for n in info.x if n not in gcols]
        lin_cat = [n for n in lin if info.iscat[col_index[n]]]
        if lin_cat:
            raise ValueError("GAM here supports numeric linear predictors only; encode categoricals first")
        gams, names = [], list(lin)
        for g, k, s in zip(gcols, nk, sc):
            x = X[col_index[g]].double()
            ok = ~torch.isnan(x)
            qs = torch.quantile(x[ok][: 1 << 22], torch.linspace(0, 1, int(k), dtype=torch.float64, device=x.device))
            knots = torch.unique(qs)
            B = bspline_basis(torch.nan_to_num(x, nan=float(x[ok].mean())), knots)
            center = B.mean(0)
            gams.append(dict(col=g, knots=knots.cpu().tolist(), center=center.cpu().tolist(), mean=float(x[ok].mean()),
                             scale=float(s), nb=B.shape[1]))
            names += [f"{g}_{i}" for i in range(B.shape[1])]
        model = GAMModel(model_key or make_key("gam"), p, info)
        model.device = X.device
        model.base_x = list(info.x)
        model.col_index = col_index
        model.lin_x = lin
        model.gams = gams
        Xg = model._expand(X)
        ginfo = DataInfo(names, np.zeros(len(names), np.int32), [None] * len(names), info.response, info.response_domain)
        P1 = len(names) + 1
        pen = torch.zeros(P1, P1, dtype=torch.float64)
        off = len(lin)
        for g in gams:
            nb = g["nb"]
            D = torch.diff(torch.eye(nb, dtype=torch.float64), n=2, dim=0)
            pen[off:off + nb, off:off + nb] = g["scale"] * (D.T @ D)
            off += nb
        gp = {k: v for k, v in p.items() if k not in ("gam_columns", "num_knots", "scale", "bs", "knot_ids", "keep_gam_cols")}
        tr = GLMTrainer(gp)
        tr.penalty = pen
        glm = tr.fit(Xg, y, w, offset, ginfo, None)
        model.glm = glm
        model.output["coefficients"] = glm.output["coefficients"]
        model.output["knots"] = {g["col"]: g["knots"] for g in gams}
        model.output["training_metrics"] = model.metrics_for(X, y, w, offset)
        if valid is not None:
            Xv, yv, wv, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv, ov)
        if p["keep_gam_cols"]:
            from ..frame import H2OFrame
            model.output["gam_transformed_center_key"] = H2OFrame.from_tensor(Xg.T, names).frame_id
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
