"""Generalized Low Rank Models (reference: ``hex/glrm/GLRM.java``, ``GlrmLoss.java``,
``GlrmRegularizer.java``, ``GlrmInitialization``).

A ≈ X·Y with X [N, k] (row representation) and Y [k, P] (archetypes), fitted by alternating
proximal-gradient steps (H2O's ``alpha`` step with adaptive increase/decrease) on the masked loss
over observed entries. Losses: Quadratic, Absolute, Huber, Poisson, Logistic, Hinge, Periodic
(numerics; categoricals are one-hot expanded and fitted with the same loss). Regularizers for X
and Y: None, Quadratic, L2, L1, NonNegative, OneSparse, UnitOneSparse, Simplex with gamma_x/gamma_y.
Init: Random, SVD (top-k GramSVD), PlusPlus (k-means++ rows), User. All tensors stay in HBM;
each half-step is two GEMMs on the [N, P] masked residual.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from .base import DataInfo, Model, make_key
from .datainfo import Expander

GLRM_DEFAULTS = dict(k=1, loss="Quadratic", multi_loss="Categorical", loss_by_col=None, loss_by_col_idx=None,
                     period=1, regularization_x="None", regularization_y="None", gamma_x=0.0, gamma_y=0.0,
                     max_iterations=1000, max_updates=2000, init_step_size=1.0, min_step_size=1e-4, seed=-1,
                     init="PlusPlus", svd_method="Randomized", user_y=None, user_x=None, expand_user_y=True,
                     impute_original=False, recover_svd=False, transform="NONE", representation_name=None)


def _loss(name, u, a, period=1):
    n = name.lower().replace("_", "")
    if n == "quadratic":
        return (u - a) ** 2
    if n == "absolute":
        return (u - a).abs()
    if n == "huber":
        d = (u - a).abs()
        return torch.where(d <= 1, 0.5 * d * d, d - 0.5)
    if n == "poisson":
        return torch.exp(u) - a * u + torch.where(a > 0, a * torch.log(a.clamp(min=1e-300)) - a, torch.zeros_like(a))
    if n == "logistic":
        return torch.log1p(torch.exp(-(2 * a - 1) * u))
    if n == "hinge":
        return torch.relu(1 - (2 * a - 1) * u)
    if n == "periodic":
        return 1 - torch.cos((a - u) * 2 * math.pi / period)
    raise ValueError(f"unknown GLRM loss {name}")


def _multi_loss(kind, U, A):
    """Loss of one categorical column's one-hot block (GlrmLoss Categorical / Ordinal): U [N, L] fitted
    scores, A [N, L] one-hot target. Categorical: (1 - u_a)_+ + sum_{j != a} (1 + u_j)_+ ; Ordinal: the
    level index a is reached by the cumulative thresholds, sum_{j < a} (1 - u_j)_+ + sum_{j >= a} (1 + u_j)_+."""
    k = kind.lower()
    if k == "categorical":
        return (torch.relu(1 - U) * A + torch.relu(1 + U) * (1 - A)).sum(1)
    if k == "ordinal":
        L = A.shape[1]
        a = A.argmax(1, keepdim=True)
        j = torch.arange(L, device=U.device)[None, :]
        below = (j < a).to(U.dtype)
        return (torch.relu(1 - U) * below + torch.relu(1 + U) * (1 - below)).sum(1)
    raise ValueError(f"unknown GLRM multi_loss {kind}")


class LossPlan:
    """Per-column losses of the expanded matrix (loss / loss_by_col / loss_by_col_idx for numeric columns,
    multi_loss for every categorical block)."""

    def __init__(self, p, ex, info):
        by = {}
        lbc, idx = p.get("loss_by_col"), p.get("loss_by_col_idx")
        if lbc:
            lbc = [lbc] if isinstance(lbc, str) else list(lbc)
            if idx is None:
                raise ValueError("loss_by_col needs loss_by_col_idx")
            idx = [idx] if isinstance(idx, (int, str)) else list(idx)
            if len(idx) != len(lbc):
                raise ValueError("loss_by_col and loss_by_col_idx must have the same length")
            for c, l in zip(idx, lbc):
                j = info.x.index(c) if isinstance(c, str) else int(c)
                by[j] = l
        self.num = {}
        for i, j in enumerate(ex.nums):
            self.num.setdefault(str(by.get(j, p["loss"])), []).append(ex.num_off + i)
        self.cat = []
        for i, j in enumerate(ex.cats):
            lo, hi = ex.cat_offsets[i], ex.cat_offsets[i] + ex.cat_sizes[i]
            self.cat.append((lo, hi, str(by.get(j, p.get("multi_loss") or "Categorical"))))
        self.period = p.get("period", 1)

    def total(self, U, A, mask):
        tot = U.new_zeros(())
        for l, cols in self.num.items():
            c = torch.as_tensor(cols, device=U.device)
            tot = tot + (mask[:, c] * _loss(l, U[:, c], A[:, c], self.period)).sum()
        for lo, hi, kind in self.cat:
            m = mask[:, lo]
            if kind.lower() in ("categorical", "ordinal"):
                tot = tot + (m * _multi_loss(kind, U[:, lo:hi], torch.nan_to_num(A[:, lo:hi]))).sum()
            else:
                tot = tot + (mask[:, lo:hi] * _loss(kind, U[:, lo:hi], A[:, lo:hi], self.period)).sum()
        return tot


def _reg_value(name, M, axis):
    n = name.lower().replace("_", "")
    if n == "none":
        return torch.zeros((), dtype=M.dtype, device=M.device)
    if n in ("quadratic", "l2"):
        return (M * M).sum() if n == "quadratic" else M.norm(dim=axis).sum()
    if n == "l1":
        return M.abs().sum()
    return torch.zeros((), dtype=M.dtype, device=M.device)   # constraint sets: handled by the prox


def _prox(name, M, step_gamma, axis):
    """Proximal operator of the regularizer along rows of X (axis=1) / columns of Y (axis=0)."""
    n = name.lower().replace("_", "")
    if n in ("none",):
        return M
    if n == "quadratic":
        return M / (1 + 2 * step_gamma)
    if n == "l2":
        nrm = M.norm(dim=axis, keepdim=True)
        return M * (1 - step_gamma / nrm.clamp(min=1e-300)).clamp(min=0)
    if n == "l1":
        return torch.sign(M) * (M.abs() - step_gamma).clamp(min=0)
    if n == "nonnegative":
        return M.clamp(min=0)
    if n in ("onesparse", "unitonesparse"):
        idx = M.argmax(dim=axis, keepdim=True)
        out = torch.zeros_like(M)
        val = torch.ones_like(M.gather(axis, idx)) if n == "unitonesparse" else M.gather(axis, idx).clamp(min=0)
        return out.scatter(axis, idx, val)
    if n == "simplex":
        # Euclidean projection onto the probability simplex along `axis`
        Mt = M if axis == 1 else M.T
        u, _ = torch.sort(Mt, dim=1, descending=True)
        css = torch.cumsum(u, 1) - 1
        ind = torch.arange(1, Mt.shape[1] + 1, device=M.device, dtype=M.dtype)
        cond = u - css / ind > 0
        rho = cond.float().cumsum(1).argmax(1, keepdim=True)
        theta = css.gather(1, rho) / (rho + 1).to(M.dtype)
        P = (Mt - theta).clamp(min=0)
        return P if axis == 1 else P.T
    raise ValueError(f"unknown GLRM regularizer {name}")


class GLRMModel(Model):
    algo = "glrm"

    def __init__(self, key, params, info):
        super().__init__(key, params, info)
        self.output["model_category"] = "DimReduction"
        self.Y = None
        self.expander = None

    @property
    def model_category(self):
        return "DimReduction"

    def _encode(self, X):
        Z = self.expander.transform(X.to(self.device)).double()
        nan_rows = torch.isnan(X.to(self.device))
        return Z, nan_rows

    def _fit_x(self, Z, mask, iters=50):
        """Best representation of new rows for the fixed archetypes (GLRM scoring)."""
        Y = self.Y.to(Z.device)
        p = self.params
        Xr = Z.new_zeros(Z.shape[0], Y.shape[0])
        step = 1.0
        for _ in range(iters):
            Xr = Xr.requires_grad_(True)
            L = self.plan.total(Xr @ Y, Z, mask) if getattr(self, "plan", None) else (mask * _loss(p["loss"], Xr @ Y, Z)).sum()
            g, = torch.autograd.grad(L, Xr)
            with torch.no_grad():
                Xr = _prox(p["regularization_x"], Xr - step * g / max(Z.shape[1], 1), step * float(p["gamma_x"]), 1)
        return Xr.detach()

    def _predict_tensor(self, X, offset=None):
        Z, _ = self._encode(X)
        mask = (~torch.isnan(Z)).double()
        Zf = torch.nan_to_num(Z)
        Xr = self._fit_x(Zf, mask)
        R = Xr @ self.Y.to(Z.device)
        ex = self.expander
        if ex.standardize and ex.nums:
            k = ex.num_off
            R[:, k:] = R[:, k:] * ex.num_sd[None, :] + ex.num_mean[None, :]
        if self.params.get("impute_original"):
            # impute_original: one column per ORIGINAL column (numerics de-transformed, categoricals = the
            # level with the highest fitted score of their one-hot block)
            cols = []
            for j in range(len(self.info.x)):
                if j in ex.cats:
                    i = ex.cats.index(j)
                    lo = ex.cat_offsets[i]
                    cols.append(R[:, lo:lo + ex.cat_sizes[i]].argmax(1).to(R.dtype))
                else:
                    cols.append(R[:, ex.num_off + ex.nums.index(j)])
            R = torch.stack(cols, 1)
        return R.float()

    def prediction_names(self):
        if self.params.get("impute_original"):
            return [f"reconstr_{n}" for n in self.info.x]
        return [f"reconstr_{n}" for n in self.expander.names]

    def archetypes(self):
        return self.Y.cpu().tolist()

    def to_state(self):
        s = super().to_state()
        s["Y"] = self.Y.cpu().tolist()
        s["expander"] = self.expander.to_state()
        return s

    def _restore(self, s):
        super()._restore(s)
        self.Y = torch.tensor(s["Y"], dtype=torch.float64)
        self.expander = Expander.from_state(self.info, s["expander"])


class GLRMTrainer:
    def __init__(self, params):
        p = dict(GLRM_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from .shared_tree import resolve_seed
        t0 = time.time()
        p = self.p
        dev = X.device
        seed = resolve_seed(p["seed"])
        gen = torch.Generator().manual_seed(seed & 0x7FFFFFFF)
        t = str(p["transform"]).upper()
        ex = Expander(info, standardize=t in ("STANDARDIZE", "NORMALIZE"), use_all_factor_levels=True,
                      center_only=(t == "DEMEAN")).fit(X)
        # missing entries are excluded from the loss: keep NaNs through the expansion
        Zfull = ex.transform(X).double()
        mask = torch.ones_like(Zfull)
        for j in ex.nums:
            col = ex.num_off + ex.nums.index(j)
            mask[:, col] = (~torch.isnan(X[j])).double()
        for i, j in enumerate(ex.cats):
            na = torch.isnan(X[j])
            lo, hi = ex.cat_offsets[i], ex.cat_offsets[i] + ex.cat_sizes[i]
            mask[na, lo:hi] = 0
        A = Zfull
        N, P = A.shape
        k = int(p["k"])
        init = str(p["init"]).lower().replace("_", "")
        if init == "user" and p.get("user_y") is not None:
            uy = p["user_y"]
            Y = torch.as_tensor(uy.as_tensor().numpy() if hasattr(uy, "as_tensor") else np.asarray(uy), dtype=torch.float64).to(dev)
        elif init == "svd":
            U, S, Vt = torch.linalg.svd(A * mask, full_matrices=False)
            Y = (S[:k, None] * Vt[:k]).clone()
        elif init == "plusplus":
            from .kmeans import KMeansTrainer
            rows = [int(torch.randint(N, (1,), generator=gen))]
            d = ((A - A[rows[0]]) ** 2 * mask).sum(1)
            for _ in range(1, k):
                pr = d / d.sum().clamp(min=1e-300)
                j = int(torch.multinomial(pr.float().cpu(), 1, generator=gen))
                rows.append(j)
                d = torch.minimum(d, ((A - A[j]) ** 2 * mask).sum(1))
            Y = A[rows].clone()
        else:
            Y = torch.randn(k, P, dtype=torch.float64, generator=gen).to(dev)
        Xr = torch.randn(N, k, dtype=torch.float64, generator=gen).to(dev) * 0.1
        if init in ("svd", "plusplus"):
            Xr = torch.linalg.lstsq(Y.T, (A * mask).T).solution.T
        rx, ry = p["regularization_x"], p["regularization_y"]
        gx, gy = float(p["gamma_x"]), float(p["gamma_y"])
        plan = LossPlan(p, ex, info)
        if p.get("user_x") is not None:        # init user_x: the initial representation
            ux = p["user_x"]
            Xr = torch.as_tensor(ux.as_tensor().numpy() if hasattr(ux, "as_tensor") else np.asarray(ux),
                                 dtype=torch.float64).to(dev).reshape(N, k)

        def objective(Xr, Y):
            return float(plan.total(Xr @ Y, A, mask) + gx * _reg_value(rx, Xr, 1) + gy * _reg_value(ry, Y, 0))

        step = float(p["init_step_size"])
        obj = objective(Xr, Y)
        it = 0
        hist = []
        max_upd = int(p.get("max_updates") or 0)
        updates = 0
        for it in range(int(p["max_iterations"])):
            if max_upd > 0 and updates >= max_upd:     # max_updates: cap on accepted + rejected steps
                break
            updates += 1
            # X half-step
            Xg = Xr.clone().requires_grad_(True)
            g, = torch.autograd.grad(plan.total(Xg @ Y, A, mask), Xg)
            Xn = _prox(rx, Xr - step * g / max(P, 1), step * gx, 1)
            Yg = Y.clone().requires_grad_(True)
            g, = torch.autograd.grad(plan.total(Xn @ Yg, A, mask), Yg)
            Yn = _prox(ry, Y - step * g / max(N, 1), step * gy, 0)
            nobj = objective(Xn, Yn)
            if nobj < obj:
                Xr, Y = Xn, Yn
                step *= 1.05
                conv = (obj - nobj) / max(abs(obj), 1e-300) < 1e-7
                obj = nobj
                hist.append(dict(iteration=it, step_size=step, objective=obj))
                if conv:
                    break
            else:
                step /= 2
                if step < float(p["min_step_size"]):
                    break
            if self.job is not None and it % 20 == 0:
                self.job.check_cancelled()
        model = GLRMModel(model_key or make_key("glrm"), p, info)
        model.device = dev
        model.expander = ex
        model.Y = Y
        model.plan = plan
        if p.get("recover_svd"):
            # GLRM.recoverSVD: SVD of the rank-k product X Y (singular values and right vectors)
            _, Sv, Vt = torch.linalg.svd(Xr @ Y, full_matrices=False)
            model.output["singular_vals"] = Sv[:k].cpu().tolist()
            model.output["eigenvectors"] = Vt[:k].T.cpu().tolist()
        model.output.update(objective=obj, iterations=it + 1, step_size=step, archetypes=Y.cpu().tolist(),
                            names_expanded=ex.names, scoring_history=hist)
        from ..frame import H2OFrame
        rep = H2OFrame.from_tensor(Xr.float(), [f"Arch{i + 1}" for i in range(k)])
        model.output["representation_name"] = rep.frame_id
        model.output["training_metrics"] = dict(model_category="DimReduction", numerr=float((mask * (Xr @ Y - A) ** 2).sum()),
                                                 nobs=N)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
