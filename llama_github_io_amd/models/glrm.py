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

from ..parallel import collectives as coll
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


def _red(t):
    """Sum over every rank's rows (no-op in one process)."""
    if not coll.is_dist():
        return t
    return coll.all_reduce_(t.contiguous().to(coll.comm_device())).to(t.device)


def _top_svd_from_gram(G, k):
    """Top-k singular values / right vectors of a tall matrix from its Gram (sign: largest |entry| > 0)."""
    ev, V = torch.linalg.eigh(G)
    ev, V = ev.flip(0)[:k].clamp(min=0), V.flip(1)[:, :k]
    sgn = torch.sign(V.gather(0, V.abs().argmax(0, keepdim=True)))
    V = V * torch.where(sgn == 0, torch.ones_like(sgn), sgn)
    return ev.sqrt(), V.T


def _row_normals(seed, stream, row0, n, k, dev):
    """Standard normals [n, k] drawn per GLOBAL row (Box-Muller on counter-based uniforms): the same
    initial representation however the rows are split."""
    cols = []
    for j in range(k):
        u1 = coll.row_uniform(seed, stream + 2 * j, row0, n, dev).clamp(min=1e-300)
        u2 = coll.row_uniform(seed, stream + 2 * j + 1, row0, n, dev)
        cols.append(torch.sqrt(-2 * torch.log(u1)) * torch.cos(2 * math.pi * u2))
    return torch.stack(cols, 1) if cols else torch.zeros(n, 0, dtype=torch.float64, device=dev)


def _pick_row(d, u, A, row0):
    """Row of A at the global inverse-CDF position u * sum(d) (k-means++ draw over row shards)."""
    tot = float(_red(d.sum().reshape(1)))
    cs = torch.cumsum(d, 0)
    off = 0.0
    if coll.is_dist():
        sums = coll.all_gather_object(float(cs[-1]) if cs.numel() else 0.0)
        off = sum(sums[:coll.rank()])
    target = u * tot
    row = torch.zeros(A.shape[1], dtype=A.dtype, device=A.device)
    hit = torch.zeros(1, dtype=torch.float64, device=A.device)
    owner = (cs.numel() > 0 and off < target <= off + float(cs[-1])) or (target <= 0 and row0 == 0 and cs.numel() > 0)
    if owner:
        j = int(torch.searchsorted(cs, torch.tensor([target - off], dtype=cs.dtype, device=cs.device)).clamp(
            max=cs.numel() - 1))
        row = A[j].clone()
        hit[0] = 1.0
    row, hit = _red(row), _red(hit)
    return row / max(float(hit), 1.0)


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

    @staticmethod
    def _user_y(U, ex, info, k, P, expand):
        """Initial archetypes from user_y (GLRM.java:187,400-425). ``expand_user_y`` (default): user_y holds the
        ORIGINAL columns (categoricals as level indices) and is expanded — one-hot categoricals first, then the
        numerics, as DataInfo permutes them; otherwise user_y already holds the P expanded columns."""
        if U.shape[0] != k:
            raise ValueError(f"The user-specified Y must have k = {k} rows")
        if not expand:
            if U.shape[1] != P:
                raise ValueError(f"The user-specified Y must have the same number of columns ({P}) as the "
                                 "training observations")
            return U.clone()
        if U.shape[1] != info.F:
            raise ValueError(f"The user-specified Y must have the same number of columns ({info.F}) as the "
                             "training observations")
        Y = torch.zeros(k, P, dtype=torch.float64, device=U.device)
        for i, j in enumerate(ex.cats):
            lv = torch.nan_to_num(U[:, j], nan=-1).long() - (0 if ex.use_all else 1)
            lo, n = ex.cat_offsets[i], ex.cat_sizes[i]
            for r in range(k):
                if 0 <= int(lv[r]) < n:
                    Y[r, lo + int(lv[r])] = 1.0
        for t, j in enumerate(ex.nums):
            Y[:, ex.num_off + t] = U[:, j]
        return Y

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from .shared_tree import resolve_seed
        t0 = time.time()
        p = self.p
        dev = X.device
        seed = resolve_seed(p["seed"])
        gen = torch.Generator().manual_seed(seed & 0x7FFFFFFF)
        t = str(p["transform"]).upper()
        dist_ = coll.is_dist()
        ex = Expander(info, standardize=t in ("STANDARDIZE", "NORMALIZE"), use_all_factor_levels=True,
                      center_only=(t == "DEMEAN")).fit(X, reduce=coll.all_reduce_ if dist_ else None)
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
        # row-sharded (GLRM.java's MRTasks): X stays with its rows, Y and every sum over rows (objective,
        # Y gradient, Gram of the SVD init) are all-reduced -> the single-process archetypes on every rank
        row0 = coll.row_offset(N) if dist_ else 0
        Ng = int(coll.all_reduce_scalar(N)) if dist_ else N
        k = int(p["k"])
        init = str(p["init"]).lower().replace("_", "")
        if init == "user" and p.get("user_y") is not None:
            uy = p["user_y"]
            U = torch.as_tensor(uy.as_tensor().numpy() if hasattr(uy, "as_tensor") else np.asarray(uy),
                                dtype=torch.float64).to(dev)
            Y = self._user_y(U, ex, info, k, P, bool(p.get("expand_user_y", True)))
        elif init == "svd":
            Am = torch.nan_to_num(A) * mask
            S, Vt = _top_svd_from_gram(_red(Am.T @ Am), k)
            Y = (S[:, None] * Vt).clone()
        elif init == "plusplus":
            Af = torch.nan_to_num(A)
            first = int(torch.randint(Ng, (1,), generator=gen))
            y0 = torch.zeros(P, dtype=A.dtype, device=dev)
            if row0 <= first < row0 + N:
                y0 = Af[first - row0].clone()
            ys = [_red(y0)]
            d = ((Af - ys[0]) ** 2 * mask).sum(1)
            for _ in range(1, k):
                u = float(torch.rand(1, generator=gen, dtype=torch.float64))
                yj = _pick_row(d, u, Af, row0)
                ys.append(yj)
                d = torch.minimum(d, ((Af - yj) ** 2 * mask).sum(1))
            Y = torch.stack(ys, 0)
        else:
            Y = torch.randn(k, P, dtype=torch.float64, generator=gen).to(dev)
        Xr = _row_normals(seed, 0x61A5, row0, N, k, dev) * 0.1
        if init in ("svd", "plusplus"):
            Xr = torch.linalg.lstsq(Y.T, (A * mask).T).solution.T
        rx, ry = p["regularization_x"], p["regularization_y"]
        gx, gy = float(p["gamma_x"]), float(p["gamma_y"])
        plan = LossPlan(p, ex, info)
        if p.get("user_x") is not None:        # init user_x: the initial representation (this rank's rows)
            ux = p["user_x"]
            ua = torch.as_tensor(ux.as_tensor().numpy() if hasattr(ux, "as_tensor") else np.asarray(ux),
                                 dtype=torch.float64).reshape(-1, k)
            if ua.shape[0] == Ng and Ng != N:
                ua = ua[row0:row0 + N]
            Xr = ua.to(dev).reshape(N, k)

        def objective(Xr, Y):
            local = plan.total(Xr @ Y, A, mask) + gx * _reg_value(rx, Xr, 1)
            return float(_red(local.reshape(1))) + float(gy * _reg_value(ry, Y, 0))

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
            g = _red(g)
            Yn = _prox(ry, Y - step * g / max(Ng, 1), step * gy, 0)
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
            # (X Y)^T (X Y) = Y^T (X^T X) Y with the k x k X^T X summed over the row shards
            Sv, Vt = _top_svd_from_gram(Y.T @ _red(Xr.T @ Xr) @ Y, k)
            model.output["singular_vals"] = Sv.cpu().tolist()
            model.output["eigenvectors"] = Vt.T.cpu().tolist()
        model.output.update(objective=obj, iterations=it + 1, step_size=step, archetypes=Y.cpu().tolist(),
                            names_expanded=ex.names, scoring_history=hist)
        import contextlib
        from ..frame import H2OFrame
        from ..parallel import dframe
        ctx = dframe.shard_ctx(dframe.make_shard(N)) if dist_ else contextlib.nullcontext()
        with ctx:                     # the representation keeps the training frame's row distribution
            rep = H2OFrame.from_tensor(Xr.float(), [f"Arch{i + 1}" for i in range(k)])
        model.output["representation_name"] = rep.frame_id
        numerr = float(_red((mask * torch.nan_to_num(Xr @ Y - A) ** 2).sum().reshape(1)))
        model.output["training_metrics"] = dict(model_category="DimReduction", numerr=numerr, nobs=Ng)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
