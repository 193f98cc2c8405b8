"""Generalized Additive Models (reference: ``hex/gam/GAM.java``, ``GAMModel.java``,
``hex/gam/GamSplines/*`` and ``hex/gam/MatrixFrameUtils/Gen*GamOneColumn.java``).

Smoother families (``bs`` per ``gam_columns`` entry, as in the reference):

* ``0`` cubic regression spline (the default): the natural-cubic "cardinal" basis on ``num_knots``
  quantile knots, f(x) = a⁻β_j + a⁺β_{j+1} + c⁻δ_j + c⁺δ_{j+1} with δ = [0; B⁻¹D; 0]β, and penalty
  S = DᵀB⁻¹D; the sum-to-zero identifiability constraint is a QR reparameterisation (X Z, ZᵀSZ),
  which drops one column.
* ``1`` thin-plate regression spline with knots, for one or several columns jointly: radial basis
  η(‖x − k_j‖) (r^{2m−d}, ×log r in even dimension) plus the polynomial null space of degree m−1;
  the radial coefficients are constrained orthogonal to the polynomials at the knots (QR), penalty =
  the η kernel matrix among the knots; then centred like the CR smoothers.
* ``2`` monotone I-splines of order ``spline_orders``: integrated M-splines (values in [0, 1]), with
  non-negative coefficients when ``splines_non_negative`` (the default) — a monotone increasing fit;
  penalty on second differences; not centred (it would break monotonicity).
* ``3`` M-splines (normalised B-splines) of order ``spline_orders``, centred, second-difference
  penalty.

Categorical (and any other) linear predictors are expanded by the GLM; every smoother's penalty
``scale · S`` enters the penalized IRLSM solve on the device Gram (coefficient bounds for I-splines).
Scoring rebuilds the bases from the stored knots / transforms.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from ..parallel import collectives as coll
from .base import DataInfo, Model, make_key

GAM_DEFAULTS = dict(gam_columns=None, num_knots=None, scale=None, bs=None, knot_ids=None, keep_gam_cols=False,
                    spline_orders=None, splines_non_negative=None, standardize=False, family="AUTO", lambda_=0.0,
                    alpha=0.0, seed=-1, scale_tp_penalty_mat=False, standardize_tp_gam_cols=False)


# ------------------------------------------------------------------------------------------------ B-splines
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
        zero = torch.zeros(1, dtype=torch.float64, device=x.device)
        a = torch.where(left_den > 0, (xc[:, None] - t[None, :n]) / left_den.clamp(min=1e-300)[None, :], zero)
        b = torch.where(right_den > 0, (t[None, k + 1:k + 1 + n] - xc[:, None]) / right_den.clamp(min=1e-300)[None, :], zero)
        B = a * B[:, :n] + b * B[:, 1:n + 1]
    return B


def mspline_basis(x, knots, order):
    """Normalised B-splines (M-splines, NBSplinesTypeI): M_i = order·B_i / (t_{i+order} − t_i)."""
    deg = order - 1
    B = bspline_basis(x, knots, deg)
    t = torch.cat([knots[:1].repeat(deg), knots, knots[-1:].repeat(deg)])
    span = (t[order:order + B.shape[1]] - t[:B.shape[1]]).clamp(min=1e-300)
    return B * (order / span)[None, :]


def ispline_basis(x, knots, order):
    """I-splines: I_i(x) = Σ_{j ≥ i} B_{j, order+1}(x) (integrated M-splines), dropping the constant first
    column (it is 1 everywhere and aliases the intercept)."""
    B = bspline_basis(x, knots, order)          # order+1 = degree order
    cs = torch.flip(torch.cumsum(torch.flip(B, [1]), 1), [1])
    return cs[:, 1:]


def _diff_penalty(nb):
    D = torch.diff(torch.eye(nb, dtype=torch.float64), n=2, dim=0) if nb > 2 else torch.zeros(0, nb, dtype=torch.float64)
    return D.T @ D


# ------------------------------------------------------------------------------------------------ cubic regression
def _cr_mats(knots):
    """D ((k−2)×k), B ((k−2)×(k−2)), F = [0; B⁻¹D; 0] and S = DᵀB⁻¹D of the cardinal cubic basis."""
    k = knots.numel()
    h = knots[1:] - knots[:-1]
    D = torch.zeros(k - 2, k, dtype=torch.float64)
    Bm = torch.zeros(k - 2, k - 2, dtype=torch.float64)
    for i in range(k - 2):
        D[i, i] = 1 / h[i]
        D[i, i + 1] = -1 / h[i] - 1 / h[i + 1]
        D[i, i + 2] = 1 / h[i + 1]
        Bm[i, i] = (h[i] + h[i + 1]) / 3
        if i < k - 3:
            Bm[i, i + 1] = Bm[i + 1, i] = h[i + 1] / 6
    BinvD = torch.linalg.solve(Bm, D) if k > 2 else torch.zeros(0, k, dtype=torch.float64)
    F = torch.cat([torch.zeros(1, k, dtype=torch.float64), BinvD, torch.zeros(1, k, dtype=torch.float64)])
    S = D.T @ BinvD
    return F, S


def cr_basis(x, knots, F):
    """Rows of the cardinal natural cubic basis (x clamped to the knot range)."""
    kn = knots.to(x.device)
    Fd = F.to(x.device)
    xc = x.clamp(float(kn[0]), float(kn[-1]))
    j = torch.clamp(torch.searchsorted(kn, xc, right=True) - 1, 0, kn.numel() - 2)
    xl, xr = kn[j], kn[j + 1]
    h = xr - xl
    am = (xr - xc) / h
    ap = (xc - xl) / h
    cm = ((xr - xc) ** 3 / h - h * (xr - xc)) / 6
    cp = ((xc - xl) ** 3 / h - h * (xc - xl)) / 6
    n, k = xc.numel(), kn.numel()
    X = cm[:, None] * Fd[j] + cp[:, None] * Fd[j + 1]
    rows = torch.arange(n, device=x.device)
    X[rows, j] += am
    X[rows, j + 1] += ap
    return X


# ------------------------------------------------------------------------------------------------ thin plate
def _tp_m(d):
    return d // 2 + 1 if (2 * (d // 2 + 1) > d) else d // 2 + 2      # smallest m with 2m > d


def _tp_eta(r, m, d):
    p = 2 * m - d
    if d % 2 == 0:
        c = ((-1) ** (m + 1 + d // 2)) / (2 ** (2 * m - 1) * math.pi ** (d / 2) * math.factorial(m - 1)
                                         * math.factorial(m - d // 2))
        return c * torch.where(r > 0, r ** p * torch.log(r.clamp(min=1e-300)), torch.zeros_like(r))
    c = math.gamma(d / 2 - m) / (2 ** (2 * m) * math.pi ** (d / 2) * math.factorial(m - 1))
    return c * r ** p


def _tp_poly_exps(d, m):
    """Exponent vectors of the polynomials of total degree < m in d variables (the null space)."""
    out = []

    def rec(prefix, left, dims):
        if dims == 0:
            out.append(tuple(prefix))
            return
        for e in range(left + 1):
            rec(prefix + [e], left - e, dims - 1)
    rec([], m - 1, d)
    return sorted(out, key=lambda e: (sum(e), [-v for v in e]))


def _tp_poly(Xd, exps):
    return torch.stack([torch.prod(torch.stack([Xd[:, i] ** e[i] for i in range(Xd.shape[1])], 1), 1) for e in exps], 1)


def tp_basis(Xd, st):
    """[radial part (reparameterised) | polynomial part] for rows Xd [n, d].

    ``standardize_tp_gam_cols`` (``st["inv_std"]``): distances between data and knots are measured on coordinates
    scaled by 1/sd of each column, and the polynomial part is taken of x - mean/sd, as the reference's
    GamUtilsThinPlateRegression.calculateDistance / calculatePolynomialBasis do with standardizeGAM."""
    K = torch.as_tensor(st["knots"], dtype=torch.float64, device=Xd.device)
    inv = st.get("inv_std")
    if inv is not None:
        iv = torch.as_tensor(inv, dtype=torch.float64, device=Xd.device)
        mu = torch.as_tensor(st["means"], dtype=torch.float64, device=Xd.device)
        r = torch.cdist(Xd * iv, K * iv)
        Xp = Xd - mu * iv
    else:
        r = torch.cdist(Xd, K)
        Xp = Xd
    E = _tp_eta(r, st["m"], Xd.shape[1])
    Zr = torch.as_tensor(st["Zr"], dtype=torch.float64, device=Xd.device)
    P = _tp_poly(Xp, st["exps"])
    return torch.cat([E @ Zr, P], 1)


# ------------------------------------------------------------------------------------------------ model
class GAMModel(Model):
    algo = "gam"

    def _smoother(self, X, g):
        dev = X.device
        cols = [torch.nan_to_num(X[self.col_index[c]].double(), nan=g["means"][i]) for i, c in enumerate(g["cols"])]
        bs = g["bs"]
        if bs == 0:
            B = cr_basis(cols[0], torch.as_tensor(g["knots"], dtype=torch.float64), torch.as_tensor(g["F"], dtype=torch.float64))
        elif bs == 1:
            B = tp_basis(torch.stack(cols, 1), g)
        elif bs == 2:
            B = ispline_basis(cols[0], torch.as_tensor(g["knots"], dtype=torch.float64, device=dev), g["order"])
        else:
            B = mspline_basis(cols[0], torch.as_tensor(g["knots"], dtype=torch.float64, device=dev), g["order"])
        if g.get("Z") is not None:
            B = B @ torch.as_tensor(g["Z"], dtype=torch.float64, device=dev)
        return B

    def _expand(self, X):
        X = X.to(self.device)
        out = [X[self.col_index[n]].double() for n in self.lin_x]
        for g in self.gams:
            B = self._smoother(X, g)
            out += [B[:, i] for i in range(B.shape[1])]
        return torch.stack(out, 0).float()

    def _predict_tensor(self, X, offset=None):
        return self.glm._predict_tensor(self._expand(X.to(self.device)), offset)

    def coef(self):
        return self.glm.output["coefficients"]


def _as_list(v, n, default):
    if v is None:
        return [default] * n
    v = list(v) if isinstance(v, (list, tuple)) else [v]
    return v + [default] * (n - len(v)) if len(v) < n else v[:n]


def _quantile_knots(x, k):
    """Knots at the k evenly spaced quantiles of the column (exact over every row, row-sharded too)."""
    from .quantile import weighted_quantiles
    qs = weighted_quantiles(x, torch.linspace(0, 1, int(k), dtype=torch.float64).tolist())
    return torch.unique(qs.to(x.device))


def _sum_rows(t: torch.Tensor) -> torch.Tensor:
    """Column sums over every rank's rows."""
    s = t.sum(0)
    if coll.is_dist():
        s = coll.all_reduce_(s.contiguous().to(coll.comm_device())).to(t.device)
    return s


def _global_rows(Xd: torch.Tensor, ids, row0: int) -> torch.Tensor:
    """Rows at GLOBAL row indices ``ids`` of a row-sharded matrix [N, d] (the owner contributes its row;
    one all-reduce of k x d values)."""
    ids = torch.as_tensor(list(ids), dtype=torch.long)
    out = torch.zeros(len(ids), Xd.shape[1], dtype=Xd.dtype, device=Xd.device)
    mine = (ids >= row0) & (ids < row0 + Xd.shape[0])
    if bool(mine.any()):
        out[mine.to(Xd.device)] = Xd[(ids[mine] - row0).to(Xd.device)]
    if coll.is_dist():
        out = coll.all_reduce_(out.to(coll.comm_device())).to(Xd.device)
    return out


def _rows_at_sorted_ranks(Xd: torch.Tensor, ranks, row0: int) -> torch.Tensor:
    """Rows whose stable sort position by column 0 (ties in global row order) is ``ranks`` — the rows
    ``Xd[argsort(Xd[:, 0], stable=True)[ranks]]`` of the single-process code, found over row shards with
    exact order statistics and a tie count instead of a global sort."""
    from ..parallel.order_stats import order_statistics
    x = Xd[:, 0].double()
    out = []
    for r in ranks:
        a = order_statistics(x, [int(r) + 1])[0]
        less = float((x < a).sum())
        tie = torch.nonzero(x == a).squeeze(1)
        if coll.is_dist():
            less = coll.all_reduce_scalar(less)
            off, _ = coll.exclusive_offset(int(tie.numel()))
        else:
            off = 0
        t = int(r) - int(less)
        row = torch.zeros(Xd.shape[1], dtype=Xd.dtype, device=Xd.device)
        if off <= t < off + tie.numel():
            row = Xd[tie[t - off]].clone()
        if coll.is_dist():
            row = coll.all_reduce_(row.to(coll.comm_device())).to(Xd.device)
        out.append(row)
    return torch.stack(out, 0)


class GAMTrainer:
    def __init__(self, params):
        p = dict(GAM_DEFAULTS)
        if "lambda" in params:
            params = dict(params)
            params["lambda_"] = params.pop("lambda")
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self._explicit = {k for k, v in params.items() if v is not None}
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from .glm import GLMTrainer
        t0 = time.time()
        p = self.p
        gcols = p["gam_columns"]
        if not gcols:
            raise ValueError("GAM needs gam_columns")
        groups = [[g] if isinstance(g, str) else list(g) for g in gcols]
        n = len(groups)
        bs = [int(b) for b in _as_list(p["bs"], n, 0)]
        for gi, g in enumerate(groups):
            if len(g) > 1 and bs[gi] != 1:
                raise ValueError(f"gam column group {g}: several columns need the thin-plate smoother (bs=1)")
        nk = [int(k) for k in _as_list(p["num_knots"], n, 10)]
        sc = [float(s) for s in _as_list(p["scale"], n, 0.001)]
        orders = [int(o) for o in _as_list(p["spline_orders"], n, 3)]
        nonneg = [bool(v) for v in _as_list(p["splines_non_negative"], n, True)]
        col_index = {nm: j for j, nm in enumerate(info.x)}
        gam_names = {c for g in groups for c in g}
        lin = [nm for nm in info.x if nm not in gam_names]
        dev = X.device
        row0 = coll.row_offset(X.shape[1]) if coll.is_dist() else 0
        n_glob = int(coll.all_reduce_scalar(X.shape[1])) if coll.is_dist() else X.shape[1]
        gams, names, pens, bounds = [], [], [], []
        for gi, (g, k, s, b) in enumerate(zip(groups, nk, sc, bs)):
            cols = [X[col_index[c]].double() for c in g]
            means = []
            for c in cols:
                okc = ~torch.isnan(c)
                sm = torch.stack([torch.where(okc, c, torch.zeros_like(c)).sum(), okc.double().sum()])
                if coll.is_dist():
                    sm = coll.all_reduce_(sm.to(coll.comm_device())).cpu()
                means.append(float(sm[0] / sm[1]))
            filled = [torch.nan_to_num(c, nan=mu) for c, mu in zip(cols, means)]
            st = dict(cols=g, bs=b, means=means, scale=s)
            if b == 0:
                knots = _quantile_knots(filled[0][~torch.isnan(cols[0])], k)
                if knots.numel() < 3:
                    raise ValueError(f"gam column {g[0]} needs at least 3 distinct knots")
                F, S = _cr_mats(knots.cpu())
                st.update(knots=knots.cpu().tolist(), F=F.tolist())
                B = cr_basis(filled[0], knots.cpu(), F)
            elif b == 1:
                Xd = torch.stack(filled, 1)
                d = Xd.shape[1]
                m = _tp_m(d)
                exps = _tp_poly_exps(d, m)
                kn = min(k, n_glob)
                if p.get("knot_ids") and gi < len(p["knot_ids"]) and p["knot_ids"][gi] is not None:
                    kid = p["knot_ids"][gi]
                    kid = kid if isinstance(kid, (list, tuple)) else [kid]
                    K = _global_rows(Xd, [int(v) for v in kid], row0)
                else:
                    ranks = torch.unique(torch.round(torch.linspace(0, n_glob - 1, kn, dtype=torch.float64)).long())
                    if coll.is_dist():
                        K = _rows_at_sorted_ranks(Xd, ranks.tolist(), row0)
                    else:
                        K = Xd[torch.argsort(Xd[:, 0], stable=True)[ranks.to(dev)]]
                if K.shape[0] <= len(exps):
                    raise ValueError(f"thin-plate smoother {g} needs more than {len(exps)} knots")
                inv = None
                if p.get("standardize_tp_gam_cols"):
                    # 1 / sample sd of each column (GAM.java: _predictVec.vec(c).sigma(), NAs skipped)
                    inv = []
                    for c, mu in zip(cols, means):
                        okc = ~torch.isnan(c)
                        v = torch.stack([torch.where(okc, (c - mu) ** 2, torch.zeros_like(c)).sum(), okc.double().sum()])
                        if coll.is_dist():
                            v = coll.all_reduce_(v.to(coll.comm_device())).cpu()
                        sd = math.sqrt(float(v[0]) / max(float(v[1]) - 1.0, 1.0))
                        inv.append(1.0 / sd if sd > 0 else 1.0)
                    st["inv_std"] = inv
                ivk = torch.as_tensor(inv, dtype=torch.float64, device=K.device) if inv is not None else None
                Kd = K * ivk if ivk is not None else K                    # the distance coordinates of the knots
                T = _tp_poly(K, exps)                                      # [k, M]
                Q, _ = torch.linalg.qr(T, mode="complete")
                Zr = Q[:, len(exps):]                                      # radial coefs orthogonal to T at the knots
                Ek = _tp_eta(torch.cdist(Kd, Kd), m, d)
                S_r = Zr.T @ Ek @ Zr
                st.update(knots=K.cpu().tolist(), m=m, exps=exps, Zr=Zr.cpu().tolist())
                B = tp_basis(Xd, st)
                S = torch.zeros(B.shape[1], B.shape[1], dtype=torch.float64)
                S[:S_r.shape[0], :S_r.shape[0]] = S_r.cpu()
                if p.get("scale_tp_penalty_mat"):
                    S = S / S.abs().max().clamp(min=1e-300)
            else:
                order = orders[gi]
                knots = _quantile_knots(filled[0][~torch.isnan(cols[0])], k)
                st.update(knots=knots.cpu().tolist(), order=order)
                B = (ispline_basis if b == 2 else mspline_basis)(filled[0], knots, order)
                S = _diff_penalty(B.shape[1])
            if b != 2:                         # sum-to-zero identifiability constraint (QR reparameterisation)
                c = _sum_rows(B) / n_glob
                Q, _ = torch.linalg.qr(c[:, None].cpu(), mode="complete")
                Z = Q[:, 1:]
                st["Z"] = Z.tolist()
                B = B @ Z.to(B.device)
                S = Z.T @ S.cpu() @ Z
            st["nb"] = B.shape[1]
            tag = "_".join(g)
            names += [f"{tag}_{suffix}_{i}" for i in range(B.shape[1])
                      for suffix in [{0: "cr", 1: "tp", 2: "is", 3: "ms"}[b]]]
            pens.append(s * S)
            bounds.append((b == 2 and nonneg[gi], B.shape[1]))
            gams.append(st)
        model = GAMModel(model_key or make_key("gam"), p, info)
        model.device = dev
        model.base_x = list(info.x)
        model.col_index = col_index
        model.lin_x = lin
        model.gams = gams
        Xg = model._expand(X)
        lin_cat = np.array([int(info.iscat[col_index[nm]]) for nm in lin], dtype=np.int32)
        ginfo = DataInfo(lin + names, np.concatenate([lin_cat, np.zeros(len(names), np.int32)]),
                         [info.domains[col_index[nm]] for nm in lin] + [None] * len(names),
                         info.response, info.response_domain)
        gp = {k: v for k, v in p.items() if k not in ("gam_columns", "num_knots", "scale", "bs", "knot_ids", "keep_gam_cols",
                                                      "spline_orders", "splines_non_negative", "scale_tp_penalty_mat")}
        if gp.get("lambda_search") and "lambda_" not in self._explicit:
            gp.pop("lambda_", None)           # the lambda path replaces the default fixed lambda
        tr = GLMTrainer(gp)
        # the GLM expands categoricals first, then numerics (linear numerics, then every smoother column):
        # the smoothers' penalty block is the tail of the coefficient vector (before the intercept)
        n_cat_exp = sum(len(info.domains[col_index[nm]]) - (0 if gp.get("use_all_factor_levels") else 1)
                        for nm in lin if info.iscat[col_index[nm]])
        n_lin_num = sum(1 for nm in lin if not info.iscat[col_index[nm]])
        tot_sm = sum(pp.shape[0] for pp in pens)
        P1 = n_cat_exp + n_lin_num + tot_sm + 1
        pen = torch.zeros(P1, P1, dtype=torch.float64)
        off = n_cat_exp + n_lin_num
        lb = None
        for pp, (nn, nb) in zip(pens, bounds):
            pen[off:off + nb, off:off + nb] = pp
            if nn:
                lb = torch.full((P1,), -float("inf"), dtype=torch.float64) if lb is None else lb
                lb[off:off + nb] = 0.0
            off += nb
        tr.penalty = pen
        if lb is not None:
            tr.lower_bounds = lb
        glm = tr.fit(Xg, y, w, offset, ginfo, None)
        model.glm = glm
        model.output["coefficients"] = glm.output["coefficients"]
        model.output["knots"] = {"_".join(g["cols"]): g["knots"] for g in gams}
        model.output["training_metrics"] = model.metrics_for(X, y, w, offset)
        if valid is not None:
            Xv, yv, wv, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv, ov)
        if p["keep_gam_cols"]:
            from ..frame import H2OFrame
            import contextlib
            from ..parallel import dframe
            ctx = dframe.shard_ctx(dframe.make_shard(Xg.shape[1])) if coll.is_dist() else contextlib.nullcontext()
            with ctx:
                model.output["gam_transformed_center_key"] = H2OFrame.from_tensor(Xg.T, lin + names).frame_id
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
