"""Hierarchical GLM — Gaussian response with Gaussian random intercepts (reference:
``hex/glm/GLM.java:fitHGLM`` (Lee & Nelder h-likelihood fitting: augmented weighted least squares for
[beta | u], leverages of the augmented system, gamma-GLM dispersion updates for sigma_e^2 and every
random column's sigma_u^2), ``hex/ModelMetricsHGLM*.java``).

Each iteration solves the mixed-model equations on device in fp64:

    [X'WX      X'WZ          ] [beta]   [X'Wy]
    [Z'WX   Z'WZ + diag(lam) ] [ u  ] = [Z'Wy],   lam_c = sigma_e^2 / sigma_u,c^2

then takes leverages h of the augmented rows and updates the dispersions with the intercept-only gamma
GLMs of the reference in closed form (an intercept-only log-link gamma GLM with response d/(1-h) and
weights (1-h)/2 has MLE exp(b0) = sum(d) / sum(1-h)):

    sigma_e^2 = sum_i w_i (y_i - eta_i)^2 / sum_i (1 - h_i),   sigma_u,c^2 = sum_{j in c} u_j^2 / sum_{j in c} (1 - h_j)

until sum((eta - eta_old)^2) / sum(eta^2) < objective_epsilon.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..parallel import collectives as coll
from .base import DataInfo
from .datainfo import Expander


def _red(t: torch.Tensor) -> torch.Tensor:
    """Sum over every rank's rows (the reference's MRTask reductions); no-op in one process."""
    if not coll.is_dist():
        return t
    return coll.all_reduce_(t.contiguous().to(coll.comm_device())).to(t.device)


def _rsum(t: torch.Tensor) -> float:
    return float(_red(t.sum().reshape(1)))


def _random_indices(info: DataInfo, random_columns):
    out = []
    for c in (random_columns if isinstance(random_columns, (list, tuple)) else [random_columns]):
        j = info.x.index(c) if isinstance(c, str) else int(c)
        if not (0 <= j < info.F) or not info.iscat[j]:
            raise ValueError(f"random column {c!r} must be a categorical predictor")
        out.append(j)
    return out


def random_design(X, rand_idx, sizes, dev):
    """Dense one-hot [N, Q] of the random columns (NA / unseen levels: no random effect)."""
    N = X.shape[1]
    Z = torch.zeros(N, int(sum(sizes)), dtype=torch.float64, device=dev)
    off = 0
    for j, L in zip(rand_idx, sizes):
        c = X[j]
        ok = ~torch.isnan(c) & (c >= 0) & (c < L)
        rows = torch.nonzero(ok, as_tuple=True)[0]
        Z[rows, off + c[rows].long()] = 1.0
        off += L
    return Z


def fit_hglm(trainer, X, y, w, off, info: DataInfo, model, p):
    dev = X.device
    fam = str(p.get("family", "gaussian")).lower()
    rfam = p.get("rand_family") or ["gaussian"]
    if fam != "gaussian" or any(str(r).lower() != "gaussian" for r in rfam):
        raise ValueError("HGLM supports family='gaussian' with rand_family='gaussian' (as the reference)")
    rand_idx = _random_indices(info, p.get("random_columns") or [])
    if not rand_idx:
        raise ValueError("HGLM needs random_columns")
    # GLMModel.GLMParameters.validate (hex/glm/GLMModel.java:534-548): one link per random column, identity only
    rlink = p.get("rand_link")
    if rlink not in (None, [], ()):
        rlink = [rlink] if isinstance(rlink, str) else list(rlink)
        if len(rlink) != len(rand_idx):
            raise ValueError("HGLM _rand_link: must have the same length as random_columns.")
        for lk in rlink:
            if str(lk).lower().replace("_", "") not in ("identity", "familydefault"):
                raise ValueError("HGLM only supports identity link functions for now.")
    link = str(p.get("link") or "family_default").lower().replace("_", "")
    if link not in ("identity", "familydefault"):
        raise ValueError("HGLM only supports identity link functions for now.")
    fixed_idx = [j for j in range(info.F) if j not in rand_idx]
    finfo = DataInfo([info.x[j] for j in fixed_idx], np.asarray(info.iscat)[fixed_idx],
                     [info.domains[j] for j in fixed_idx], info.response, info.response_domain)
    N = X.shape[1]
    w = torch.ones(N, dtype=torch.float64, device=dev) if w is None else w.double()
    yv = y.double()
    ok = ~torch.isnan(yv)
    w = torch.where(ok, w, torch.zeros_like(w))
    yv = torch.where(ok, yv, torch.zeros_like(yv))
    offv = torch.zeros(N, dtype=torch.float64, device=dev) if off is None else off.double()
    Xf = X[fixed_idx] if fixed_idx else X[:0]
    ex = Expander(finfo, standardize=p.get("standardize", True),
                  use_all_factor_levels=p.get("use_all_factor_levels", False)).fit(
                      Xf, w, reduce=coll.all_reduce_ if coll.is_dist() else None)
    M1 = torch.cat([ex.transform(Xf, dtype=torch.float64), torch.ones(N, 1, dtype=torch.float64, device=dev)], 1)
    sizes = [len(info.domains[j]) for j in rand_idx]
    Z = random_design(X, rand_idx, sizes, dev)
    M = torch.cat([M1, Z], 1)
    P1, Q = M1.shape[1], Z.shape[1]
    col_of = torch.cat([torch.full((L,), k, dtype=torch.long) for k, L in enumerate(sizes)]).to(dev)
    r = yv - offv
    W = _rsum(w)
    rbar = _rsum(w * r) / W
    var_y = _rsum(w * (r - rbar) ** 2) / max(W - 1, 1.0)
    sig_e = float(p.get("init_sig_e") or 0.0) or 0.6 * max(var_y, 1e-12)
    su = p.get("init_sig_u")
    sig_u = torch.full((len(sizes),), float(su) if su else 0.4 * max(var_y, 1e-12), dtype=torch.float64, device=dev)
    Gm = _red(M.T @ (w[:, None] * M))
    rhs = _red(M.T @ (w * r))
    eps = float(p.get("objective_epsilon") or 0)
    eps = eps if eps > 0 else 1e-6
    max_it = int(p.get("max_iterations") or 0)
    max_it = max_it if max_it > 0 else 50
    eta_old = torch.zeros(N, dtype=torch.float64, device=dev)
    converged = False
    it = 0
    for it in range(1, max_it + 1):
        lam = sig_e / sig_u[col_of]
        A = Gm.clone()
        A[P1:, P1:] += torch.diag(lam)
        L = torch.linalg.cholesky(A + 1e-12 * torch.eye(P1 + Q, dtype=A.dtype, device=dev))
        Ainv = torch.cholesky_inverse(L)
        coef = Ainv @ rhs
        eta = M @ coef
        h_data = w * ((M @ Ainv) * M).sum(1)
        h_rand = lam * torch.diagonal(Ainv)[P1:]
        u = coef[P1:]
        dres = w * (r - eta) ** 2
        sig_e = _rsum(dres) / max(_rsum((w > 0).double().mul(1 - h_data)), 1e-12)
        num = torch.zeros(len(sizes), dtype=torch.float64, device=dev).index_add_(0, col_of, u * u)
        den = torch.zeros(len(sizes), dtype=torch.float64, device=dev).index_add_(0, col_of, 1 - h_rand)
        sig_u = (num / den.clamp(min=1e-12)).clamp(min=1e-12)
        conv = _rsum((eta - eta_old) ** 2) / max(_rsum(eta ** 2), 1e-300)
        eta_old = eta
        if conv < eps:
            converged = True
            break
    beta_std = coef[:P1]
    braw, ic = ex.destandardize(beta_std[:-1], float(beta_std[-1]))
    model.expander = ex
    model.beta = beta_std[None, :].clone()
    model.hglm = dict(fixed_idx=fixed_idx, rand_idx=rand_idx, sizes=sizes, u=u.clone())
    # h-likelihood: log f(y | u) + log f(u)
    nobs = _rsum((w > 0).double())
    hlik = -0.5 * (nobs * math.log(2 * math.pi * sig_e) + _rsum(dres) / sig_e)
    for k, Lk in enumerate(sizes):
        uk = u[col_of == k]
        hlik += -0.5 * (Lk * math.log(2 * math.pi * float(sig_u[k])) + float((uk * uk).sum()) / float(sig_u[k]))
    names = ex.names + ["Intercept"]
    se_all = torch.sqrt(torch.diagonal(Ainv).clamp(min=0) * sig_e)
    rnames = []
    for j, Lk in zip(rand_idx, sizes):
        rnames += [f"{info.x[j]}.{lv}" for lv in info.domains[j]]
    model.output.update(
        family="gaussian", link="identity", HGLM=True, converge=converged, iterations=it,
        coefficients=dict(zip(names, braw.cpu().tolist() + [ic])),
        standardized_coefficients=dict(zip(names, beta_std.cpu().tolist())),
        ubeta=u.cpu().tolist(), random_coefficient_names=rnames,
        random_coefficients=dict(zip(rnames, u.cpu().tolist())),
        varfix=sig_e, varranef=sig_u.cpu().tolist(), tau=sig_e, phi=sig_u.cpu().tolist(),
        sefe=se_all[:P1].cpu().tolist(), sere=se_all[P1:].cpu().tolist(), hlik=hlik,
        random_columns=[info.x[j] for j in rand_idx])
    return model


def hglm_eta(model, X, offset=None):
    """Linear predictor with the fitted random intercepts (unseen / NA levels contribute 0)."""
    hg = model.hglm
    Xf = X[hg["fixed_idx"]] if hg["fixed_idx"] else X[:0]
    Zf = model.expander.transform(Xf.to(model.device), dtype=torch.float64)
    b = model.beta.to(Zf.device)
    eta = Zf @ b[0, :-1] + b[0, -1]
    Z = random_design(X.to(Zf.device), hg["rand_idx"], hg["sizes"], Zf.device)
    eta = eta + Z @ hg["u"].to(Zf.device)
    if offset is not None:
        eta = eta + offset.double().to(Zf.device)
    return eta[:, None]
