"""PSVM — kernel SVM (reference: ``hex/psvm/PSVM.java``, ``psvm/PrimalDualIPM.java``,
``IncompleteCholeskyFactorization``).

As the reference: the label-scaled Gaussian kernel Q = diag(y) K diag(y) is approximated by a pivoted
incomplete Cholesky factorization (rank ``rank_ratio·N``, default √N), computed on device column by column,
and the SVM dual is solved by ``primal_dual_ipm`` — PrimalDualIPM.java: barrier parameter t = mu_factor·2N/η
from the surrogate gap η, Newton directions through the Sherman-Morrison-Woodbury identity on the rank-r
factor (one r×r Cholesky per iteration), fraction-to-boundary line search, stop when the primal / dual
residuals are <= ``feasible_threshold`` and η <= ``surrogate_gap_threshold``. The model is
f(x) = Σ αᵢ yᵢ K(xᵢ, x) + ρ with the kernel through the factor (h(x) = L⁻¹·k(pivots, x), w = Hᵀ(α∘y));
ρ is the mean of yₛ - f₀(xₛ) over up to 1000 support vectors (CalculateRhoTask).
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from .base import DataInfo, Model, make_key
from .datainfo import Expander

PSVM_DEFAULTS = dict(hyper_param=1.0, kernel_type="gaussian", gamma=-1.0, rank_ratio=-1.0, positive_weight=1.0,
                     negative_weight=1.0, disable_training_metrics=False, sv_threshold=1e-4, fact_threshold=1e-5,
                     feasible_threshold=1e-3, surrogate_gap_threshold=1e-3, mu_factor=10.0, max_iterations=200, seed=-1,
                     zero_threshold=1e-9)


def primal_dual_ipm(Hl, y, c, max_iter=200, mu_factor=10.0, feasible_threshold=1e-3, sgap_threshold=1e-3,
                    x_epsilon=1e-9, tradeoff=0.0):
    """SVM dual  min ½ αᵀQα - 1ᵀα,  0 <= α <= c,  yᵀα = 0  with Q ≈ Hl Hlᵀ (Hl = label-scaled ICF factor),
    by the primal-dual interior point method of PrimalDualIPM.java. Returns (α, iterations, converged)."""
    N, r = Hl.shape
    x = torch.zeros(N, dtype=torch.float64, device=Hl.device)
    la = c / 10
    xi = c / 10
    nu = 0.0
    eye = torch.eye(r, dtype=torch.float64, device=Hl.device)
    converged, it = False, 0
    for it in range(int(max_iter)):
        eta = float((la * c).sum() + (x * (xi - la)).sum())             # SurrogateGapTask
        t = mu_factor * 2 * N / eta
        z = Hl @ (Hl.T @ x) - tradeoff * x + nu * y - 1.0                # computePartialZ + CheckConvergence
        resd = float(torch.linalg.vector_norm(la - xi + z))
        resp = abs(float((y * x).sum()))
        if resp <= feasible_threshold and resd <= feasible_threshold and eta <= sgap_threshold:
            converged = True
            break
        m_lx = x.clamp(min=x_epsilon)                                    # UpdateVarsTask
        m_ux = (c - x).clamp(min=x_epsilon)
        tlx, tux = 1.0 / (t * m_lx), 1.0 / (t * m_ux)
        xilx = (xi / m_lx).clamp(min=x_epsilon)
        laux = (la / m_ux).clamp(min=x_epsilon)
        d = 1.0 / (xilx + laux)
        z = tlx - tux - z
        Lc = torch.linalg.cholesky(eye + Hl.T @ (d[:, None] * Hl))      # I + Hlᵀ D Hl

        def solve_col(b):                                                 # (D⁻¹ + Hl Hlᵀ)⁻¹ b (Woodbury)
            v = torch.cholesky_solve((Hl.T @ (d * b))[:, None], Lc)[:, 0]
            return d * b - d * (Hl @ v)
        vz = torch.cholesky_solve((Hl.T @ (d * z))[:, None], Lc)[:, 0]  # computeDeltaNu
        vl = torch.cholesky_solve((Hl.T @ (d * y))[:, None], Lc)[:, 0]
        tw, tl = z - Hl @ vz, y - Hl @ vl
        dnu = float((y * (tw * d + x)).sum() / (y * tl * d).sum())
        dx = solve_col(z - dnu * y)                                       # computeDeltaX
        dxi = tlx - xilx * dx - xi                                        # LineSearchTask
        dla = tux + laux * dx - la
        inf = torch.full_like(x, float("inf"))
        ap = torch.minimum(torch.where(dx > 0, (c - x) / dx, inf), torch.where(dx < 0, -x / dx, inf)).min()
        ad = torch.minimum(torch.where(dxi < 0, -xi / dxi, inf), torch.where(dla < 0, -la / dla, inf)).min()
        ap = min(float(ap), 1.0) * 0.99
        ad = min(float(ad), 1.0) * 0.99
        x = x + ap * dx                                                   # MakeStepTask
        xi = xi + ad * dxi
        la = la + ad * dla
        nu += ad * dnu
    return x, it + 1, converged


def _rbf(A, B, gamma):
    d = (A * A).sum(1)[:, None] - 2 * A @ B.T + (B * B).sum(1)[None, :]
    return torch.exp(-gamma * d.clamp(min=0))


def icf(Z, rank, gamma, tol):
    """Pivoted incomplete Cholesky of the RBF kernel: returns H [N, r] and pivot row ids."""
    N = Z.shape[0]
    diag = torch.ones(N, dtype=torch.float64, device=Z.device)
    H = torch.zeros(N, rank, dtype=torch.float64, device=Z.device)
    piv = []
    for j in range(rank):
        i = int(torch.argmax(diag))
        if float(diag[i]) <= tol:
            H = H[:, :j]
            break
        piv.append(i)
        kcol = _rbf(Z, Z[i:i + 1], gamma)[:, 0]
        h = (kcol - H[:, :j] @ H[i, :j]) / math.sqrt(float(diag[i]))
        H[:, j] = h
        diag = (diag - h * h).clamp(min=0)
    return H, torch.as_tensor(piv, device=Z.device)


class PSVMModel(Model):
    algo = "psvm"

    def _features(self, X):
        Z = self.expander.transform(X.to(self.device)).double()
        Kp = _rbf(Z, self.pivots_z.to(Z.device), self.gamma_)
        return torch.linalg.solve_triangular(self.L.to(Z.device), Kp.T, upper=False).T

    def _decision(self, X):
        Hn = self._features(X)
        return Hn @ self.wvec.to(Hn.device) + self.b

    def _predict_tensor(self, X, offset=None):
        f = self._decision(X)
        p1 = (f > 0).double()
        return torch.stack([1 - p1, p1], 1).float()

    def to_state(self):
        s = super().to_state()
        s.update(pivots=self.pivots_z.cpu().tolist(), L=self.L.cpu().tolist(), w=self.wvec.cpu().tolist(), b=self.b,
                 gamma=self.gamma_, expander=self.expander.to_state())
        return s

    def _restore(self, s):
        super()._restore(s)
        self.pivots_z = torch.tensor(s["pivots"], dtype=torch.float64)
        self.L = torch.tensor(s["L"], dtype=torch.float64)
        self.wvec = torch.tensor(s["w"], dtype=torch.float64)
        self.b, self.gamma_ = s["b"], s["gamma"]
        self.expander = Expander.from_state(self.info, s["expander"])


class PSVMTrainer:
    def __init__(self, params):
        p = dict(PSVM_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        t0 = time.time()
        p = self.p
        if len(info.response_domain) != 2:
            raise ValueError("PSVM supports binary classification only")
        dev = X.device
        ex = Expander(info, standardize=True, use_all_factor_levels=True).fit(X)
        Z = ex.transform(X).double()
        N, P = Z.shape
        gamma = float(p["gamma"]) if float(p["gamma"]) > 0 else 1.0 / max(P, 1)
        rr = float(p["rank_ratio"])
        rank = int(math.ceil(math.sqrt(N))) if rr <= 0 else max(1, int(rr * N))
        rank = min(rank, N)
        H, piv = icf(Z, rank, gamma, float(p["fact_threshold"]))
        r = H.shape[1]
        Lm = H[piv]                                  # K(piv, piv) ≈ L Lᵀ, lower triangular in pivot order
        yy = torch.where(y > 0.5, 1.0, -1.0).double()
        C = float(p["hyper_param"])
        c = torch.where(yy > 0, C * float(p["positive_weight"]), C * float(p["negative_weight"])).double()
        if str(p.get("kernel_type", "gaussian")).lower() != "gaussian":
            raise ValueError("kernel_type: only 'gaussian' is available (as in the reference)")
        alpha, iters, conv = primal_dual_ipm(yy[:, None] * H, yy, c, int(p["max_iterations"]), float(p["mu_factor"]),
                                             float(p["feasible_threshold"]), float(p["surrogate_gap_threshold"]),
                                             float(p.get("zero_threshold") or 1e-9))
        thr = float(p["sv_threshold"])
        sv = alpha > thr                                                  # RegulateAlphaTask
        bsv = sv & (c - alpha <= thr)
        wvec = H.T @ (alpha * yy)
        f0 = H @ wvec
        idx = torch.nonzero(sv).flatten()
        if idx.numel() > 1000:
            idx = idx[torch.randperm(idx.numel(), generator=torch.Generator().manual_seed(0))[:1000].to(idx.device)]
        rho = float((yy[idx] - f0[idx]).mean()) if idx.numel() else 0.0    # CalculateRhoTask
        model = PSVMModel(model_key or make_key("psvm"), p, info)
        model.device = dev
        model.expander = ex
        model.pivots_z = Z[piv]
        model.L = Lm
        model.wvec = wvec
        model.b = rho
        model.gamma_ = gamma
        model.output.update(svs_count=int(sv.sum()), bsv_count=int(bsv.sum()), rho=rho, rank=r, gamma=gamma,
                            ipm_iterations=iters, ipm_converged=conv)
        if not p["disable_training_metrics"]:
            model.output["training_metrics"] = model.metrics_for(X, y, w)
        if valid is not None:
            Xv, yv, wv2, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv2, ov)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
