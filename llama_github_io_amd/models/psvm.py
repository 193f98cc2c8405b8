"""PSVM — kernel SVM (reference: ``hex/psvm/PSVM.java``, ``psvm/kernel``, ``IncompleteCholeskyFactorization``).

Same structure as the reference: the Gaussian kernel matrix is approximated by a pivoted
incomplete Cholesky factorization K ≈ H Hᵀ of rank ``rank_ratio·N`` (default √N), computed on
device column by column; the SVM is then solved in the factor space. Where PSVM runs a parallel
interior-point method on the dual, here the equivalent primal (squared-hinge, L2) problem in the
H features is solved with L-BFGS on device. Scoring maps new rows through the pivots:
h(x) = L⁻¹·k(pivots, x). Outputs: number of support vectors (margin violators), rho (bias).
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
                     feasible_threshold=1e-3, surrogate_gap_threshold=1e-3, mu_factor=10.0, max_iterations=200, seed=-1)


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
        cw = torch.where(yy > 0, float(p["positive_weight"]), float(p["negative_weight"])).double()
        C = float(p["hyper_param"])
        wv = torch.zeros(r, dtype=torch.float64, device=dev, requires_grad=True)
        bb = torch.zeros(1, dtype=torch.float64, device=dev, requires_grad=True)
        opt = torch.optim.LBFGS([wv, bb], lr=1, max_iter=int(p["max_iterations"]), line_search_fn="strong_wolfe",
                                tolerance_grad=1e-10, tolerance_change=1e-14)

        def closure():
            opt.zero_grad()
            m = (1 - yy * (H @ wv + bb)).clamp(min=0)
            loss = 0.5 * (wv * wv).sum() + C * (cw * m * m).sum()
            loss.backward()
            return loss
        opt.step(closure)
        model = PSVMModel(model_key or make_key("psvm"), p, info)
        model.device = dev
        model.expander = ex
        model.pivots_z = Z[piv]
        model.L = Lm
        model.wvec = wv.detach()
        model.b = float(bb.detach())
        model.gamma_ = gamma
        with torch.no_grad():
            marg = yy * (H @ model.wvec + model.b)
        model.output.update(svs_count=int((marg < 1 + float(p["sv_threshold"])).sum()),
                            bsv_count=int((marg < 0).sum()), rho=-model.b, rank=r, gamma=gamma)
        if not p["disable_training_metrics"]:
            model.output["training_metrics"] = model.metrics_for(X, y, w)
        if valid is not None:
            Xv, yv, wv2, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv2, ov)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
