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
import torch.distributed as dist

from ..parallel import collectives as coll

from .base import DataInfo, Model, make_key
from .datainfo import Expander

PSVM_DEFAULTS = dict(hyper_param=1.0, kernel_type="gaussian", gamma=-1.0, rank_ratio=-1.0, positive_weight=1.0,
                     negative_weight=1.0, disable_training_metrics=False, sv_threshold=1e-4, fact_threshold=1e-5,
                     feasible_threshold=1e-3, surrogate_gap_threshold=1e-3, mu_factor=10.0, max_iterations=200, seed=-1,
                     zero_threshold=1e-9)


def _red(t: torch.Tensor, op=None) -> torch.Tensor:
    """All-reduce over the row shards (no-op in one process): the reductions of PSVM's MRTasks."""
    if not coll.is_dist():
        return t
    return coll.all_reduce_(t.contiguous().to(coll.comm_device()), op).to(t.device)


def primal_dual_ipm(Hl, y, c, max_iter=200, mu_factor=10.0, feasible_threshold=1e-3, sgap_threshold=1e-3,
                    x_epsilon=1e-9, tradeoff=0.0):
    """SVM dual  min ½ αᵀQα - 1ᵀα,  0 <= α <= c,  yᵀα = 0  with Q ≈ Hl Hlᵀ (Hl = label-scaled ICF factor),
    by the primal-dual interior point method of PrimalDualIPM.java. Returns (α, iterations, converged).

    Rows (of Hl, y, c, α and the dual vectors) may be sharded over the ranks: everything row-wise stays
    local and an iteration needs four all-reduces — [Hlᵀα, surrogate gap, yᵀα], [‖residual‖², Hlᵀ D Hl,
    Hlᵀ D z, Hlᵀ D y] (the r x r Woodbury system is then solved identically on every rank), the two sums of
    Δν, and the two step-length minima."""
    N_loc, r = Hl.shape
    N = int(_red(torch.tensor([float(N_loc)], dtype=torch.float64)).item())
    dev = Hl.device
    x = torch.zeros(N_loc, dtype=torch.float64, device=dev)
    la = c / 10
    xi = c / 10
    nu = 0.0
    eye = torch.eye(r, dtype=torch.float64, device=dev)
    converged, it = False, 0
    for it in range(int(max_iter)):
        A = _red(torch.cat([Hl.T @ x, torch.stack([(la * c).sum() + (x * (xi - la)).sum(), (y * x).sum()])]))
        eta, resp = float(A[r]), abs(float(A[r + 1]))                    # SurrogateGapTask
        t = mu_factor * 2 * N / eta
        z = Hl @ A[:r] - tradeoff * x + nu * y - 1.0                     # computePartialZ + CheckConvergence
        m_lx = x.clamp(min=x_epsilon)                                    # UpdateVarsTask
        m_ux = (c - x).clamp(min=x_epsilon)
        tlx, tux = 1.0 / (t * m_lx), 1.0 / (t * m_ux)
        xilx = (xi / m_lx).clamp(min=x_epsilon)
        laux = (la / m_ux).clamp(min=x_epsilon)
        d = 1.0 / (xilx + laux)
        zz = tlx - tux - z
        B = _red(torch.cat([((la - xi + z) ** 2).sum().reshape(1), (Hl.T @ (d[:, None] * Hl)).reshape(-1),
                            Hl.T @ (d * zz), Hl.T @ (d * y)]))
        resd = math.sqrt(max(float(B[0]), 0.0))
        if resp <= feasible_threshold and resd <= feasible_threshold and eta <= sgap_threshold:
            converged = True
            break
        G = B[1:1 + r * r].reshape(r, r)
        Lc = torch.linalg.cholesky(eye + G)                              # I + Hlᵀ D Hl
        vz = torch.cholesky_solve(B[1 + r * r:1 + r * r + r, None], Lc)[:, 0]   # computeDeltaNu
        vl = torch.cholesky_solve(B[1 + r * r + r:, None], Lc)[:, 0]
        tw, tl = zz - Hl @ vz, y - Hl @ vl
        S = _red(torch.stack([(y * (tw * d + x)).sum(), (y * tl * d).sum()]))
        dnu = float(S[0] / S[1])
        bb = zz - dnu * y                                                 # computeDeltaX (Woodbury, linear in b)
        dx = d * bb - d * (Hl @ (vz - dnu * vl))
        dxi = tlx - xilx * dx - xi                                        # LineSearchTask
        dla = tux + laux * dx - la
        inf = torch.full_like(x, float("inf"))
        ap = torch.minimum(torch.where(dx > 0, (c - x) / dx, inf), torch.where(dx < 0, -x / dx, inf))
        ad = torch.minimum(torch.where(dxi < 0, -xi / dxi, inf), torch.where(dla < 0, -la / dla, inf))
        M = torch.stack([ap.min() if ap.numel() else inf.new_tensor(float("inf")),
                         ad.min() if ad.numel() else inf.new_tensor(float("inf"))])
        M = _red(M, dist.ReduceOp.MIN)
        ap = min(float(M[0]), 1.0) * 0.99
        ad = min(float(M[1]), 1.0) * 0.99
        x = x + ap * dx                                                   # MakeStepTask
        xi = xi + ad * dxi
        la = la + ad * dla
        nu += ad * dnu
    return x, it + 1, converged


def _rbf(A, B, gamma):
    d = (A * A).sum(1)[:, None] - 2 * A @ B.T + (B * B).sum(1)[None, :]
    return torch.exp(-gamma * d.clamp(min=0))


def icf(Z, rank, gamma, tol, gid=None):
    """Pivoted incomplete Cholesky of the RBF kernel over (possibly row-sharded) rows: returns the local
    rows of H [n, r], the pivots' feature rows [r, P] and their global row ids. Each column: the global
    argmax of the residual diagonal (lowest global row id on ties), the owner's pivot row (z_i, H[i, :j])
    all-reduced to every rank, then the local kernel column (IncompleteCholeskyFactorization.java)."""
    n, P = Z.shape
    dev = Z.device
    gid = torch.arange(n, dtype=torch.float64, device=dev) if gid is None else gid
    diag = torch.ones(n, dtype=torch.float64, device=dev)
    H = torch.zeros(n, rank, dtype=torch.float64, device=dev)
    pz, pid = [], []
    sharded = coll.is_dist()
    for j in range(rank):
        if n:
            mx = diag.max()
            cand = gid[diag == mx].min()
        else:
            mx, cand = torch.tensor(-1.0, dtype=torch.float64, device=dev), torch.tensor(0.0, device=dev)
        if sharded:
            mine = torch.stack([mx.double(), -cand.double()]).to(coll.comm_device())
            allc = coll.all_gather_into_(torch.empty(coll.world() * 2, dtype=torch.float64, device=mine.device),
                                         mine).cpu().reshape(-1, 2)
            top = allc[:, 0].max()
            tie = allc[:, 0] == top
            g_best = float(-allc[tie, 1].max())
            dval = float(top)
        else:
            g_best, dval = float(cand), float(mx)
        if dval <= tol:
            H = H[:, :j]
            break
        own = gid == g_best
        row = torch.zeros(P + j, dtype=torch.float64, device=dev)
        if bool(own.any()):
            i = int(torch.nonzero(own)[0])
            row = torch.cat([Z[i].double(), H[i, :j]])
        row = _red(row)
        zi, hi_ = row[:P], row[P:]
        pz.append(zi); pid.append(g_best)
        kcol = _rbf(Z, zi[None, :].to(Z.dtype), gamma)[:, 0].double()
        h = (kcol - H[:, :j] @ hi_) / math.sqrt(dval)
        H[:, j] = h
        diag = (diag - h * h).clamp(min=0)
    r = H.shape[1]
    PZ = torch.stack(pz) if pz else torch.zeros(0, P, dtype=torch.float64, device=dev)
    return H, PZ, pid[:r]


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
        sharded = coll.is_dist()
        ex = Expander(info, standardize=True, use_all_factor_levels=True).fit(
            X, reduce=coll.all_reduce_ if sharded else None)
        Z = ex.transform(X).double()
        n, P = Z.shape
        start, N = coll.exclusive_offset(n)
        gid = torch.arange(start, start + n, dtype=torch.float64, device=dev)
        gamma = float(p["gamma"]) if float(p["gamma"]) > 0 else 1.0 / max(P, 1)
        rr = float(p["rank_ratio"])
        rank = int(math.ceil(math.sqrt(N))) if rr <= 0 else max(1, int(rr * N))
        rank = min(rank, N)
        H, PZ, piv = icf(Z, rank, gamma, float(p["fact_threshold"]), gid)
        r = H.shape[1]
        # K(piv, piv) ≈ L Lᵀ, lower triangular in pivot order: the pivots' rows of H, from their owners
        own = torch.isin(gid, torch.tensor(piv, dtype=torch.float64, device=dev))
        Lm = torch.zeros(r, r, dtype=torch.float64, device=dev)
        if bool(own.any()):
            pos = {g: k for k, g in enumerate(piv)}
            for i in torch.nonzero(own).flatten().tolist():
                Lm[pos[float(gid[i])]] = H[i]
        Lm = _red(Lm)
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
        wvec = _red(H.T @ (alpha * yy))
        f0 = H @ wvec
        cnt = _red(torch.stack([sv.double().sum(), bsv.double().sum()]))
        nsv = int(cnt[0])
        # CalculateRhoTask: mean of y - f0 over up to 1000 support vectors (a per-global-row draw)
        pick = sv if nsv <= 1000 else sv & (coll.row_uniform(0, 11, start, n, dev) < 1000.0 / nsv)
        rs = _red(torch.stack([(yy - f0)[pick].sum(), pick.double().sum()]))
        rho = float(rs[0] / rs[1]) if float(rs[1]) > 0 else 0.0
        model = PSVMModel(model_key or make_key("psvm"), p, info)
        model.device = dev
        model.expander = ex
        model.pivots_z = PZ
        model.L = Lm
        model.wvec = wvec
        model.b = rho
        model.gamma_ = gamma
        model.output.update(svs_count=nsv, bsv_count=int(cnt[1]), rho=rho, rank=r, gamma=gamma,
                            ipm_iterations=iters, ipm_converged=conv)
        if not p["disable_training_metrics"]:
            model.output["training_metrics"] = model.metrics_for(X, y, w)
        if valid is not None:
            Xv, yv, wv2, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv2, ov)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
