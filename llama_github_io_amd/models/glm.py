"""Generalized Linear Models (reference: ``hex/glm/GLM.java``, ``GLMModel.java`` (families, links,
defaults), ``GLMTask.java`` (GLMIterationTask / Gram), ``hex/gram/Gram.java`` (Cholesky),
``hex/optimization/L_BFGS.java``, ``ComputationState.java`` (objective, lambda path)).

Solver layout on MI355X:

* IRLSM: per iteration the working weights/response are elementwise device ops; the weighted Gram
  ``ZᵀWZ`` runs on the MFMA Gram kernel (``ops.gram``) and ``ZᵀWz`` on the cross-product kernel;
  the (P+1)² system is solved in fp64 on device — Cholesky for ridge, cyclic coordinate descent on
  the Gram for L1/elastic-net (H2O's COD over the Gram). Rank-1 statistics are all-reduced over
  RCCL when the frame is row-sharded (one process per GPU).
* L-BFGS: the full objective (``obj_reg``·negative log-likelihood + elastic-net) is evaluated on
  device with autograd (multinomial, ordinal, very wide problems).
* ``lambda_search``: H2O's path from ``λmax = max|∇|/max(α, 1e-2)`` down ``nlambdas`` steps to
  ``λmax·lambda_min_ratio`` with warm starts; the default single λ is ``10·lambda_min_ratio·λmax``.

Families: gaussian, binomial, quasibinomial, fractionalbinomial, multinomial, ordinal, poisson,
gamma, tweedie, negativebinomial; links: identity, logit, log, inverse, tweedie (power), ologit.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch
import torch.distributed

from .. import metrics as mm
from ..parallel import collectives as coll
from ..ops import gram as G
from .base import DataInfo, Model, make_key
from .datainfo import Expander
from .params import canon
from ..ops.segment import segment_sum

_MIN, _MAX = torch.distributed.ReduceOp.MIN, torch.distributed.ReduceOp.MAX

GLM_DEFAULTS = dict(family="AUTO", link="family_default", solver="AUTO", alpha=None, lambda_=None, lambda_search=False,
                    nlambdas=-1, lambda_min_ratio=-1.0, standardize=True, intercept=True, max_iterations=-1,
                    beta_epsilon=1e-4, objective_epsilon=-1.0, gradient_epsilon=-1.0, tweedie_variance_power=0.0,
                    tweedie_link_power=1.0, theta=1e-10, compute_p_values=False, remove_collinear_columns=False,
                    missing_values_handling="MeanImputation", non_negative=False, obj_reg=-1.0, prior=-1.0,
                    max_active_predictors=-1, use_all_factor_levels=False, beta_constraints=None,
                    interactions=None, interaction_pairs=None, early_stopping=True, cold_start=False,
                    calc_like=False, dispersion_parameter_method="pearson", lambda_min=None, seed=-1, startval=None,
                    plug_values=None, build_null_model=False)

DEFAULT_LINK = {"gaussian": "identity", "binomial": "logit", "quasibinomial": "logit", "fractionalbinomial": "logit",
                "poisson": "log", "gamma": "inverse", "tweedie": "tweedie", "negativebinomial": "log",
                "multinomial": "multinomial", "ordinal": "ologit"}


# ------------------------------------------------------------------------------------------------
class Family:
    def __init__(self, name, link, tvp=0.0, tlp=1.0, theta=1e-10):
        self.name, self.link, self.tvp, self.tlp, self.theta = name, link, tvp, tlp, theta

    def linkinv(self, eta):
        l = self.link
        if l == "identity":
            return eta
        if l == "logit":
            return torch.sigmoid(eta)
        if l == "log":
            return torch.exp(eta.clamp(max=700))
        if l == "inverse":
            e = torch.where(eta.abs() < 1e-10, torch.full_like(eta, 1e-10) * torch.sign(eta + 1e-300), eta)
            return 1.0 / e
        if l == "tweedie":
            return torch.exp(eta.clamp(max=700)) if self.tlp == 0 else eta.clamp(min=1e-10).pow(1.0 / self.tlp)
        raise ValueError(l)

    def linkfn(self, mu):
        l = self.link
        if l == "identity":
            return mu
        if l == "logit":
            m = mu.clamp(1e-10, 1 - 1e-10)
            return torch.log(m / (1 - m))
        if l == "log":
            return torch.log(mu.clamp(min=1e-10))
        if l == "inverse":
            return 1.0 / mu.clamp(min=1e-10)
        if l == "tweedie":
            return torch.log(mu.clamp(min=1e-10)) if self.tlp == 0 else mu.clamp(min=1e-10).pow(self.tlp)
        raise ValueError(l)

    def dlink(self, mu):
        """g'(mu)."""
        l = self.link
        if l == "identity":
            return torch.ones_like(mu)
        if l == "logit":
            m = mu.clamp(1e-10, 1 - 1e-10)
            return 1.0 / (m * (1 - m))
        if l == "log":
            return 1.0 / mu.clamp(min=1e-10)
        if l == "inverse":
            return -1.0 / (mu * mu).clamp(min=1e-20)
        if l == "tweedie":
            m = mu.clamp(min=1e-10)
            return 1.0 / m if self.tlp == 0 else self.tlp * m.pow(self.tlp - 1)
        raise ValueError(l)

    def variance(self, mu):
        n = self.name
        if n == "gaussian":
            return torch.ones_like(mu)
        if n in ("binomial", "quasibinomial", "fractionalbinomial"):
            m = mu.clamp(1e-10, 1 - 1e-10)
            return m * (1 - m)
        if n == "poisson":
            return mu.clamp(min=1e-10)
        if n == "gamma":
            return (mu * mu).clamp(min=1e-20)
        if n == "tweedie":
            return mu.clamp(min=1e-10).pow(self.tvp)
        if n == "negativebinomial":
            return mu + self.theta * mu * mu
        raise ValueError(n)

    def deviance(self, y, mu):
        n = self.name
        if n == "gaussian":
            return (y - mu) ** 2
        if n in ("binomial", "quasibinomial", "fractionalbinomial"):
            m = mu.clamp(1e-15, 1 - 1e-15)
            return -2 * (y * torch.log(m) + (1 - y) * torch.log(1 - m))
        if n == "poisson":
            m = mu.clamp(min=1e-15)
            return 2 * (torch.where(y > 0, y * torch.log(y.clamp(min=1e-300) / m), torch.zeros_like(y)) - (y - m))
        if n == "gamma":
            m = mu.clamp(min=1e-15)
            yy = y.clamp(min=1e-15)
            return 2 * (-torch.log(yy / m) + (y - m) / m)
        if n == "tweedie":
            p = self.tvp
            m = mu.clamp(min=1e-15)
            if p == 0:
                return (y - mu) ** 2
            if p == 1:
                return 2 * (torch.where(y > 0, y * torch.log(y.clamp(min=1e-300) / m), torch.zeros_like(y)) - (y - m))
            if p == 2:
                yy = y.clamp(min=1e-15)
                return 2 * (-torch.log(yy / m) + (y - m) / m)
            return 2 * (torch.where(y > 0, y.clamp(min=0).pow(2 - p) / ((1 - p) * (2 - p)), torch.zeros_like(y))
                        - y * m.pow(1 - p) / (1 - p) + m.pow(2 - p) / (2 - p))
        if n == "negativebinomial":
            th = self.theta
            m = mu.clamp(min=1e-15)
            t1 = torch.where(y > 0, y * torch.log(y.clamp(min=1e-300) / m), torch.zeros_like(y))
            return 2 * (t1 - (y + 1 / th) * torch.log((1 + th * y) / (1 + th * m)))
        raise ValueError(n)

    def loglik(self, y, mu, w, phi):
        """Weighted log-likelihood at dispersion ``phi`` (GLMModel likelihood for calc_like)."""
        n = self.name
        if n == "gaussian":
            return _gsum((w * (-0.5 * (y - mu) ** 2 / phi - 0.5 * math.log(2 * math.pi * phi))).sum())
        if n in ("binomial", "quasibinomial", "fractionalbinomial"):
            m = mu.clamp(1e-15, 1 - 1e-15)
            return _gsum((w * (y * torch.log(m) + (1 - y) * torch.log(1 - m))).sum())
        if n == "poisson":
            return _gsum((w * (y * torch.log(mu.clamp(min=1e-300)) - mu - torch.lgamma(y + 1))).sum())
        if n == "gamma":
            k = 1.0 / phi
            yc = y.clamp(min=1e-300)
            return _gsum((w * (k * torch.log(k * yc / mu) - k * yc / mu - torch.log(yc) - math.lgamma(k))).sum())
        if n == "negativebinomial":
            th = self.theta
            r = 1.0 / th
            return _gsum((w * (torch.lgamma(y + r) - torch.lgamma(y + 1) - math.lgamma(r) + r * math.log(r)
                               - r * torch.log(r + mu) + y * torch.log(mu.clamp(min=1e-300))
                               - y * torch.log(r + mu))).sum())
        return float("nan")

    def loglik_aic(self, y, mu, w, dev_sum, nobs, rank):
        n = self.name
        if n == "gaussian":
            W = _gsum(w.sum())
            return float(W * (math.log(2 * math.pi * dev_sum / W) + 1) + 2) + 2 * rank
        if n in ("binomial", "quasibinomial", "fractionalbinomial"):
            return dev_sum + 2 * rank
        if n == "poisson":
            ll = _gsum((w * (y * torch.log(mu.clamp(min=1e-300)) - mu - torch.lgamma(y + 1))).sum())
            return float(-2 * ll) + 2 * rank
        return float("nan")


def estimate_dispersion(family, y, mu, w, nobs, rank, res_dev, method="pearson", max_it=50, eps=1e-4):
    """Dispersion φ (GLM.java estimateDispersion / dispersion_parameter_method): ``pearson`` Σ w(y-μ)²/V(μ) /
    (n - p), ``deviance`` D / (n - p), ``ml`` maximum likelihood (gaussian: D / n; gamma: Newton on the shape
    1/φ; negative binomial: Newton on θ with μ fixed). Families without a dispersion return 1."""
    n = family.name
    if n in ("binomial", "poisson", "quasibinomial", "fractionalbinomial", "multinomial", "ordinal"):
        return 1.0
    dfree = max(nobs - rank, 1)
    method = str(method).lower()
    if method == "deviance":
        return res_dev / dfree
    if method == "ml":
        if n == "gaussian":
            return res_dev / max(nobs, 1)
        if n == "gamma":
            from scipy.special import digamma, polygamma
            yc = y.clamp(min=1e-300)
            W = _gsum(w.sum())
            c = _gsum((w * (torch.log(yc / mu) - yc / mu)).sum())
            k = 1.0 / max(estimate_dispersion(family, y, mu, w, nobs, rank, res_dev, "pearson"), 1e-8)
            for _ in range(max_it):
                g = W * (math.log(k) + 1 - float(digamma(k))) + c
                h = W * (1.0 / k - float(polygamma(1, k)))
                nk = k - g / h if h != 0 else k
                nk = nk if nk > 0 else k / 2
                if abs(nk - k) < eps * k:
                    k = nk
                    break
                k = nk
            return 1.0 / k
        if n == "negativebinomial":
            from scipy.special import digamma, polygamma
            yy, mm_, ww = y.double().cpu().numpy(), mu.double().cpu().numpy(), w.double().cpu().numpy()
            th = max(family.theta, 1e-3)
            for _ in range(max_it):       # d/dθ of the NB log-likelihood (r = 1/θ), Newton in r
                r = 1.0 / th
                g = (ww * (digamma(yy + r) - digamma(r) + np.log(r) + 1 - np.log(r + mm_) - (yy + r) / (r + mm_))).sum()
                h = (ww * (polygamma(1, yy + r) - polygamma(1, r) + 1 / r - 2 / (r + mm_)
                           + (yy + r) / (r + mm_) ** 2)).sum()
                nr = r - g / h if h != 0 else r
                nr = nr if nr > 0 else r / 2
                if abs(nr - r) < eps * r:
                    r = nr
                    th = 1.0 / r
                    break
                th = 1.0 / nr
            return th
        raise ValueError(f"dispersion_parameter_method='ml' is not available for family {n}")
    return _gsum((w * (y - mu) ** 2 / family.variance(mu).clamp(min=1e-30)).sum()) / dfree


def tweedie_loglik(y, mu, w, p, phi, eps=8e-17, max_rows=200_000):
    """Weighted Tweedie log-likelihood for 1 < p < 2 (compound Poisson-gamma; ``TweedieEstimator``): the
    density of y > 0 by Dunn & Smyth's series W = sum_j W_j evaluated in log space over the window of
    significant terms around j_max = y^(2-p) / (phi (2-p)) (terms below ``eps`` x the largest are dropped),
    y = 0 in closed form. Row-sharded: rows of a fixed global-index sample, sums all-reduced."""
    y, mu, w = y.double(), mu.double().clamp(min=1e-300), w.double()
    if y.numel() > max_rows:
        sel = torch.linspace(0, y.numel() - 1, max_rows, device=y.device).long()
        scale = y.numel() / max_rows
        y, mu, w = y[sel], mu[sel], w[sel] * scale
    a = (2 - p) / (1 - p)
    kappa = mu ** (2 - p) / (2 - p)
    ll = -kappa / phi
    pos = y > 0
    if bool(pos.any()):
        yp, mp = y[pos], mu[pos]
        z = -a * torch.log(yp) + a * math.log(p - 1) - (1 - a) * math.log(phi) - math.log(2 - p)
        jmax = (yp ** (2 - p) / (phi * (2 - p))).clamp(min=1.0)
        sd = float(jmax.max().sqrt())
        half = int(min(4096, math.ceil(math.sqrt(max(-2 * math.log(eps), 1.0)) * 2 * sd + 20)))
        j0 = (jmax.round() - half).clamp(min=1.0)
        j = j0[:, None] + torch.arange(2 * half + 1, dtype=torch.float64, device=y.device)[None, :]
        lw = j * z[:, None] - torch.lgamma(1 + j) - torch.lgamma(-j * a)
        logW = torch.logsumexp(lw, 1)
        ll_pos = -torch.log(yp) + logW + (yp * mp ** (1 - p) / (1 - p) - mp ** (2 - p) / (2 - p)) / phi
        ll = ll.clone()
        ll[pos] = ll_pos
    return _gsum((w * ll).sum())


def estimate_tweedie(y, mu, w, p0, phi0, fix_phi=False, learning_rate=0.5, eps=8e-17):
    """ML (p, phi) of the Tweedie family with mu fixed (GLM.updateTweediePandPhi / updateTweedieVariancePower:
    Nelder-Mead over the likelihood; p kept in (1, 2), phi > 0)."""
    from scipy.optimize import minimize

    def nll(v):
        pp = 1 + 1 / (1 + math.exp(-v[0]))                     # (1, 2)
        ph = phi0 if fix_phi else math.exp(v[1])
        val = tweedie_loglik(y, mu, w, pp, ph, eps)
        return -val if math.isfinite(val) else 1e300

    pc = p0 if 1 < p0 < 2 else 1.5
    x0 = [math.log((pc - 1) / (2 - pc)), math.log(max(phi0, 1e-10))]
    step = max(learning_rate, 1e-3)
    simplex = [x0, [x0[0] + step, x0[1]], [x0[0], x0[1] + step]]
    r = minimize(nll, x0, method="Nelder-Mead",
                 options=dict(initial_simplex=simplex, xatol=1e-6, fatol=1e-9, maxiter=400))
    pp = 1 + 1 / (1 + math.exp(-r.x[0]))
    return pp, (phi0 if fix_phi else math.exp(r.x[1])), -float(r.fun)


def variance_inflation_factors(ex, X, w):
    """VIF of every numeric predictor: 1 / (1 - R²_j) of regressing it on the other numeric predictors,
    = diag(R⁻¹) of their weighted correlation matrix (GLM generate_variable_inflation_factors)."""
    if len(ex.nums) < 2:
        return {ex.info.x[j]: float("nan") for j in ex.nums}
    Xn = torch.stack([torch.nan_to_num(X[j].double(), nan=float(ex.num_mean[i])) for i, j in enumerate(ex.nums)], 1)
    wd = w.double()
    W = _gsum(wd.sum())
    mu = _gvec((Xn * wd[:, None]).sum(0)) / W
    Xc = Xn - mu
    C = _gvec((Xc * wd[:, None]).T @ Xc) / W
    sd = C.diagonal().clamp(min=1e-300).sqrt()
    R = C / (sd[:, None] * sd[None, :])
    v = torch.linalg.pinv(R).diagonal()
    return {ex.info.x[j]: float(v[i]) for i, j in enumerate(ex.nums)}


# ------------------------------------------------------------------------------------------------
class GLMModel(Model):
    algo = "glm"

    def get_regression_influence_diagnostics(self):
        """Frame of the DFBETAS columns computed with ``influence='dfbetas'`` (GLMModel RID frame)."""
        fr = getattr(self, "_rid", None)
        if fr is None:
            raise ValueError("train the GLM with influence='dfbetas' first")
        return fr

    def __init__(self, key, params, info):
        super().__init__(key, params, info)
        self.expander: Expander | None = None
        self.beta = None        # standardized-space coefficients [K, P+1] (last = intercept)
        self.family = None

    def _eta(self, X, offset=None):
        if getattr(self, "hglm", None) is not None:
            from .hglm import hglm_eta
            return hglm_eta(self, X, offset)
        Z = self.expander.transform(X.to(self.device))
        b = self.beta.to(Z.device)
        eta = G.zbeta(Z, b[:, :-1].T.contiguous()) + b[:, -1]
        if offset is not None:
            eta = eta + offset.double()[:, None]
        return eta

    def _predict_tensor(self, X, offset=None):
        return self._from_eta(self._eta(X, offset))

    def _from_eta(self, eta):
        fam = self.output["family"]
        if fam == "multinomial":
            return torch.softmax(eta, 1).float()
        if fam == "ordinal":
            th = torch.as_tensor(self.output["ordinal_thresholds"], dtype=torch.float64, device=eta.device)
            cdf = torch.sigmoid(th[None, :] - eta[:, :1])
            cdf = torch.cat([cdf, torch.ones_like(cdf[:, :1])], 1)
            probs = torch.diff(torch.cat([torch.zeros_like(cdf[:, :1]), cdf], 1), dim=1).clamp(min=0)
            return probs.float()
        f = Family(fam, self.output["link"], self.params.get("tweedie_variance_power", 0.0),
                   self.params.get("tweedie_link_power", 1.0), self.params.get("theta", 1e-10))
        mu = f.linkinv(eta[:, 0])
        if fam in ("binomial", "quasibinomial", "fractionalbinomial") and self.model_category == "Binomial":
            return torch.stack([1 - mu, mu], 1).float()
        return mu.float()

    def metrics_for(self, X, y, w=None, offset=None):
        """ModelMetrics*GLM of a scored frame: the family metrics plus residual / null deviance (null model = the
        training mean response through the link, with the frame's offset), their degrees of freedom and AIC
        (hex/glm/GLMMetricBuilder)."""
        m = super().metrics_for(X, y, w, offset)
        fam = self.output.get("family")
        if m is None or fam in ("multinomial", "ordinal") or getattr(self, "hglm", None) is not None:
            return m
        dev = self.device
        f = Family(fam, self.output["link"], self.params.get("tweedie_variance_power", 0.0),
                   self.params.get("tweedie_link_power", 1.0), self.params.get("theta", 1e-10))
        eta = self._eta(X, offset)[:, 0]
        mu = f.linkinv(eta)
        yy = y.to(dev).double()
        ww = torch.ones_like(yy) if w is None else w.to(dev).double()
        ok = ~torch.isnan(yy) & (ww > 0)
        yy, ww, mu = yy[ok], ww[ok], mu[ok]
        res_dev = float((ww * f.deviance(yy, mu)).sum())
        ymu = self.output.get("training_ymu")
        if ymu is None:
            ymu = float((ww * yy).sum() / ww.sum().clamp(min=1e-300))
        null_eta = f.linkfn(torch.full_like(yy, float(ymu)))
        if offset is not None:
            null_eta = null_eta + offset.to(dev).double()[ok]
        null_dev = float((ww * f.deviance(yy, f.linkinv(null_eta))).sum())
        nobs = int(ok.sum())
        rank = int((self.beta.abs() > 0).sum())
        m.update(residual_deviance=res_dev, null_deviance=null_dev,
                 null_degrees_of_freedom=nobs - (1 if self.params.get("intercept", True) else 0),
                 residual_degrees_of_freedom=nobs - rank,
                 AIC=f.loglik_aic(yy, mu, ww, res_dev, nobs, rank))
        return m

    def predict_labels(self, P):
        """Ordinal (GLMModel.score0): the first class whose cumulative probability exceeds 1/2 (eta_c > 0), else the
        last class — the median of the predicted distribution, not its mode."""
        if self.output.get("family") != "ordinal" or P.dim() != 2:
            return None
        cum = P.double().cumsum(1)[:, :-1] > 0.5
        K = P.shape[1]
        first = torch.where(cum.any(1), cum.int().argmax(1), torch.full_like(cum[:, 0], K - 1, dtype=torch.long))
        return first

    # ---- h2o-py accessors
    def coef(self):
        return self.output.get("coefficients")

    def coef_norm(self):
        return self.output.get("standardized_coefficients")

    def null_deviance(self, train=True, valid=False, xval=False):
        return self.output.get("null_deviance")

    def residual_deviance(self, train=True, valid=False, xval=False):
        return self.output.get("residual_deviance")

    def aic(self, train=True, valid=False, xval=False):
        return self.output.get("aic")

    def null_degrees_of_freedom(self, *a, **k):
        return self.output.get("null_degrees_of_freedom")

    def residual_degrees_of_freedom(self, *a, **k):
        return self.output.get("residual_degrees_of_freedom")

    def to_state(self):
        s = super().to_state()
        s["beta"] = self.beta.cpu().tolist()
        s["expander"] = self.expander.to_state()
        hg = getattr(self, "hglm", None)
        if hg is not None:
            s["hglm"] = dict(hg, u=hg["u"].cpu().tolist())
        return s

    def _restore(self, s):
        super()._restore(s)
        self.beta = torch.tensor(s["beta"], dtype=torch.float64)
        hg = s.get("hglm")
        if hg is not None:
            from .base import DataInfo
            fi = hg["fixed_idx"]
            finfo = DataInfo([self.info.x[j] for j in fi], np.asarray(self.info.iscat)[fi],
                             [self.info.domains[j] for j in fi], self.info.response, self.info.response_domain)
            self.expander = Expander.from_state(finfo, s["expander"])
            self.hglm = dict(hg, u=torch.tensor(hg["u"], dtype=torch.float64))
        else:
            self.expander = Expander.from_state(self.info, s["expander"])

    def coefs_random(self):
        """Random-effect coefficients of an HGLM model (``ubeta`` by level)."""
        return self.output.get("random_coefficients")

    @staticmethod
    def getGLMRegularizationPath(model):
        return model.output.get("regularization_path")


# ------------------------------------------------------------------------------------------------
def _gsum(x) -> float:
    """Global sum of a per-rank scalar partial (row-sharded training; identity otherwise)."""
    v = float(x)
    return coll.all_reduce_scalar(v) if coll.is_dist() else v


def _gvec(t: torch.Tensor) -> torch.Tensor:
    """Global sum of a per-rank vector partial (in place)."""
    return coll.all_reduce_(t) if coll.is_dist() else t


def _soft(x, t):
    return torch.sign(x) * (x.abs() - t).clamp(min=0)


def solve_penalized(Gm, r, l1, l2, intercept, beta0=None, non_negative=False, max_iter=500, tol=1e-8, lb=None, ub=None):
    """min ½βᵀGβ - rᵀβ + l2/2‖β₋₀‖² + l1‖β₋₀‖₁ (last coefficient = intercept, unpenalized), optionally
    inside the box ``lb <= β <= ub`` (beta_constraints: projected coordinate descent)."""
    P = Gm.shape[0]
    pen = torch.ones(P, dtype=torch.float64, device=Gm.device)
    if intercept:
        pen[-1] = 0
    boxed = lb is not None or ub is not None
    if l1 == 0 and not non_negative and not boxed:
        A = Gm + torch.diag(l2 * pen)
        jitter = 0.0
        for _ in range(6):
            try:
                L = torch.linalg.cholesky(A + jitter * torch.eye(P, dtype=A.dtype, device=A.device))
                return torch.cholesky_solve(r[:, None], L)[:, 0]
            except Exception:  # noqa: BLE001 - singular Gram: add ridge jitter (Gram.java addDiag)
                jitter = 1e-8 if jitter == 0 else jitter * 100
        return torch.linalg.lstsq(A, r[:, None]).solution[:, 0]
    # cyclic coordinate descent on the Gram: native C++ (csrc/glm_solver.cpp) on the host copy of G (P x P)
    import ctypes
    from ..ops import _native as nat
    b = torch.zeros(P, dtype=torch.float64, device=Gm.device) if beta0 is None else beta0.clone()
    Gh = np.ascontiguousarray(Gm.double().cpu().numpy())
    rh = np.ascontiguousarray(r.double().cpu().numpy())
    bh = np.ascontiguousarray(b.double().cpu().numpy())
    penh = np.ascontiguousarray(pen.cpu().numpy())
    nan = np.full(P, np.nan)
    lbh = np.ascontiguousarray(nan if lb is None else np.where(np.isinf(lb.cpu().numpy()), np.nan, lb.cpu().numpy()))
    ubh = np.ascontiguousarray(nan if ub is None else np.where(np.isinf(ub.cpu().numpy()), np.nan, ub.cpu().numpy()))
    lib = nat.rt()
    fn = lib.h2o_gram_cd
    dp = ctypes.POINTER(ctypes.c_double)
    fn.argtypes = [dp, dp, ctypes.c_int, ctypes.c_double, ctypes.c_double, dp, ctypes.c_int, dp, dp, dp, ctypes.c_int,
                   ctypes.c_double]
    fn.restype = ctypes.c_int
    ptr = lambda a_: a_.ctypes.data_as(dp)  # noqa: E731
    fn(ptr(Gh), ptr(rh), P, float(l1), float(l2), ptr(penh), int(bool(non_negative)), ptr(lbh), ptr(ubh), ptr(bh),
       int(max_iter), float(tol))
    return torch.as_tensor(bh, device=Gm.device)


class GLMTrainer:
    def __init__(self, params):
        p = dict(GLM_DEFAULTS)
        if "lambda" in params:
            params = dict(params)
            params["lambda_"] = params.pop("lambda")
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None
        self.penalty = None     # optional (P+1)x(P+1) quadratic penalty (GAM)
        self.lower_bounds = None  # optional (P+1) coefficient lower bounds (GAM I-splines)

    def _family(self, info):
        fam = canon(self.p["family"])
        if fam == "auto":
            if info.response_domain is None:
                fam = "gaussian"
            else:
                fam = "binomial" if len(info.response_domain) == 2 else "multinomial"
        if info.response_domain is not None and fam not in ("binomial", "quasibinomial", "multinomial", "ordinal",
                                                            "fractionalbinomial"):
            raise ValueError(f"family {self.p['family']!r} needs a numeric response; {info.response!r} is categorical")
        link = canon(self.p["link"])
        if link in ("familydefault", "auto", ""):
            link = DEFAULT_LINK[fam]
        return fam, link

    def _validate(self, fam, link, y, info):
        """The reference's family / solver checks (``hex/glm/GLM.java:876-953``), on global response ranges."""
        def err(field, msg):     # ModelBuilder.error(): "ERRR on field: _family: ..."
            raise ValueError(f"ERRR on field: _{field}: {msg}")
        solver = canon(self.p["solver"])
        if solver in ("gradientdescentlh", "gradientdescentsqerr") and fam != "ordinal":
            err("solver", "Solvers GRADIENT_DESCENT_LH and GRADIENT_DESCENT_SQERR are only supported for ordinal "
                           "regression.  Do not choose them unless you specify your family to be ordinal")
        ncls = len(info.response_domain) if info.response_domain is not None else 1
        yy = y[~torch.isnan(y)] if y is not None else None
        lo = float(coll.all_reduce_scalar(float(yy.min()) if yy is not None and yy.numel() else float("inf"),
                                          op=_MIN)) if yy is not None else 0.0
        hi = float(coll.all_reduce_scalar(float(yy.max()) if yy is not None and yy.numel() else float("-inf"),
                                          op=_MAX)) if yy is not None else 0.0
        # Vec.isBinary is a property of the whole column: the local 0/1 test is reduced (MIN over the ranks) so
        # that every rank raises, or none does, before the GLM collectives start
        binary = 1.0
        if fam == "binomial" and ncls == 1 and yy is not None:
            binary = float(coll.all_reduce_scalar(1.0 if bool(((yy == 0) | (yy == 1)).all()) else 0.0, op=_MIN))
        if fam == "binomial" and ncls != 2 and not (ncls == 1 and lo >= 0 and hi <= 1 and binary > 0.5):
            err("family", "Binomial requires the response to be a 2-class categorical or a binary column (0/1)")
        if fam in ("multinomial", "ordinal") and ncls <= 2:
            err("family", f"{fam.capitalize()} requires a categorical response with at least 3 levels (for 2 class "
                           "problem use family=binomial.")
        if fam == "ordinal" and link in ("oprobit", "ologlog"):
            err("family", "Ordinal regression only supports ologit as link.")
        if fam in ("poisson", "negativebinomial"):
            if ncls != 1:
                err("family", "Poisson and Negative Binomial require the response to be numeric.")
            if lo < 0:
                err("family", "Poisson and Negative Binomial require response >= 0")
            if fam == "negativebinomial" and float(self.p["theta"]) <= 0:
                err("theta", "Illegal Negative Binomial theta value.  Valid theta values be > 0 and <= 1.")
        if fam == "gamma" and lo <= 0:
            err("family", "Response value for gamma distribution must be greater than 0.")
        if fam in ("tweedie", "quasibinomial") and ncls != 1:
            err("family", f"{fam.capitalize()} requires the response to be numeric.")
        if fam == "fractionalbinomial" and (lo < 0 or hi > 1):
            err("response_column", f"Response '{info.response}' must be between 0 and 1 for fractional_binomial family. "
                                     f"Min: {lo:f}, Max: {hi:f}")

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        t0 = time.time()
        p = self.p
        dev = X.device
        if p.get("HGLM"):
            from .hglm import fit_hglm
            model = GLMModel(model_key or make_key("glm"), p, info)
            model.device = dev
            fit_hglm(self, X, y, w, offset, info, model, p)
            model.output["training_metrics"] = model.metrics_for(X, y, w, offset)
            if valid is not None:
                Xv, yv, wv, ov = valid
                model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv, ov)
            model.output["run_time_ms"] = int((time.time() - t0) * 1000)
            return model
        fam, link = self._family(info)
        self._validate(fam, link, y, info)
        N = X.shape[1]
        w = torch.ones(N, dtype=torch.float64, device=dev) if w is None else w.double()
        y = y.double()
        ok = ~torch.isnan(y)
        if canon(p["missing_values_handling"]) == "skip":
            ok &= ~torch.isnan(X).any(0)
        w = torch.where(ok, w, torch.zeros_like(w))
        y = torch.where(ok, y, torch.zeros_like(y))
        off = torch.zeros(N, dtype=torch.float64, device=dev) if offset is None else offset.double()
        ex = Expander(info, standardize=p["standardize"], use_all_factor_levels=p["use_all_factor_levels"] or
                      fam == "multinomial", missing=p["missing_values_handling"],
                      plug_values=p.get("plug_values")).fit(X, w, reduce=coll.all_reduce_ if coll.is_dist() else None)
        intercept = bool(p["intercept"])
        Zi = ex.transform(X, extra=1.0 if intercept else 0.0)  # [N, P + 1] f32: the design + intercept column
        alpha = p["alpha"]
        alpha = float((alpha if isinstance(alpha, (int, float)) else alpha[0]) if alpha is not None else
                      (0.0 if canon(p["solver"]) == "lbfgs" else 0.5))
        W = float(coll.all_reduce_scalar(float(w.sum())) if coll.is_dist() else w.sum())
        nobs = int(coll.all_reduce_scalar(float((w > 0).sum()))) if coll.is_dist() else int((w > 0).sum())
        obj_reg = float(p["obj_reg"]) if p["obj_reg"] and p["obj_reg"] > 0 else 1.0 / W
        model = GLMModel(model_key or make_key("glm"), p, info)
        model.device = dev
        model.expander = ex
        model.output.update(family=fam, link=link, alpha=alpha)
        solver = canon(p["solver"])
        self._ck_beta, self._ck_iter, self._n_iter, self._tweedie_phi = None, 0, None, None
        if p.get("checkpoint"):
            self._checkpoint(p, fam, link, solver, info, ex, model)
        if fam == "multinomial" and solver != "lbfgs":
            beta, path = self._fit_multinomial_irls(Zi, y, w, off, alpha, obj_reg, intercept, info, nobs)
            lam_best = path[-1]["lambda"] if path else 0.0
        elif fam in ("multinomial", "ordinal") or solver == "lbfgs":
            beta, path = self._fit_lbfgs_or_multi(fam, link, Zi, y, w, off, alpha, obj_reg, intercept, info, ex)
            lam_best = path[-1]["lambda"] if path else 0.0
        else:
            family = Family(fam, link, float(p["tweedie_variance_power"]), float(p["tweedie_link_power"]), float(p["theta"]))
            beta, path, lam_best = self._fit_irls(family, Zi, y, w, off, alpha, obj_reg, intercept, valid, ex, nobs)
            if fam == "tweedie" and p.get("fix_tweedie_variance_power") is False:
                beta, path, lam_best, family = self._tweedie_power(family, beta, Zi, y, w, off, alpha, obj_reg, intercept,
                                                                   valid, ex, nobs, model)
            beta = beta[None, :]
        pr = float(p.get("prior") if p.get("prior") is not None else -1.0)
        if pr != -1.0:
            # GLM.java: prior probability of y == 1 when the training rows were sampled; the intercept moves by
            # -log(ymu (1 - prior) / (prior (1 - ymu))) once the fit is done
            if not 0.0 < pr < 1.0:
                raise ValueError("prior must be in (exclusive) range (0,1)")
            if fam != "binomial":
                raise ValueError("prior is only allowed with family = binomial")
            sw = float(coll.all_reduce_scalar(float((w * y).sum())) if coll.is_dist() else (w * y).sum())
            ymu = sw / W
            beta = beta.clone()
            beta[..., -1] += -math.log(ymu * (1 - pr) / (pr * (1 - ymu)))
            for e in path:
                if e.get("coefs") is not None:
                    e["coefs"] = list(e["coefs"])
                    e["coefs"][-1] = float(e["coefs"][-1]) - math.log(ymu * (1 - pr) / (pr * (1 - ymu)))
        model.beta = beta
        if getattr(self, "_n_iter", None) is not None:
            model.output["iterations"] = self._n_iter
        model.output["lambda_best"] = lam_best
        model.output["lambda"] = [e["lambda"] for e in path]
        model.output["regularization_path"] = dict(lambdas=[e["lambda"] for e in path], alphas=[alpha] * len(path),
                                                   explained_deviance_train=[e.get("dev_explained") for e in path],
                                                   coefficients=[self._path_raw(ex, e.get("coefs")) for e in path],
                                                   coefficients_std=[e.get("coefs") for e in path],
                                                   coefficient_names=ex.names + ["Intercept"])
        self._outputs(model, fam, link, Zi, y, w, off, ex, nobs, X, offset)
        if getattr(self, "collinear", None) is not None:
            model.output["removed_collinear_columns"] = list(self.collinear)
        if valid is not None:
            Xv, yv, wv, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv, ov)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model

    def _checkpoint(self, p, fam, link, solver, info, ex, model):
        """Continue from a previous GLM (GLM.java: checkpoint is IRLSM only; the previous coefficients start
        the IRLS iterations, whose count continues from the checkpoint's; scoring history carries over)."""
        from ..core import dkv
        ck = p["checkpoint"]
        prev = dkv.get(ck) if isinstance(ck, str) else getattr(ck, "_model", ck)
        if prev is None or getattr(prev, "algo", None) != "glm":
            raise ValueError(f"checkpoint {ck!r} is not a GLM model")
        if solver != "irlsm":
            raise ValueError("GLM checkpoint is supported only for IRLSM.  Please specify it explicitly.  "
                             "Do not use AUTO or default")
        if fam in ("multinomial", "ordinal"):
            raise ValueError("GLM checkpoint is supported for single-response families only")
        for k, mine, theirs in (("family", fam, prev.output.get("family")), ("link", link, prev.output.get("link")),
                                ("x", list(info.x), list(prev.info.x)), ("response", info.response, prev.info.response)):
            if mine != theirs:
                raise ValueError(f"checkpoint: {k} cannot change ({theirs!r} -> {mine!r})")
        self._ck_iter = int(prev.output.get("iterations") or 0)
        raw = self._std_to_raw(prev.expander, prev.beta[0].double())
        self._ck_beta = self._raw_to_std(ex, raw)
        model.output["scoring_history"] = list(prev.output.get("scoring_history") or [])
        model.output["checkpoint"] = prev.key

    def _tweedie_power(self, family, beta, Zi, y, w, off, alpha, obj_reg, intercept, valid, ex, nobs, model):
        """fix_tweedie_variance_power = False (GLM.java Tweedie p / phi estimation): alternate the IRLSM fit of
        beta at the current power with the ML (p, phi) of the fitted means, until p moves less than
        dispersion_epsilon (reference defaults: start p = tweedie_variance_power, phi = init_dispersion_parameter)."""
        p = self.p
        if str(p.get("dispersion_parameter_method") or "ml").lower() != "ml":
            raise ValueError("fix_tweedie_variance_power=False needs dispersion_parameter_method='ml'")
        lr = float(p.get("dispersion_learning_rate") or 0.5)
        if lr <= 0:
            raise ValueError("dispersion_learning_rate must > 0")
        teps = float(p.get("tweedie_epsilon") or 8e-17)
        if teps <= 0:
            raise ValueError("tweedie_epsilon must exceed 0.")
        fix_phi = bool(p.get("fix_dispersion_parameter"))
        pw, phi = float(p["tweedie_variance_power"]), float(p.get("init_dispersion_parameter") or 1.0)
        deps = float(p.get("dispersion_epsilon") or 1e-4)
        hist = []
        path = lam = None
        for it in range(int(p.get("max_iterations_dispersion") or 10)):
            mu = family.linkinv(G.zbeta(Zi, beta, off))
            npw, nphi, ll = estimate_tweedie(y, mu, w, pw, phi, fix_phi, lr, teps)
            hist.append(dict(iteration=it, tweedie_variance_power=npw, dispersion=nphi, loglikelihood=ll))
            moved = abs(npw - pw)
            pw, phi = npw, nphi
            family = Family(family.name, family.link, pw, float(p["tweedie_link_power"]), float(p["theta"]))
            self.p = dict(p, startval=None)
            beta, path, lam = self._fit_irls(family, Zi, y, w, off, alpha, obj_reg, intercept, valid, ex, nobs,
                                             beta_init=beta)
            self.p = p
            if moved < deps:
                break
        model.output["tweedie_variance_power"] = pw
        model.output["tweedie_estimation_history"] = hist
        self._tweedie_phi = phi
        self.p = dict(p, tweedie_variance_power=pw)
        model.params["tweedie_variance_power"] = pw
        return beta, path, lam, family

    # ---- IRLSM with Gram kernel + Cholesky / COD, optional lambda path
    def _fit_irls(self, fam: Family, Zi, y, w, off, alpha, obj_reg, intercept, valid, ex, nobs, beta_init=None):
        p = self.p
        dev = Zi.device
        P1 = Zi.shape[1]
        ymu = _gsum((w * y).sum()) / _gsum(w.sum())
        beta = torch.zeros(P1, dtype=torch.float64, device=dev)
        if intercept:
            beta[-1] = float(fam.linkfn(torch.tensor([min(max(ymu, 1e-6), 1 - 1e-6) if fam.name in ("binomial", "quasibinomial", "fractionalbinomial") else ymu], dtype=torch.float64))[0])
        if beta_init is None and getattr(self, "_ck_beta", None) is not None:
            beta_init = self._ck_beta
        if beta_init is not None:            # warm start (checkpoint / Tweedie power re-fit)
            beta = beta_init.clone().to(dev)
        lb, ub = self._bounds(ex, P1, dev)
        fixed = torch.zeros(P1, dtype=torch.bool, device=dev)    # coefficients pinned at 0
        if p.get("build_null_model"):
            fixed[:-1] = True                                    # intercept-only model (GLM build_null_model)
        if p.get("startval") is not None:
            sv = torch.as_tensor([float(v) for v in p["startval"]], dtype=torch.float64, device=dev)
            if sv.numel() != P1:
                raise ValueError(f"startval needs {P1} values (coefficients in order, intercept last)")
            beta = self._raw_to_std(ex, sv)
        if p.get("remove_collinear_columns"):
            fixed |= self._collinear(Zi, w, intercept)
            self.collinear = [ex.names[j] for j in torch.nonzero(fixed[:-1]).flatten().tolist()]
        beta = torch.where(fixed, torch.zeros_like(beta), beta)
        beta_start = beta.clone()
        lam_in = p["lambda_"]
        # gradient at the null model -> lambda max: only when a lambda is derived from it (search / default lambda)
        # or a lambda path's early stopping compares against it — a single given lambda skips its two passes
        lmax = float("inf")
        if lam_in is None or (isinstance(lam_in, (list, tuple)) and len(lam_in) > 1):
            eta = G.zbeta(Zi, beta, off)
            mu = fam.linkinv(eta)
            gvec = fam.dlink(mu)
            var = fam.variance(mu)
            grad = -(_gvec(G.xtv(Zi, (w * (y - mu) / (var * gvec)).float())) * obj_reg)
            if intercept:
                grad[-1] = 0
            lmax = float(grad.abs().max()) / max(alpha, 1e-2)
        lmr = float(p["lambda_min_ratio"])
        if lmr <= 0:
            lmr = 1e-4 if (nobs >> 4) > (P1 - 1) else 1e-2
            if alpha == 0:
                lmr *= 1e-2
        if lam_in is not None:
            lambdas = [float(v) for v in (lam_in if isinstance(lam_in, (list, tuple)) else [lam_in])]
        elif p["lambda_search"]:
            nl = int(p["nlambdas"]) if int(p["nlambdas"]) > 0 else (100 if alpha > 0 else 30)
            dec = lmr ** (1.0 / max(nl - 1, 1))
            lambdas = [lmax * dec ** i for i in range(nl)]
        else:
            lambdas = [10 * lmr * lmax]
        max_it = int(p["max_iterations"]) if int(p["max_iterations"]) > 0 else (50 if fam.name != "gaussian" else 1)
        if fam.name == "gaussian" and fam.link == "identity":
            max_it = max(max_it, 1)
        ck_it = getattr(self, "_ck_iter", 0)
        if ck_it:
            if int(p["max_iterations"]) > 0 and int(p["max_iterations"]) <= ck_it:
                raise ValueError(f"checkpoint: max_iterations ({p['max_iterations']}) must exceed the checkpoint's "
                                 f"iterations ({ck_it})")
            max_it = max(max_it - ck_it, 1)
        beps = float(p["beta_epsilon"])
        path = []
        best = (float("inf"), None, None)
        null_dev = _gsum((w * fam.deviance(y, torch.full_like(y, ymu))).sum())
        # early_stopping (GLM.java lambda loop): relative train-deviance improvements of the last 5 submodels;
        # once past lambda_max with >= 5 IRLS iterations done, stop when none beats 1e-4, or (validation
        # frame) when none improved the validation deviance
        es = p.get("early_stopping", True) is not False
        hist_tr, hist_va = [0.0] * 5, [0.0] * 5
        old_tr, old_va, n_iter = null_dev, None, 0
        if valid is not None and len(lambdas) > 1:
            # GLM.java seeds the validation improvements with the null model's validation deviance
            yv0, wv0 = valid[1], valid[2]
            okv0 = ~torch.isnan(yv0)
            wv0 = torch.ones_like(yv0, dtype=torch.float64) if wv0 is None else wv0.double()
            old_va = _gsum((wv0[okv0] * fam.deviance(yv0.double()[okv0],
                                                      torch.full_like(yv0.double()[okv0], ymu))).sum())
        for li, lam in enumerate(lambdas):
            l1, l2 = lam * alpha, lam * (1 - alpha)
            if p.get("cold_start") and li > 0:     # cold_start: every lambda starts from the initial coefficients
                beta = beta_start.clone()
            for it in range(max(max_it, 1)):
                # one pass over Z: eta / wi / zi evaluated inside the augmented Gram pass (P + 1 <= 64)
                gr = G.gram_irls(Zi, beta, off, y, w, fam.name, fam.link)
                if gr is None:
                    wz = G.irls_wz(Zi, beta, off, y, w, fam.name, fam.link)   # fused: one pass, fp32 wi / zi
                    if wz is None:
                        eta = G.zbeta(Zi, beta, off)
                        mu = fam.linkinv(eta)
                        gp = fam.dlink(mu)
                        var = fam.variance(mu)
                        wz = ((w / (var * gp * gp).clamp(min=1e-30)).float(), (eta - off + (y - mu) * gp).float())
                    gr = G.gram(Zi, wz[0], wz[1])      # one pass: Zᵀ W Z and Zᵀ W z
                Gm, r = gr
                if coll.is_dist():
                    Gm = coll.all_reduce_(Gm)
                    r = coll.all_reduce_(r)
                Gm = Gm * obj_reg
                r = r * obj_reg
                if self.penalty is not None:          # GAM smoothness penalty (standardized space)
                    Gm = Gm + self.penalty.to(Gm.device)
                if not intercept:
                    Gm[-1, :] = 0
                    Gm[:, -1] = 0
                    Gm[-1, -1] = 1
                    r[-1] = 0
                if bool(fixed.any()):
                    Gm[fixed, :] = 0
                    Gm[:, fixed] = 0
                    Gm[fixed, fixed] = 1
                    r[fixed] = 0
                nb = solve_penalized(Gm, r, l1, l2, intercept, beta, bool(p["non_negative"]), lb=lb, ub=ub)
                diff = float((nb - beta).abs().max())
                beta = nb
                n_iter += 1
                if self.job is not None:
                    self.job.check_cancelled()
                if diff < beps:
                    break
            eta_tr = G.zbeta(Zi, beta, off)
            mu = fam.linkinv(eta_tr)
            dev_tr = _gsum((w * fam.deviance(y, mu)).sum())
            # kept for _outputs: the training predictions / residual deviance of the returned beta are this pass's
            self._last_eta = (beta, Zi, off, eta_tr, w, y, (fam.name, fam.link), dev_tr)
            entry = dict(lambda_=lam, dev_explained=1 - dev_tr / null_dev if null_dev > 0 else 0.0,
                         coefs=beta.cpu().tolist())
            entry["lambda"] = lam
            path.append(entry)
            mapred = int(p.get("max_active_predictors") or -1)
            if mapred > 0 and int((beta[:-1].abs() > 0).sum()) > mapred and len(path) > 1:
                # GLM max_active_predictors: the path stops before the active set exceeds the limit
                path.pop()
                beta = torch.tensor(path[-1]["coefs"], dtype=torch.float64, device=dev)
                break
            score = dev_tr
            if valid is not None and len(lambdas) > 1:
                Xv, yv, wv, ov = valid
                Zv = ex.transform(Xv)
                etav = G.zbeta(Zv, beta[:-1], ov) + beta[-1]
                muv = fam.linkinv(etav)
                okv = ~torch.isnan(yv)
                wvv = torch.ones_like(yv, dtype=torch.float64) if wv is None else wv.double()
                score = _gsum((wvv[okv] * fam.deviance(yv.double()[okv], muv[okv])).sum())
            if valid is not None and len(lambdas) > 1 and score < best[0]:
                best = (score, beta.clone(), lam)
            k = (len(path) - 1) % 5
            hist_tr[k] = (old_tr - dev_tr) / old_tr if old_tr else 0.0
            old_tr = dev_tr
            if valid is not None and len(lambdas) > 1:
                hist_va[k] = (old_va - score) / old_va if old_va else 1.0
                old_va = score
            if es and len(lambdas) > 1 and lam < lmax and n_iter >= 5:
                if max(hist_tr) < 1e-4 or (valid is not None and max(hist_va) < 0):
                    break
        self._n_iter = ck_it + n_iter
        if best[1] is not None:
            return best[1], path, best[2]
        return beta, path, lambdas[-1]

    # ---- coefficient helpers (raw <-> standardized scale, beta_constraints, collinearity)
    @staticmethod
    def _std_to_raw(ex, b):
        """Inverse of :meth:`_raw_to_std` (intercept last)."""
        raw = b.clone()
        if ex.standardize and ex.nums:
            k = ex.num_off
            sd = ex.num_sd.to(b.device).double()
            mu = ex.num_mean.to(b.device).double()
            raw[k:-1] = b[k:-1] / sd
            raw[-1] = b[-1] - float((raw[k:-1] * mu).sum())
        return raw

    def _path_raw(self, ex, coefs):
        """Regularization-path coefficients on the raw scale (one list, or one per class)."""
        if coefs is None:
            return None
        b = torch.as_tensor(coefs, dtype=torch.float64)
        if b.dim() == 1:
            return self._std_to_raw(ex, b).tolist()
        return [self._std_to_raw(ex, r).tolist() for r in b]

    @staticmethod
    def _raw_to_std(ex, raw):
        """Raw-scale coefficients (intercept last) -> the standardized space the solver works in."""
        b = raw.clone()
        if ex.standardize and ex.nums:
            k = ex.num_off
            sd = ex.num_sd.to(raw.device)
            mu = ex.num_mean.to(raw.device)
            b[k:-1] = raw[k:-1] * sd
            b[-1] = raw[-1] + float((raw[k:-1] * mu).sum())
        return b

    def _bounds(self, ex, P1, dev):
        """beta_constraints (names, lower_bounds, upper_bounds) on the raw scale -> standardized bounds."""
        bc = self.p.get("beta_constraints")
        extra = getattr(self, "lower_bounds", None)       # set by GAM: non-negative I-spline coefficients
        if bc is None:
            if extra is None:
                return None, None
            return extra.to(dev), torch.full((P1,), float("inf"), dtype=torch.float64, device=dev)
        if hasattr(bc, "as_data_frame"):
            bc = bc.as_data_frame()
        import pandas as pd
        df = pd.DataFrame(bc)
        if "names" not in df.columns:
            raise ValueError("beta_constraints needs a 'names' column")
        lb = torch.full((P1,), -float("inf"), dtype=torch.float64, device=dev)
        ub = torch.full((P1,), float("inf"), dtype=torch.float64, device=dev)
        names = ex.names
        for _, row in df.iterrows():
            n = str(row["names"])
            if n not in names:
                raise ValueError(f"beta_constraints: unknown coefficient {n!r}")
            j = names.index(n)
            sc = float(ex.num_sd[j - ex.num_off]) if (ex.standardize and j >= ex.num_off) else 1.0
            if "lower_bounds" in df.columns and not pd.isna(row["lower_bounds"]):
                lb[j] = float(row["lower_bounds"]) * sc
            if "upper_bounds" in df.columns and not pd.isna(row["upper_bounds"]):
                ub[j] = float(row["upper_bounds"]) * sc
        if extra is not None:                              # GAM I-spline non-negativity on top of the user's
            lb = torch.maximum(lb, extra.to(dev))
        return lb, ub

    def _collinear(self, Zi, w, intercept):
        """remove_collinear_columns: columns whose Gram pivot (Cholesky of the weighted Gram in column
        order, intercept first) collapses are dropped (pinned to 0) — GLM.java's collinear-column check."""
        Gm = _gvec(G.gram(Zi, w.float()))
        P1 = Gm.shape[0]
        order = ([P1 - 1] if intercept else []) + list(range(P1 - 1))
        kept, drop = [], torch.zeros(P1, dtype=torch.bool, device=Gm.device)
        for j in order:
            if kept:
                A = Gm[kept][:, kept]
                bvec = Gm[kept, j]
                x = torch.linalg.lstsq(A, bvec[:, None]).solution[:, 0]
                resid = float(Gm[j, j] - bvec @ x)
            else:
                resid = float(Gm[j, j])
            if resid <= 1e-8 * max(float(Gm[j, j]), 1e-300):
                drop[j] = True
            else:
                kept.append(j)
        if intercept:
            drop[-1] = False
        return drop

    # ---- multinomial IRLSM (GLM.java fitIRLSM_multinomial): one penalized weighted least-squares
    # solve per class with the other classes' coefficients held fixed, cycled to convergence
    def _fit_multinomial_irls(self, Zi, y, w, off, alpha, obj_reg, intercept, info, nobs):
        p = self.p
        dev = Zi.device
        P1 = Zi.shape[1]
        K = len(info.response_domain)
        yl = torch.nan_to_num(y, nan=0).long().clamp(0, K - 1)
        Y = torch.nn.functional.one_hot(yl, K).double()
        B = torch.zeros(K, P1, dtype=torch.float64, device=dev)
        # null model: class log-frequencies as intercepts
        freq = _gvec((w[:, None] * Y).sum(0).contiguous())
        freq = (freq / freq.sum()).clamp(min=1e-10)
        if intercept:
            B[:, -1] = torch.log(freq) - torch.log(freq).mean()
        def probs(B):       # fp32 design, fp64 accumulation (no fp64 copy of Z)
            return torch.softmax(G.zbeta(Zi, B.T.contiguous()) + off[:, None], 1)
        lam_in = p["lambda_"]
        if lam_in is not None:
            lambdas = [float(v) for v in (lam_in if isinstance(lam_in, (list, tuple)) else [lam_in])]
        else:
            Pm = probs(B)
            g = _gvec(G.xtv(Zi, (w[:, None] * (Y - Pm)).contiguous()).contiguous()) * obj_reg    # [P1, K]
            if intercept:
                g[-1] = 0
            lmax = float(g.abs().max()) / max(alpha, 1e-2)
            lmr = float(p["lambda_min_ratio"]) if float(p["lambda_min_ratio"]) > 0 else (1e-4 if (nobs >> 4) > P1 else 1e-2)
            if alpha == 0:
                lmr *= 1e-2
            if p["lambda_search"]:
                nl = int(p["nlambdas"]) if int(p["nlambdas"]) > 0 else (100 if alpha > 0 else 30)
                dec = lmr ** (1.0 / max(nl - 1, 1))
                lambdas = [lmax * dec ** i for i in range(nl)]
            else:
                lambdas = [10 * lmr * lmax]
        max_it = int(p["max_iterations"]) if int(p["max_iterations"]) > 0 else 50
        beps = float(p["beta_epsilon"])
        path = []
        for lam in lambdas:
            l1, l2 = lam * alpha, lam * (1 - alpha)
            for it in range(max_it):
                Bold = B.clone()
                for c in range(K):
                    Pm = probs(B)
                    pc = Pm[:, c]
                    wi = (w * pc * (1 - pc)).clamp(min=1e-10 * float(w.max()) if w.numel() else 0.0)
                    eta_c = G.zbeta(Zi, B[c])
                    zi = eta_c + (Y[:, c] - pc) / (pc * (1 - pc)).clamp(min=1e-10)
                    Gm, r = G.gram(Zi, wi.float(), zi.float())
                    Gm, r = _gvec(Gm) * obj_reg, _gvec(r) * obj_reg
                    if not intercept:
                        Gm[-1, :] = 0
                        Gm[:, -1] = 0
                        Gm[-1, -1] = 1
                        r[-1] = 0
                    B[c] = solve_penalized(Gm, r, l1, l2, intercept, B[c], bool(p["non_negative"]))
                if self.job is not None:
                    self.job.check_cancelled()
                if float((B - Bold).abs().max()) < beps:
                    break
            if intercept:                        # softmax is shift-invariant: centre the intercepts
                B[:, -1] -= B[:, -1].mean()
            path.append(dict(lambda_=lam, **{"lambda": lam}, coefs=B.cpu().tolist()))
        return B, path

    # ---- multinomial / ordinal / L-BFGS: device autograd objective
    def _fit_lbfgs_or_multi(self, fam, link, Zi, y, w, off, alpha, obj_reg, intercept, info, ex):
        p = self.p
        dev = Zi.device
        Zd = Zi.double()
        P1 = Zi.shape[1]
        K = len(info.response_domain) if fam in ("multinomial", "ordinal") else 1
        lam_in = p["lambda_"]
        lam = float(lam_in if isinstance(lam_in, (int, float)) else (lam_in[0] if lam_in else 0.0)) if lam_in is not None else None
        pen = torch.ones(P1, dtype=torch.float64, device=dev)
        if intercept:
            pen[-1] = 0
        if fam == "multinomial":
            B = torch.zeros(K, P1, dtype=torch.float64, device=dev, requires_grad=True)
            yl = y.long()

            def nll(B):
                eta = Zd @ B.T + off[:, None]
                return -(w * torch.log_softmax(eta, 1).gather(1, yl[:, None])[:, 0]).sum() * obj_reg
            params = [B]
        elif fam == "ordinal":
            B = torch.zeros(1, P1, dtype=torch.float64, device=dev, requires_grad=True)
            th_raw = torch.zeros(K - 1, dtype=torch.float64, device=dev, requires_grad=True)
            yl = y.long()
            sqerr = canon(p["solver"]) == "gradientdescentsqerr"
            cls = torch.arange(K - 1, device=dev)

            def nll(B):
                th = torch.cumsum(torch.cat([th_raw[:1], torch.nn.functional.softplus(th_raw[1:])]), 0)
                eta = (Zd[:, :-1] @ B[0, :-1]) + off
                if sqerr:
                    # GRADIENT_DESCENT_SQERR (GLMTask.computeGradientMultipliersSQERR): threshold c's linear
                    # predictor e_c = th_c - eta must be negative for c < y and positive for c >= y; each
                    # violation costs 0.5 e_c^2
                    e = th[None, :] - eta[:, None]
                    below = cls[None, :] < yl[:, None]
                    viol = torch.where(below, e > 0, e <= 0)
                    return (w * (0.5 * torch.where(viol, e * e, torch.zeros_like(e))).sum(1)).sum() * obj_reg
                cdf = torch.sigmoid(th[None, :] - eta[:, None])
                cdf = torch.cat([torch.zeros_like(cdf[:, :1]), cdf, torch.ones_like(cdf[:, :1])], 1)
                pr = (cdf.gather(1, (yl + 1)[:, None]) - cdf.gather(1, yl[:, None]))[:, 0].clamp(min=1e-15)
                return -(w * torch.log(pr)).sum() * obj_reg
            params = [B, th_raw]
        else:
            family = Family(fam, link, float(p["tweedie_variance_power"]), float(p["tweedie_link_power"]), float(p["theta"]))
            B = torch.zeros(1, P1, dtype=torch.float64, device=dev, requires_grad=True)

            def nll(B):
                mu = family.linkinv(Zd @ B[0] + off)
                return 0.5 * (w * family.deviance(y, mu)).sum() * obj_reg
            params = [B]
        if lam is None:
            Bz = B.detach().clone().requires_grad_(True)
            g = _gvec(torch.autograd.grad(nll(Bz), Bz)[0].contiguous())
            lmax = float((g * pen).abs().max()) / max(alpha, 1e-2)
            nobs = int(_gsum((w > 0).sum()))
            lmr = float(p["lambda_min_ratio"]) if float(p["lambda_min_ratio"]) > 0 else (1e-4 if (nobs >> 4) > P1 else 1e-2)
            if alpha == 0:
                lmr *= 1e-2
            lam = 10 * lmr * lmax
        l1, l2 = lam * alpha, lam * (1 - alpha)
        opt = torch.optim.LBFGS(params, lr=1.0, max_iter=int(p["max_iterations"]) if int(p["max_iterations"]) > 0 else 500,
                                tolerance_grad=1e-9, tolerance_change=1e-12, history_size=20, line_search_fn="strong_wolfe")

        def closure():
            # the data term is a sum over rows: its value and gradient are all-reduced over the shards, so
            # every rank takes the identical L-BFGS step; the penalty is added once, after the reduce
            opt.zero_grad()
            data = nll(B)
            data.backward()
            if coll.is_dist():
                for prm in params:
                    if prm.grad is not None:
                        coll.all_reduce_(prm.grad)
            pen_term = 0.5 * l2 * ((B * pen) ** 2).sum() + l1 * torch.sqrt((B * pen) ** 2 + 1e-12).sum()
            pen_term.backward()
            return torch.tensor(_gsum(data.detach()) + float(pen_term.detach()), dtype=torch.float64)
        opt.step(closure)
        Bd = B.detach()
        if l1 > 0:
            Bd = torch.where(Bd.abs() < 1e-6 * max(1.0, float(Bd.abs().max())), torch.zeros_like(Bd), Bd)
        if fam == "ordinal":
            th = torch.cumsum(torch.cat([th_raw[:1], torch.nn.functional.softplus(th_raw[1:])]), 0).detach()
            self._ordinal_th = th.cpu().tolist()
        return Bd, [dict(lambda_=lam, **{"lambda": lam}, coefs=Bd.cpu().tolist())]

    # ---- coefficient tables, deviances, AIC, p-values, metrics
    def _outputs(self, model, fam, link, Zi, y, w, off, ex, nobs, X, offset):
        p = self.p
        beta = model.beta
        names = ex.names + ["Intercept"]
        out = model.output
        if fam == "ordinal":
            out["ordinal_thresholds"] = self._ordinal_th
        K = beta.shape[0]
        same_dev = None
        coefs, coefs_std = {}, {}
        for k in range(K):
            braw, ic = ex.destandardize(beta[k, :-1], float(beta[k, -1]))
            suffix = "" if K == 1 else f"_{model.info.response_domain[k]}"
            coefs_std.update({n + suffix: float(v) for n, v in zip(names, beta[k].cpu().tolist())})
            coefs.update({n + suffix: float(v) for n, v in zip(ex.names, braw.cpu().tolist())})
            coefs["Intercept" + suffix] = ic
        out["coefficients"] = coefs
        out["standardized_coefficients"] = coefs_std
        out["coefficients_table"] = [dict(names=n, coefficients=coefs[n], standardized_coefficients=coefs_std.get(n))
                                     for n in coefs]
        if fam not in ("multinomial", "ordinal") and K == 1 and getattr(model, "hglm", None) is None:
            # training predictions from the training design (it already holds the intercept column): no second
            # expander transform of X
            le, self._last_eta = getattr(self, "_last_eta", None), None
            if (le is not None and le[1] is Zi and le[2] is off and le[0].shape == beta[0].shape
                    and torch.equal(le[0].to(beta.device, torch.float64), beta[0].double())):
                eta = le[3]                    # the fit's last deviance pass already holds Z.beta + off
                same_dev = le                  # ... and the residual deviance of that beta (checked below)
            else:
                eta = G.zbeta(Zi, beta[0].to(Zi.device), off)
            P = model._from_eta(eta[:, None])
        else:
            P = model._predict_tensor(X, offset)
        cat = model.model_category
        yv = y.float()
        ok = w > 0
        if fam not in ("multinomial", "ordinal"):
            family = Family(fam, link, float(p["tweedie_variance_power"]), float(p["tweedie_link_power"]), float(p["theta"]))
            mu = (P[:, 1] if P.dim() == 2 else P).double()
            if (same_dev is not None and same_dev[4] is w and same_dev[5] is y and fam != "tweedie"
                    and same_dev[6] == (family.name, family.link)):
                res_dev = same_dev[7]
            else:
                res_dev = _gsum((w * family.deviance(y, mu)).sum())
            ymu = _gsum((w * y).sum()) / _gsum(w.sum())
            out["training_ymu"] = float(ymu)
            null_mu = torch.full_like(y, ymu)
            if offset is not None:
                null_mu = family.linkinv(family.linkfn(null_mu) + off)
            null_dev = _gsum((w * family.deviance(y, null_mu)).sum())
            rank = int((beta[0].abs() > 0).sum())
            out.update(residual_deviance=res_dev, null_deviance=null_dev, null_degrees_of_freedom=nobs - (1 if p["intercept"] else 0),
                       residual_degrees_of_freedom=nobs - rank, aic=family.loglik_aic(y, mu, w, res_dev, nobs, rank))
            if p.get("fix_dispersion_parameter"):
                self._disp = float(p.get("init_dispersion_parameter") or 1.0)
            elif getattr(self, "_tweedie_phi", None) is not None:
                self._disp = self._tweedie_phi
            else:
                self._disp = estimate_dispersion(family, y, mu, w, nobs, rank, res_dev,
                                                 p.get("dispersion_parameter_method") or "pearson",
                                                 int(p.get("max_iterations_dispersion") or 50),
                                                 float(p.get("dispersion_epsilon") or 1e-4))
            if family.name in ("gaussian", "gamma", "tweedie", "negativebinomial"):
                out["dispersion"] = self._disp
            if p.get("calc_like"):
                phi = self._disp if family.name != "negativebinomial" else 1.0
                ll = family.loglik(y, mu, w, phi)
                k = rank + (1 if family.name in ("gaussian", "gamma", "negativebinomial") else 0)
                out["loglikelihood"] = ll
                out["aic"] = -2 * ll + 2 * k
            if p["compute_p_values"]:
                self._p_values(model, family, Zi, y, w, off, beta[0], names, nobs, rank, ex)
            if p.get("influence"):
                self._influence(model, family, X, y, w, off, ex, nobs)
        else:
            probs = P.double()
            yl = y.long().clamp(min=0)
            res_dev = _gsum(-2 * (w * torch.log(probs.gather(1, yl[:, None])[:, 0].clamp(min=1e-15))).sum())
            freq = _gvec(segment_sum(yl, w, probs.shape[1]))
            freq = freq / freq.sum()
            null_dev = _gsum(-2 * (w * torch.log(freq[yl].clamp(min=1e-15))).sum())
            rank = int((beta.abs() > 0).sum())
            out.update(residual_deviance=res_dev, null_deviance=null_dev, aic=res_dev + 2 * rank,
                       null_degrees_of_freedom=nobs - 1, residual_degrees_of_freedom=nobs - rank)
        lab = model.predict_labels(P)
        tm = mm.make_metrics(cat, yv[ok], P[ok], w[ok].float(), model.info.response_domain,
                             labels=None if lab is None else lab[ok])
        if tm is not None:
            tm.update(null_deviance=out.get("null_deviance"), residual_deviance=out.get("residual_deviance"),
                      AIC=out.get("aic"))
            if cat == "Regression":
                tm["mean_residual_deviance"] = out["residual_deviance"] / max(_gsum(w.sum()), 1e-300)
        out["training_metrics"] = tm
        if tm is not None and "loglikelihood" in out:
            tm["loglikelihood"] = out["loglikelihood"]
        if p.get("generate_variable_inflation_factors"):
            out["variable_inflation_factors"] = variance_inflation_factors(ex, X, w)
        imp = [(n[: n.rfind("_")] if K > 1 else n, abs(v)) for n, v in coefs_std.items() if not n.startswith("Intercept")]
        agg = {}
        for n, v in imp:
            agg[n] = agg.get(n, 0.0) + v
        from .base import variable_importance
        out["variable_importances"] = variable_importance(list(agg.keys()), list(agg.values()))

    def _influence(self, model, family, X, y, w, off, ex, nobs):
        """Regression influence diagnostics (RegressionInfluenceDiagnosticsTasks): DFBETAS of every row and
        coefficient on the raw scale. Gaussian: (β - β₍ᵢ₎)ⱼ / (s₍ᵢ₎ √(XᵀX)⁻¹ⱼⱼ) with the leave-one-out β₍ᵢ₎ and
        s₍ᵢ₎ in closed form; binomial: rᵢwᵢ/(1 - hᵢ) · (G⁻¹xᵢ)ⱼ / seⱼ with G = XᵀWX, hᵢ = wᵢμᵢ(1-μᵢ)xᵢᵀG⁻¹xᵢ."""
        p = self.p
        if str(p["influence"]).lower() != "dfbetas":
            raise ValueError("influence must be 'dfbetas'")
        if family.name not in ("gaussian", "binomial") or float(p.get("lambda_") or 0.0) != 0.0:
            raise ValueError("influence='dfbetas' needs family gaussian or binomial and lambda = 0")
        if coll.is_dist():
            raise ValueError("influence diagnostics need a single-process frame")
        raw = Expander(ex.info, standardize=False, use_all_factor_levels=ex.use_all).fit(X, w)
        Xr = raw.transform(X).double()
        Xr = torch.cat([Xr, torch.ones(Xr.shape[0], 1, dtype=Xr.dtype, device=Xr.device)], 1)
        braw, ic = ex.destandardize(model.beta[0, :-1], float(model.beta[0, -1]))
        b = torch.cat([braw.double(), torch.tensor([ic], dtype=torch.float64, device=braw.device)])
        eta = Xr @ b + off
        mu = family.linkinv(eta)
        r = y.double() - mu
        wd = w.double()
        if family.name == "gaussian":
            G = (Xr * wd[:, None]).T @ Xr
            Gi = torch.linalg.pinv(G)
            XGi = Xr @ Gi
            h = wd * (XGi * Xr).sum(1)
            pdim = Xr.shape[1]
            s2 = float((wd * r * r).sum()) / max(nobs - pdim, 1)
            s2i = ((nobs - pdim) * s2 - wd * r * r / (1 - h).clamp(min=1e-12)) / max(nobs - pdim - 1, 1)
            dbeta = XGi * (wd * r / (1 - h).clamp(min=1e-12))[:, None]          # β - β₍ᵢ₎
            D = dbeta / (s2i.clamp(min=1e-300).sqrt()[:, None] * Gi.diagonal().clamp(min=1e-300).sqrt()[None, :])
        else:
            vw = wd * mu * (1 - mu)
            G = (Xr * vw[:, None]).T @ Xr
            Gi = torch.linalg.pinv(G)
            XGi = Xr @ Gi
            h = vw * (XGi * Xr).sum(1)
            se = Gi.diagonal().clamp(min=1e-300).sqrt()
            D = XGi * (r * wd / (1 - h).clamp(min=1e-12))[:, None] / se[None, :]
        D = torch.where((wd > 0)[:, None], D, torch.zeros_like(D))
        from ..frame import H2OFrame
        names = ["DFBETA_" + n for n in list(raw.names) + ["Intercept"]]
        fr = H2OFrame.from_tensor(D.float(), names)
        model.output["regression_influence_diagnostics"] = fr.frame_id
        model._rid = fr

    def _p_values(self, model, family, Zi, y, w, off, beta, names, nobs, rank, ex):
        lam = model.output.get("lambda_best", 0.0)
        if lam and lam > 0:
            model.output["warnings"] = ["p-values are only computed for lambda = 0"]
        eta = G.zbeta(Zi, beta, off)
        mu = family.linkinv(eta)
        gp = family.dlink(mu)
        var = family.variance(mu)
        wi = w / (var * gp * gp).clamp(min=1e-30)
        Gm = _gvec(G.gram(Zi, wi.float()))
        if family.name in ("binomial", "poisson", "quasibinomial", "fractionalbinomial"):
            disp = 1.0
        else:        # dispersion_parameter_method / fix_dispersion_parameter (estimated in _outputs)
            disp = getattr(self, "_disp", None)
            if disp is None:
                disp = _gsum((w * (y - mu) ** 2 / var.clamp(min=1e-30)).sum()) / max(nobs - rank, 1)
        cov = torch.linalg.pinv(Gm) * disp
        se_std = cov.diagonal().clamp(min=0).sqrt()
        # raw-scale standard errors: numeric coefficient j scales by 1/sd_j; intercept via the delta method
        P = beta.numel() - 1
        Tm = torch.eye(P + 1, dtype=torch.float64, device=beta.device)
        if ex.standardize and ex.nums:
            k = ex.num_off
            sd = ex.num_sd
            for i in range(len(ex.nums)):
                Tm[k + i, k + i] = 1.0 / float(sd[i])
                Tm[P, k + i] = -float(ex.num_mean[i]) / float(sd[i])
        cov_raw = Tm @ cov @ Tm.T
        se = cov_raw.diagonal().clamp(min=0).sqrt()
        braw, ic = ex.destandardize(beta[:-1], float(beta[-1]))
        bvec = torch.cat([braw, torch.tensor([ic], dtype=torch.float64, device=braw.device)])
        zval = bvec / se.clamp(min=1e-300)
        from scipy import stats
        use_t = family.name not in ("binomial", "poisson", "quasibinomial", "fractionalbinomial")
        zv = zval.cpu().numpy()
        pv = 2 * (stats.t.sf(np.abs(zv), max(nobs - rank, 1)) if use_t else stats.norm.sf(np.abs(zv)))
        model.output["std_errs"] = dict(zip(names, se.cpu().tolist()))
        model.output["z_values"] = dict(zip(names, zv.tolist()))
        model.output["p_values"] = dict(zip(names, pv.tolist()))
        model.output["dispersion"] = disp
        model.output["standardized_std_errs"] = dict(zip(names, se_std.cpu().tolist()))


def make_glm_model(model: GLMModel, coefs: dict) -> GLMModel:
    """``H2OGeneralizedLinearEstimator.makeGLMModel``: copy of ``model`` with user coefficients (raw scale)."""
    import copy
    m = copy.copy(model)
    m.output = dict(model.output)
    ex = model.expander
    P = len(ex.names)
    b = torch.zeros(1, P + 1, dtype=torch.float64)
    raw = torch.tensor([coefs.get(n, 0.0) for n in ex.names], dtype=torch.float64)
    ic = float(coefs.get("Intercept", 0.0))
    if ex.standardize and ex.nums:
        k = ex.num_off
        mu, sd = ex.num_mean.cpu(), ex.num_sd.cpu()
        std = raw.clone()
        std[k:] = raw[k:] * sd
        ic_std = ic + float((raw[k:] * mu).sum())
    else:
        std, ic_std = raw, ic
    b[0, :P] = std
    b[0, P] = ic_std
    m.beta = b.to(model.beta.device)
    m.output["coefficients"] = dict(coefs)
    return m
