"""Cox Proportional Hazards (reference: ``hex/coxph/CoxPH.java``, ``CoxPHModel.java``).

Partial likelihood with Efron (default) or Breslow ties, counting-process ``start_column``,
``stratify_by``, weights and offset. The log partial likelihood is written as vectorised device
ops over rows sorted by stop time (risk-set sums are suffix cumsums picked at the end of each
unique-time group; Efron's l/d correction is a per-event-row term), so gradient and Hessian come
from autograd and Newton–Raphson with step halving runs to ``lre_min`` like the reference.
Outputs: coefficients, exp(coef), se, z, p, loglik, null loglik, LR/Wald/score tests, concordance;
``predict`` is the centered linear predictor (``lp``).
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from .base import DataInfo, Model, make_key
from .datainfo import Expander

COX_DEFAULTS = dict(start_column=None, stop_column=None, stratify_by=None, ties="efron", init=0.0, lre_min=9.0,
                    max_iterations=20, interactions=None, use_all_factor_levels=False, single_node_mode=False)


def _loglik_fn(Z, time_, event, w, off, start, strata, ties):
    """Return f(beta) = log partial likelihood (torch, differentiable)."""
    dev = Z.device
    groups = []
    for s in (torch.unique(strata) if strata is not None else [None]):
        idx = torch.arange(Z.shape[0], device=dev) if s is None else torch.nonzero(strata == s).flatten()
        t = time_[idx]
        order = torch.argsort(t, descending=True, stable=True)
        ridx = idx[order]
        ts = t[order]
        # unique-time groups over the descending order: group end = last index with that time
        uniq, inv, counts = torch.unique_consecutive(ts, return_inverse=True, return_counts=True)
        gend = torch.cumsum(counts, 0) - 1
        ev = event[ridx]
        d = torch.zeros(len(uniq), dtype=torch.float64, device=dev).index_add_(0, inv, ev)
        # position of each event row within its tie group (0..d-1)
        evc = torch.cumsum(ev, 0)
        gstart_ev = torch.cat([torch.zeros(1, dtype=torch.float64, device=dev), torch.cumsum(d, 0)[:-1]])
        lpos = (evc - ev) - gstart_ev[inv]
        entry = None
        if start is not None:
            st = start[ridx]
            st_order = torch.argsort(st, descending=True, stable=True)
            st_sorted = st[st_order]
            # number of rows (in descending-start order) with start >= each unique time
            n_ge = torch.searchsorted(-st_sorted.contiguous(), -uniq.contiguous(), right=True)
            entry = (ridx[st_order], n_ge)
        groups.append((ridx, inv, gend, ev, d, lpos, entry))

    def f(beta):
        total = 0.0
        for ridx, inv, gend, ev, d, lpos, entry in groups:
            eta = Z[ridx] @ beta + off[ridx]
            r = w[ridx] * torch.exp(eta)
            R = torch.cumsum(r, 0)[gend]
            if entry is not None:
                eidx, n_ge = entry
                re = w[eidx] * torch.exp(Z[eidx] @ beta + off[eidx])
                cre = torch.cat([torch.zeros(1, dtype=re.dtype, device=re.device), torch.cumsum(re, 0)])
                R = R - cre[n_ge]
            S0 = torch.zeros_like(R).index_add_(0, inv, r * ev)
            Rg = R[inv]
            if ties == "efron":
                frac = torch.where(d[inv] > 0, lpos / d[inv].clamp(min=1), torch.zeros_like(lpos))
                den = Rg - frac * S0[inv]
            else:
                den = Rg
            wi = w[ridx] * ev
            total = total + (wi * (eta - torch.log(den.clamp(min=1e-300)))).sum()
        return total
    return f


class CoxPHModel(Model):
    algo = "coxph"

    def __init__(self, key, params, info):
        super().__init__(key, params, info)
        self.output["model_category"] = "CoxPH"

    @property
    def model_category(self):
        return "CoxPH"

    def _predict_tensor(self, X, offset=None):
        keep = getattr(self, "keep", None)
        X = X.to(self.device)
        Z = self.expander.transform(X if keep is None else X[keep]).double()
        lp = Z @ self.beta.to(Z.device) - self._lp_base(X)
        if offset is not None:
            lp = lp + offset.double()
        return lp.float()

    def _lp_base(self, X):
        """Per-row centring term: the weighted mean linear predictor of the row's stratum
        (CoxPHModel.java:405 subtracts _lpBase[stratum]); rows of an unseen stratum get NaN."""
        bases = self.output.get("lp_base")
        sv = getattr(self, "strata_values", [])
        if not self.strata_idx or not bases or not sv:
            return float(self.output["lp_mean"])
        N = X.shape[1]
        out = torch.full((N,), float("nan"), dtype=torch.float64, device=X.device)
        S = X[self.strata_idx].double()
        for k, vals in enumerate(sv):
            m = torch.ones(N, dtype=torch.bool, device=X.device)
            for j, v in enumerate(vals):
                m &= S[j] == float(v)
            out = torch.where(m, torch.full_like(out, float(bases[k])), out)
        return out

    def prediction_names(self):
        return ["lp"]

    def coef(self):
        return self.output["coefficients"]

    def to_state(self):
        s = super().to_state()
        s["beta"] = self.beta.cpu().tolist()
        s["expander"] = self.expander.to_state()
        s["keep"] = getattr(self, "keep", None)
        s["strata_idx"] = getattr(self, "strata_idx", [])
        s["special_idx"] = getattr(self, "special_idx", [])
        s["strata_values"] = getattr(self, "strata_values", [])
        return s

    def _restore(self, s):
        super()._restore(s)
        self.beta = torch.tensor(s["beta"], dtype=torch.float64)
        self.keep = s.get("keep")
        self.strata_idx = s.get("strata_idx") or []
        self.special_idx = s.get("special_idx") or []
        self.strata_values = s.get("strata_values") or []
        sub = self.info if self.keep is None else DataInfo([self.info.x[j] for j in self.keep],
                                                          np.asarray(self.info.iscat)[self.keep],
                                                          [self.info.domains[j] for j in self.keep],
                                                          self.info.response, self.info.response_domain)
        self.expander = Expander.from_state(sub, s["expander"])


class CoxPHTrainer:
    def __init__(self, params):
        p = dict(COX_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        """``y`` is the event indicator column; ``stop_column`` (and ``start_column``) must be in ``info.x``."""
        t0 = time.time()
        p = self.p
        stop = p["stop_column"]
        if stop is None or stop not in info.x:
            raise ValueError("CoxPH needs stop_column among the frame columns")
        j_stop = info.x.index(stop)
        special = [j_stop]
        start = None
        if p["start_column"]:
            j_start = info.x.index(p["start_column"])
            special.append(j_start)
            start = X[j_start].double()
        strata = None
        strata_idx = []
        strata_values = []
        if p["stratify_by"]:
            sb = p["stratify_by"] if isinstance(p["stratify_by"], (list, tuple)) else [p["stratify_by"]]
            for c in sb:
                j = info.x.index(c)
                special.append(j)
                strata_idx.append(j)
            S = X[strata_idx].double()
            if bool(torch.isnan(S).any()):
                # genmodel's Strata key casts NaN to 0: an NA stratum could not be looked up by a MOJO scorer
                raise ValueError("stratify_by columns must not contain missing values")
            # stratum id = row of the unique (value tuple) table: no positional code collisions
            uniq, strata = torch.unique(S.T, dim=0, return_inverse=True)
            strata_values = uniq.cpu().tolist()
        keep = [j for j in range(info.F) if j not in special]
        sub = DataInfo([info.x[j] for j in keep], np.asarray(info.iscat)[keep], [info.domains[j] for j in keep],
                       info.response, info.response_domain)
        Xs = X[keep]
        N = X.shape[1]
        dev = X.device
        w = torch.ones(N, dtype=torch.float64, device=dev) if w is None else w.double()
        ev = y.double()
        if info.response_domain is not None:
            ev = (ev == len(info.response_domain) - 1).double()
        ok = ~torch.isnan(y) & ~torch.isnan(X[j_stop])
        w = torch.where(ok, w, torch.zeros_like(w))
        ex = Expander(sub, standardize=False, use_all_factor_levels=p["use_all_factor_levels"]).fit(Xs, w)
        Z = ex.transform(Xs).double()
        off = torch.zeros(N, dtype=torch.float64, device=dev) if offset is None else offset.double()
        ties = str(p["ties"]).lower()
        f = _loglik_fn(Z, torch.nan_to_num(X[j_stop].double()), torch.nan_to_num(ev), w, off, start, strata, ties)
        P = Z.shape[1]
        beta = torch.full((P,), float(p["init"]), dtype=torch.float64, device=dev)
        ll0 = float(f(torch.zeros(P, dtype=torch.float64, device=dev)))
        ll = float(f(beta))
        it = 0
        for it in range(int(p["max_iterations"])):
            g = torch.autograd.functional.jacobian(f, beta)
            H = torch.autograd.functional.hessian(f, beta)
            step = torch.linalg.solve(-H + 1e-12 * torch.eye(P, dtype=H.dtype, device=dev), g)
            t = 1.0
            while True:
                nb = beta + t * step
                nll = float(f(nb))
                if nll >= ll - 1e-12 or t < 1e-6:
                    break
                t /= 2
            lre = -math.log10(abs(nll - ll) / max(abs(nll), 1e-300)) if nll != ll else float("inf")
            beta, ll = nb, nll
            if lre >= float(p["lre_min"]):
                break
        H = torch.autograd.functional.hessian(f, beta)
        cov = torch.linalg.pinv(-H)
        se = cov.diagonal().clamp(min=0).sqrt()
        z = beta / se.clamp(min=1e-300)
        from scipy import stats
        pv = 2 * stats.norm.sf(np.abs(z.cpu().numpy()))
        g0 = torch.autograd.functional.jacobian(f, torch.zeros(P, dtype=torch.float64, device=dev))
        H0 = torch.autograd.functional.hessian(f, torch.zeros(P, dtype=torch.float64, device=dev))
        score = float(g0 @ torch.linalg.pinv(-H0) @ g0)
        model = CoxPHModel(model_key or make_key("coxph"), p, info)
        model.device = dev
        model.expander = ex
        model.beta = beta
        model.keep, model.strata_idx = keep, strata_idx
        model.special_idx = [j for j in special if j not in strata_idx]
        model.strata_values = strata_values
        lp = Z @ beta
        model.output["lp_mean"] = float((w * lp).sum() / w.sum())
        # weighted design means: the MOJO's x_mean_cat / x_mean_num (lp_mean = z_mean . beta)
        model.output["z_mean"] = ((w[:, None] * Z).sum(0) / w.sum()).cpu().tolist()
        if strata is not None:
            # one mean (and lp base) per stratum, in strata_values order (CoxPH.java:400-408)
            K = len(strata_values)
            ws = torch.zeros(K, dtype=torch.float64, device=dev).index_add_(0, strata, w)
            zs = torch.zeros(K, Z.shape[1], dtype=torch.float64, device=dev).index_add_(0, strata, w[:, None] * Z)
            zmean_s = zs / ws.clamp(min=1e-300)[:, None]
            model.output["z_mean_strata"] = zmean_s.cpu().tolist()
            model.output["lp_base"] = (zmean_s @ beta).cpu().tolist()
        names = ex.names
        model.output["coefficients"] = dict(zip(names, beta.cpu().tolist()))
        model.output["coefficients_table"] = [dict(names=n, coefficients=float(b), exp_coef=math.exp(float(b)),
                                                   se_coef=float(s), z_coef=float(zz), p_value=float(pp))
                                              for n, b, s, zz, pp in zip(names, beta.cpu(), se.cpu(), z.cpu(), pv)]
        wald = float(beta @ torch.linalg.pinv(cov) @ beta)
        model.output.update(loglik=ll, null_loglik=ll0, loglik_test=2 * (ll - ll0), wald_test=wald, score_test=score,
                            iterations=it + 1, n=int((w > 0).sum()), total_event=float((w * torch.nan_to_num(ev)).sum()),
                            ties=ties)
        model.output["concordance"] = _concordance(torch.nan_to_num(X[j_stop].double()), torch.nan_to_num(ev), lp, w)
        model.output["training_metrics"] = dict(model_category="CoxPH", concordance=model.output["concordance"],
                                                loglik=ll)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model


def _concordance(t, e, lp, w, max_n=4000):
    """Harrell's C on (a sample of) the training rows."""
    ok = w > 0
    t, e, lp = t[ok], e[ok], lp[ok]
    if t.numel() > max_n:
        idx = torch.randperm(t.numel(), generator=torch.Generator().manual_seed(0))[:max_n].to(t.device)
        t, e, lp = t[idx], e[idx], lp[idx]
    ti, tj = t[:, None], t[None, :]
    comp = (ti < tj) & (e[:, None] > 0)
    conc = comp & (lp[:, None] > lp[None, :])
    ties = comp & (lp[:, None] == lp[None, :])
    n = float(comp.sum())
    return float((conc.sum() + 0.5 * ties.sum()) / n) if n > 0 else float("nan")
