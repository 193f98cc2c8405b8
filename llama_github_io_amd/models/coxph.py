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
import torch.distributed as dist

from ..parallel import collectives as coll
from ..parallel.order_stats import order_statistics
from .base import DataInfo, Model, make_key
from .datainfo import Expander

COX_DEFAULTS = dict(start_column=None, stop_column=None, stratify_by=None, ties="efron", init=0.0, lre_min=9.0,
                    max_iterations=20, interactions=None, use_all_factor_levels=False, single_node_mode=False)


def _red(t: torch.Tensor, op=None) -> torch.Tensor:
    """All-reduce over the row shards (no-op in one process): CoxPHTask's reduce."""
    if not coll.is_dist():
        return t
    return coll.all_reduce_(t.contiguous().to(coll.comm_device()), op).to(t.device)


def _rev_cumsum(a: torch.Tensor, K: int) -> torch.Tensor:
    """Suffix sums along the time axis of a [K*T, ...] per-stratum bucket array."""
    sh = a.shape
    b = a.reshape(K, -1, *sh[1:])
    return b.flip(1).cumsum(1).flip(1).reshape(sh)


class _CoxStats:
    """Per-(stratum, event time) sufficient statistics of the partial likelihood (reference
    ``hex/coxph/CoxPH.java`` CoxPHTask: sizeEvents, countEvents, sumRiskEvents, sumXRiskEvents,
    sumLogRiskEvents, rcumsumRisk, rcumsumXRisk; ``EfronMethod.java`` for the tie terms).

    Buckets are the distinct EVENT times per stratum (risk sets are only read there); a row is in the
    risk set of time t_k when start < t_k <= stop, i.e. for buckets (eb, sb] with sb / eb = index of the
    last event time <= stop / start. Each rank sums its rows into the buckets and one all-reduce gives the
    global statistics; suffix sums along the time axis give the risk sets. The Hessian's second-moment
    risk sums (rcumsumXXRisk, T x P x P in the reference) are never formed: sum_t A_t R2_t equals
    Z' diag(r_i (PA[sb_i] - PA[eb_i])) Z with PA the prefix sums of A, a P x P reduction of the rows."""

    def __init__(self, Z, off, w, ev, stop, start, strata, K, times, ties):
        self.Z, self.off, self.K, self.ties = Z, off, K, ties
        T = len(times)
        self.T, self.G = T, K * T
        dev = Z.device
        tt = torch.as_tensor(times, dtype=torch.float64, device=dev)
        base = 0 if strata is None else strata * T
        sb = torch.searchsorted(tt, stop.contiguous(), right=True) - 1
        self.at_risk = (w > 0) & (sb >= 0)
        self.sb = torch.where(self.at_risk, sb + base, torch.zeros_like(sb))
        if start is not None:
            eb = torch.searchsorted(tt, start.contiguous(), right=True) - 1
            self.has_eb = self.at_risk & (eb >= 0)
            self.eb = torch.where(self.has_eb, eb + base, torch.zeros_like(eb))
        else:
            self.has_eb = None
        self.evm = self.at_risk & (ev > 0)
        self.w = torch.where(self.at_risk, w, torch.zeros_like(w))
        self.P = Z.shape[1]
        # event weight / count per bucket do not depend on beta
        D = torch.zeros(self.G, dtype=torch.float64, device=dev).index_add_(0, self.sb[self.evm], self.w[self.evm])
        c = torch.zeros(self.G, dtype=torch.float64, device=dev).index_add_(
            0, self.sb[self.evm], torch.ones_like(self.w[self.evm]))
        wz = torch.zeros(self.G, self.P, dtype=torch.float64, device=dev).index_add_(
            0, self.sb[self.evm], self.w[self.evm, None] * Z[self.evm])
        dc = _red(torch.cat([D[:, None], c[:, None], wz], 1))
        self.D, self.c, self.E1 = dc[:, 0], dc[:, 1], dc[:, 2:].sum(0)
        self.ev_bucket = torch.nonzero(self.c > 0).flatten()
        cc = self.c[self.ev_bucket].long()
        # one Efron term per tied event: bucket index and fraction e / c_t (Breslow: fraction 0)
        self.eidx = torch.repeat_interleave(self.ev_bucket, cc)
        first = torch.cumsum(cc, 0) - cc
        pos = torch.arange(int(cc.sum()), device=dev) - torch.repeat_interleave(first, cc)
        self.frac = (pos.double() / self.c[self.eidx]) if ties == "efron" else torch.zeros(len(pos), dtype=torch.float64,
                                                                                             device=dev)
        self.avg = self.D[self.eidx] / self.c[self.eidx]

    def _risk(self, beta, moments):
        """Global (R0, S0, L[, R1, S1]) at ``beta``; the exponent is shifted by the global max eta (the
        likelihood and its derivatives are invariant to it)."""
        eta = self.Z @ beta + self.off
        mx = eta[self.at_risk].max().reshape(1) if bool(self.at_risk.any()) \
            else torch.full((1,), -1e300, dtype=torch.float64, device=eta.device)
        m = float(_red(mx, dist.ReduceOp.MAX))
        r = torch.where(self.at_risk, self.w * torch.exp(eta - m), torch.zeros_like(eta))
        cols = [r[:, None]] + ([r[:, None] * self.Z] if moments else [])
        V = torch.cat(cols, 1)
        G, dev = self.G, eta.device
        h = torch.zeros(3 * G, V.shape[1], dtype=torch.float64, device=dev)
        h.index_add_(0, self.sb[self.at_risk], V[self.at_risk])
        if self.has_eb is not None:
            h.index_add_(0, self.eb[self.has_eb] + G, V[self.has_eb])
        h.index_add_(0, self.sb[self.evm] + 2 * G, V[self.evm])
        L = (self.w[self.evm] * (eta[self.evm] - m)).sum().reshape(1, 1).expand(1, V.shape[1])
        h = _red(torch.cat([h, L]))
        R = _rev_cumsum(h[:G], self.K) - _rev_cumsum(h[G:2 * G], self.K)
        S = h[2 * G:3 * G]
        return eta, r, m, R, S, float(h[3 * G, 0])

    def loglik(self, beta):
        _, _, _, R, S, L = self._risk(beta, False)
        term = R[self.eidx, 0] - self.frac * S[self.eidx, 0]
        return L - float((self.avg * torch.log(term.clamp(min=1e-300))).sum())

    def derivatives(self, beta):
        """(loglik, gradient, Hessian) at ``beta``."""
        eta, r, m, R, S, L = self._risk(beta, True)
        e, f, a = self.eidx, self.frac, self.avg
        term = (R[e, 0] - f * S[e, 0]).clamp(min=1e-300)
        ll = L - float((a * torch.log(term)).sum())
        d1 = R[e, 1:] - f[:, None] * S[e, 1:]
        grad = self.E1 - (a[:, None] * d1 / term[:, None]).sum(0)
        G, dev = self.G, eta.device
        A = torch.zeros(G, dtype=torch.float64, device=dev).index_add_(0, e, a / term)
        B = torch.zeros(G, dtype=torch.float64, device=dev).index_add_(0, e, a * f / term)
        PA = A.reshape(self.K, -1).cumsum(1).reshape(-1)
        v = torch.where(self.at_risk, r * PA[self.sb], torch.zeros_like(r))
        if self.has_eb is not None:
            v = v - torch.where(self.has_eb, r * PA[self.eb], torch.zeros_like(r))
        v = v - torch.where(self.evm, r * B[self.sb], torch.zeros_like(r))
        H1 = _red((self.Z * v[:, None]).T @ self.Z)
        u = (a / term ** 2)[:, None] * d1
        H2 = d1.T @ u
        return ll, grad, -(H1 - H2)


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
            # stratum id = row of the unique (value tuple) table, merged over the ranks (a few tuples)
            uniq = torch.unique(S.T, dim=0)
            if coll.is_dist():
                parts = coll.all_gather_object(uniq.cpu().tolist())
                uniq = torch.unique(torch.tensor([r for p_ in parts for r in p_], dtype=torch.float64).reshape(
                    -1, len(strata_idx)), dim=0).to(S.device)
            strata_values = uniq.cpu().tolist()
            strata = torch.zeros(S.shape[1], dtype=torch.long, device=S.device)
            for k in range(uniq.shape[0]):
                strata = torch.where((S.T == uniq[k]).all(1), torch.full_like(strata, k), strata)
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
        ex = Expander(sub, standardize=False, use_all_factor_levels=p["use_all_factor_levels"]).fit(
            Xs, w, reduce=coll.all_reduce_ if coll.is_dist() else None)
        Z = ex.transform(Xs).double()
        off = torch.zeros(N, dtype=torch.float64, device=dev) if offset is None else offset.double()
        ties = str(p["ties"]).lower()
        stop_t, evn = torch.nan_to_num(X[j_stop].double()), torch.nan_to_num(ev)
        K = max(len(strata_values), 1)
        # the time axis: distinct event times over all ranks (one entry per time of the model's baseline
        # hazard table, as the reference's CollectDoubleDomain over the time column)
        tev = torch.unique(stop_t[(w > 0) & (evn > 0)])
        if coll.is_dist():
            tev = torch.unique(coll.all_gather_cat(tev.to(coll.comm_device()), bounded=True)).to(dev)
        cs = _CoxStats(Z, off, w, evn, stop_t, start, strata, K, tev, ties)
        P = Z.shape[1]
        beta = torch.full((P,), float(p["init"]), dtype=torch.float64, device=dev)
        ll0, g0, H0 = cs.derivatives(torch.zeros(P, dtype=torch.float64, device=dev))
        ll, g, H = cs.derivatives(beta) if float(p["init"]) != 0 else (ll0, g0, H0)
        it = 0
        for it in range(int(p["max_iterations"])):
            step = torch.linalg.solve(-H + 1e-12 * torch.eye(P, dtype=H.dtype, device=dev), g)
            t = 1.0
            while True:
                nb = beta + t * step
                nll = cs.loglik(nb)
                if nll >= ll - 1e-12 or t < 1e-6:
                    break
                t /= 2
            lre = -math.log10(abs(nll - ll) / max(abs(nll), 1e-300)) if nll != ll else float("inf")
            beta = nb
            ll, g, H = cs.derivatives(beta)
            if lre >= float(p["lre_min"]):
                break
        cov = torch.linalg.pinv(-H)
        se = cov.diagonal().clamp(min=0).sqrt()
        z = beta / se.clamp(min=1e-300)
        from scipy import stats
        pv = 2 * stats.norm.sf(np.abs(z.cpu().numpy()))
        score = float(g0 @ torch.linalg.pinv(-H0) @ g0)
        model = CoxPHModel(model_key or make_key("coxph"), p, info)
        model.device = dev
        model.expander = ex
        model.beta = beta
        model.keep, model.strata_idx = keep, strata_idx
        model.special_idx = [j for j in special if j not in strata_idx]
        model.strata_values = strata_values
        lp = Z @ beta
        # weighted design means: the MOJO's x_mean_cat / x_mean_num (lp_mean = z_mean . beta)
        sums = _red(torch.cat([(w[:, None] * Z).sum(0), torch.stack([w.sum(), (w > 0).double().sum(),
                                                                    (w * evn).sum()])]))
        zmean, wsum = sums[:P] / sums[P], sums[P]
        model.output["lp_mean"] = float(zmean @ beta)
        model.output["z_mean"] = zmean.cpu().tolist()
        if strata is not None:
            # one mean (and lp base) per stratum, in strata_values order (CoxPH.java:400-408)
            zs = torch.zeros(K, P + 1, dtype=torch.float64, device=dev).index_add_(
                0, strata, torch.cat([w[:, None] * Z, w[:, None]], 1))
            zs = _red(zs)
            zmean_s = zs[:, :P] / zs[:, P].clamp(min=1e-300)[:, None]
            model.output["z_mean_strata"] = zmean_s.cpu().tolist()
            model.output["lp_base"] = (zmean_s @ beta).cpu().tolist()
        names = ex.names
        model.output["coefficients"] = dict(zip(names, beta.cpu().tolist()))
        model.output["coefficients_table"] = [dict(names=n, coefficients=float(b), exp_coef=math.exp(float(b)),
                                                   se_coef=float(s), z_coef=float(zz), p_value=float(pp))
                                              for n, b, s, zz, pp in zip(names, beta.cpu(), se.cpu(), z.cpu(), pv)]
        wald = float(beta @ torch.linalg.pinv(cov) @ beta)
        model.output.update(loglik=ll, null_loglik=ll0, loglik_test=2 * (ll - ll0), wald_test=wald, score_test=score,
                            iterations=it + 1, n=int(sums[P + 1]), total_event=float(sums[P + 2]), ties=ties)
        dur = stop_t - start if start is not None else stop_t
        st = concordance_stats(dur[ok], evn[ok], lp[ok], strata[ok] if strata is not None else None, K)
        model.output["concordance"] = st["concordance"]
        model.output["training_metrics"] = dict(model_category="CoxPH", loglik=ll, **st)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model


def _pair_counts(d, e, lp):
    """Exact Harrell pair counts (comparable, concordant, tied) of one stratum's rows, O(n log^2 n):
    (i, j) is comparable when i had the event and d_i < d_j, or d_i == d_j with j censored; concordant
    when lp_i > lp_j (higher risk failed first), tied when lp_i == lp_j. Rows in (d asc, dead first, lp
    desc) order; a bottom-up merge counts, for every row, the dead rows before it with higher / equal
    lp rank; dead rows tied on d are not comparable and are taken back out."""
    n = len(d)
    if n < 2:
        return 0, 0, 0
    o = np.lexsort((-lp, -e, d))
    d, e, lp = d[o], e[o], lp[o]
    _, r = np.unique(lp, return_inverse=True)
    r = r.astype(np.int64)
    R1 = int(r.max()) + 2
    dead = e > 0
    pos = np.arange(n, dtype=np.int64)
    pairs = conc = tied = 0
    s = 1
    while s < n:
        blk = pos // s
        lm = (blk % 2 == 0) & dead
        ks = np.sort(blk[lm] * R1 + r[lm])
        qm = blk % 2 == 1
        base = (blk[qm] - 1) * R1
        lo = np.searchsorted(ks, base, "left")
        tot = np.searchsorted(ks, base + R1, "left") - lo
        le = np.searchsorted(ks, base + r[qm], "right") - lo
        lt = np.searchsorted(ks, base + r[qm], "left") - lo
        pairs += int(tot.sum()); conc += int((tot - le).sum()); tied += int((le - lt).sum())
        s *= 2
    # dead rows tied on d: every earlier-later pair inside a group was counted (lp desc -> lp_i >= lp_j)
    if dead.any():
        dd, ll = d[dead], r[dead]
        _, g = np.unique(dd, return_counts=True)
        _, m = np.unique(np.stack([dd, ll.astype(np.float64)], 1), axis=0, return_counts=True)
        gp, mp = int((g * (g - 1) // 2).sum()), int((m * (m - 1) // 2).sum())
        pairs -= gp; tied -= mp; conc -= gp - mp
    return pairs, conc, tied


LATTICE = 1 << 16


def concordance_stats(d, e, lp, strata=None, K=1) -> dict:
    """Harrell's concordance of the risk scores on (duration, event) per stratum (reference
    ``hex/ModelMetricsRegressionCoxPH.java`` concordanceStats: all rows, unweighted, pairs within a stratum).

    One process: exact. Row-sharded: rows move once to the rank owning their duration range (exact
    order-statistic splitters; equal durations never split), pairs inside a range are counted exactly,
    and pairs across ranges — d_i < d_j by construction — from the earlier ranges' event-row histograms on
    a 2^16-cell lattice of the scores (all-reduced), as the mergeable AUC does: a cross-range pair whose two
    scores share a cell counts as tied."""
    dev = d.device
    pairs = conc = tied = 0
    for k in range(K):
        msk = torch.ones_like(d, dtype=torch.bool) if strata is None else strata == k
        dk, ek, lk = d[msk], e[msk], lp[msk]
        if coll.is_dist():
            W = coll.world()
            n = int(_red(torch.tensor([float(dk.numel())], dtype=torch.float64)).item())
            spl = order_statistics(dk, [j * n // W + 1 for j in range(1, W)]) if n else []
            spl = torch.tensor(spl, dtype=torch.float64, device=dev)
            dest = torch.searchsorted(spl, dk.contiguous(), right=True) if len(spl) else torch.zeros_like(
                dk, dtype=torch.long)
            got = coll.exchange_rows(torch.stack([dk, ek, lk], 1), dest)
            dk, ek, lk = got[:, 0], got[:, 1], got[:, 2]
            lo_hi = _red(torch.stack([lk.min() if lk.numel() else torch.tensor(float("inf"), dtype=torch.float64),
                                      -lk.max() if lk.numel() else torch.tensor(float("inf"), dtype=torch.float64)]
                                     ).reshape(2).cpu(), dist.ReduceOp.MIN)
            lo, hi = float(lo_hi[0]), -float(lo_hi[1])
            span = hi - lo if hi > lo else 1.0
            q = ((lk - lo) / span * (LATTICE - 1)).floor().long().clamp(0, LATTICE - 1).cpu()
            H = torch.zeros(W, LATTICE, dtype=torch.float64)
            H[coll.rank()] = torch.bincount(q[ek.cpu() > 0], minlength=LATTICE).double()
            H = _red(H)
            Hb = H[:coll.rank()].sum(0)
            above = Hb.flip(0).cumsum(0).flip(0)          # dead with cell >= c
            tot = float(Hb.sum())
            pairs += tot * q.numel()
            abv = torch.cat([above[1:], torch.zeros(1, dtype=torch.float64)])
            conc += float(abv[q].sum())
            tied += float(Hb[q].sum())
        pc = _pair_counts(dk.cpu().numpy(), ek.cpu().numpy(), lk.cpu().numpy())
        pairs, conc, tied = pairs + pc[0], conc + pc[1], tied + pc[2]
    if coll.is_dist():
        pairs, conc, tied = (float(v) for v in _red(torch.tensor([pairs, conc, tied], dtype=torch.float64)))
    pairs, conc, tied = int(pairs), int(conc), int(tied)
    return dict(concordance=(conc + 0.5 * tied) / pairs if pairs else float("nan"), concordant=conc,
                discordant=pairs - conc - tied, tied_y=tied)
