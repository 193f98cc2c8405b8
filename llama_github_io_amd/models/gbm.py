"""Gradient Boosting Machine (reference: ``hex/tree/gbm/GBM.java``, ``GBMModel.java``).

Per iteration: pseudo-residuals ``z = negHalfGradient(y, f)`` (``DistributionFactory``), one tree per
class grown by the device histogram engine on (w, w·z), leaf values by the distribution's Newton step
``gammaNum/gammaDenom`` (``GBM.fitBestConstants``; median/quantile leaves for laplace / quantile /
huber), scaled by ``learn_rate * learn_rate_annealing^t`` ((K-1)/K for multinomial) and clamped to
``max_abs_leafnode_pred``; then ``f += leaf value`` per row via the leaf id each row recorded.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import metrics as mm
from ..parallel import collectives as coll
from ..ops import tree as T
from .base import DataInfo
from ..parallel.order_stats import global_quantile
from .distributions import ORDER_STAT_DISTS, get_distribution
from .shared_tree import SharedTreeModel, SharedTreeTrainer
from ..ops.segment import segment_sum

_FUSED_DIST = {"gaussian": 0, "bernoulli": 1, "quasibinomial": 2, "poisson": 3, "gamma": 4, "tweedie": 5,
               "laplace": 6, "quantile": 7, "huber": 8, "modified_huber": 9}

# fused distributions whose gamma numerator is w * z (GBM.java gammaNum of DistributionFactory): plane 2 == plane 1
_NUM_IS_WZ = frozenset({"gaussian", "bernoulli", "quasibinomial", "laplace", "quantile", "huber"})

GBM_DEFAULTS = dict(ntrees=50, max_depth=5, min_rows=10.0, learn_rate=0.1, learn_rate_annealing=1.0,
                    sample_rate=1.0, col_sample_rate=1.0, col_sample_rate_change_per_level=1.0,
                    col_sample_rate_per_tree=1.0, distribution="AUTO", tweedie_power=1.5, quantile_alpha=0.5,
                    huber_alpha=0.9, max_abs_leafnode_pred=float("inf"), pred_noise_bandwidth=0.0)


def resolve_distribution(name, info: DataInfo) -> str:
    name = (name or "AUTO").lower()
    if name == "auto":
        if info.response_domain is None:
            return "gaussian"
        return "bernoulli" if len(info.response_domain) == 2 else "multinomial"
    # GBM.init: a categorical response needs a classification distribution and vice versa
    classif = name in ("bernoulli", "quasibinomial", "multinomial", "modified_huber", "custom")
    if info.response_domain is not None and not classif:
        raise ValueError(f"distribution {name!r} is not allowed for the categorical response {info.response!r}")
    if info.response_domain is None and classif and name != "custom":
        raise ValueError(f"distribution {name!r} needs a categorical response; {info.response!r} is numeric")
    return name


class GBMModel(SharedTreeModel):
    algo = "gbm"

    def _trees_per_iter(self):
        return self.forest.K if self.forest is not None else 1

    def _predict_tensor(self, X, offset=None):
        f = self.forest.predict_raw(X)
        init = torch.as_tensor(self.init_f, dtype=torch.float32, device=f.device)
        f = f + init
        if offset is not None:
            f = f + offset.float()[:, None]
        d = self.distribution
        if d.name == "multinomial":
            return torch.softmax(f, dim=1)
        if d.name in ("bernoulli", "quasibinomial", "modified_huber"):
            p1 = torch.sigmoid(f[:, 0])
            return torch.stack([1 - p1, p1], 1)
        if d.name == "custom" and self.model_category == "Binomial":
            p1 = d.linkinv(f[:, 0]).clamp(0, 1)
            return torch.stack([1 - p1, p1], 1)
        return d.linkinv(f[:, 0])

    @property
    def distribution(self):
        return get_distribution(self.output["distribution"], tweedie_power=self.params.get("tweedie_power", 1.5),
                                quantile_alpha=self.params.get("quantile_alpha", 0.5),
                                huber_alpha=self.params.get("huber_alpha", 0.9),
                                custom_distribution_func=self.params.get("custom_distribution_func"))

    def staged_predict_proba(self, X):
        out = []
        for n in range(1, self.ntrees_built() + 1):
            out.append(self._raw(X, ntrees=n))
        return out


class GBMTrainer(SharedTreeTrainer):
    algo = "gbm"
    mode = T.MODE_SE
    model_cls = GBMModel

    def __init__(self, params):
        p = dict(GBM_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None or k not in p})
        super().__init__(p)

    def _trees_per_iter(self):
        return self.K

    def _k_cols(self, F):
        r = float(self.p.get("col_sample_rate", 1.0))
        if r >= 1.0:
            return 0
        return max(1, int(math.floor(F * r + 0.5)))

    def fit(self, X, y, w, offset, info, valid=None, model_key=None):
        dname = resolve_distribution(self.p.get("distribution"), info)
        self.dist = get_distribution(dname, tweedie_power=self.p["tweedie_power"], quantile_alpha=self.p["quantile_alpha"],
                                     huber_alpha=self.p["huber_alpha"],
                                     custom_distribution_func=self.p.get("custom_distribution_func"))
        self.dname = dname
        self.K = len(info.response_domain) if dname == "multinomial" else 1
        return super().fit(X, y, w, offset, info, valid, model_key)

    def _init_model(self, model):
        N, K, dev = self.N, self.K, self.dev
        model.output["distribution"] = self.dname
        w = self.w
        if self.K > 1:
            self.yk = torch.nn.functional.one_hot(torch.nan_to_num(self.y, nan=0).long(), K).float()
            init = np.zeros(K)  # H2O multinomial starts from 0
        else:
            init = np.array([self.dist.init_f(self.y, w, self.offset, reduce=coll.all_reduce_scalar)])
            if self.dname in ORDER_STAT_DISTS:
                # order statistic of the GLOBAL response (exact refinement over the shards, no row gather)
                if self.dname == "quantile":
                    init = np.array([global_quantile(self.y, float(self.p["quantile_alpha"]))])
                else:
                    init = np.array([global_quantile(self.y, None)])
        self.init = init
        model.init_f = init.tolist()
        self.f = torch.tensor(init, dtype=torch.float32, device=dev).repeat(N, 1).contiguous()
        if self.offset is not None:
            self.f += self.offset[:, None]
        # fused path: the step kernel writes four SoA planes [4, N] (w, wY, gamma num, gamma den); the torch
        # path builds [N, 4] rows
        self.aux = (torch.empty(4, N, dtype=torch.float32, device=dev) if self._fused()
                    else torch.empty(N, 4, dtype=torch.float32, device=dev))

    def _aux_soa(self):
        return self._fused()

    def _unit_weights(self):
        # no user weights and no row sampling: every w is exactly 1, the histogram passes skip the w plane
        return (self._fused() and getattr(self, "_wbuf", None) is None and self.p.get("weights_column") is None
                and float(self.p["sample_rate"]) >= 1.0 and not getattr(self, "_y_has_nan", True))

    def _step_skip(self):
        # planes the fused step need not store: 0 (w) when every weight is 1 and nothing reads w (the order-statistic
        # leaves read it), 2 (gamma numerator) where it equals w * z (the leaf sums then read plane 1)
        sk = 1 if self._unit_weights() and self.dname not in ORDER_STAT_DISTS else 0
        return sk | (4 if self.dname in _NUM_IS_WZ else 0)

    def _num_plane(self):
        return 1 if self._fused() and self.dname in _NUM_IS_WZ else 2

    def _lr(self, t):
        return float(self.p["learn_rate"]) * float(self.p["learn_rate_annealing"]) ** t

    def _fused(self):
        return (self.dev.type == "cuda" and self.K == 1 and self.dname in _FUSED_DIST
                and not self.p.get("sample_rate_per_class") and not float(self.p.get("pred_noise_bandwidth") or 0))

    def _prepare(self, t, k):
        d = self.dist
        f = self.f[:, k]
        if k == 0 and self.dname == "huber":
            self._flush_pending()
            self.dist.huber_delta = global_quantile((self.y - f).abs(), float(self.p["huber_alpha"]))
        if self._fused():
            # one HIP pass: previous tree's f update + sampling + residuals + leaf terms + scale maxima
            from ..ops import _native as nat
            if not hasattr(self, "_amax"):
                self._amax = torch.zeros(4 * T.AMAX_SHARDS, dtype=torch.int32, device=self.dev)
                self._wbuf = None if self.w is None or bool((self.w == 1).all()) else self.w.contiguous()
                self._y_has_nan = bool(torch.isnan(self.y).any())
            pv, pl = self._pending if getattr(self, "_pending", None) is not None else (None, None)
            p1 = {"tweedie": self.p["tweedie_power"], "quantile": self.p["quantile_alpha"],
                  "huber": getattr(self.dist, "huber_delta", 1.0)}.get(self.dname, 0.0)
            nat.call("h2o_gbm_step", self.N, self.row0, _FUSED_DIST[self.dname], self.y.data_ptr(),
                     0 if self._wbuf is None else self._wbuf.data_ptr(), self.f.data_ptr(),
                     0 if pv is None else pv.data_ptr(), 0 if pl is None else pl.data_ptr(),
                     float(self.p["sample_rate"]), (self.seed * 0x9E3779B1 + t * 7919) & ((1 << 64) - 1),
                     float(p1), self.aux.data_ptr(), self._amax.data_ptr(), self._step_skip(), nat.stream_ptr(self.dev))
            self._pending = None
            self.w_eff = None
            return self.aux
        if k == 0:
            self.w_eff = self._row_sample(float(self.p["sample_rate"]), t)
            if self.K > 1:
                self.probs = torch.softmax(self.f, dim=1)
        w = self.w_eff
        if self.K > 1:
            y = self.yk[:, k]
            z = y - self.probs[:, k]
        else:
            y = self.y
            z = d.neg_half_gradient(y, f)
        a = self.aux
        a[:, 0] = w
        a[:, 1] = w * z
        a[:, 2] = d.gamma_num(w, y, z, f)
        a[:, 3] = d.gamma_denom(w, y, z, f)
        self._z = z
        return a

    def _leaf_native(self, t, k):
        """Closed-form Newton leaves in one HIP launch (k_leaf_values) for the fused single-output path."""
        if not self._fused() or self.dname in ORDER_STAT_DISTS:
            return None
        self._vals = self.builder.leaf_values_view()
        return (int(self.dname in ("poisson", "gamma", "tweedie")), self._lr(t), 0.0,
                float(self.p.get("max_abs_leafnode_pred", float("inf"))))

    def _amax_for_build(self):
        return self._amax if self._fused() else None

    def _hist_packed(self):
        # fused path with no user weights: aux.x = 1 or a 0/1 sample mask
        return self._fused() and getattr(self, "_wbuf", None) is None and self.p.get("weights_column") is None

    def _flush_pending(self):
        pend = getattr(self, "_pending", None)
        if pend is not None:
            from ..ops import _native as nat
            vals, leaf = pend
            nat.call("h2o_add_leaf", self.N, self.f.data_ptr(), 1, vals.data_ptr(), leaf.data_ptr(), nat.stream_ptr(self.dev))
            self._pending = None

    def _leaf_values(self, ls, t, k):
        d = self.dist
        m1 = (self.K - 1) / self.K if self.K > 1 else 1.0
        if self.dname in ORDER_STAT_DISTS:
            g = self._order_stat_leaves(ls.shape[0], k)
        else:
            g = d.leaf_gamma(ls[:, 0], ls[:, 1])
        gf = self._lr(t) * m1 * g
        if self.K > 1:
            gf = gf.clamp(-1e4, 1e4)
        gf = torch.nan_to_num(gf, nan=0.0, posinf=1e4, neginf=-1e4)
        mx = float(self.p.get("max_abs_leafnode_pred", float("inf")))
        if mx < float("inf"):
            gf = gf.clamp(-mx, mx)
        self._vals = gf.float()
        return self._vals

    def _order_stat_leaves(self, L, k):
        """Weighted per-leaf median (laplace) / alpha-quantile (quantile) / huber leaf of y - f."""
        self._flush_pending()
        leaf = self.builder.leaf_of_row.long()
        diff = (self.y - self.f[:, k]).double()
        a0 = self.aux[0] if self.aux.shape[0] == 4 and self.aux.shape[1] == self.N else self.aux[:, 0]
        w = (a0 if self.w_eff is None else self.w_eff).double()
        alpha = self.p["quantile_alpha"] if self.dname == "quantile" else 0.5
        if coll.is_dist():
            # per-leaf weighted order statistics over every shard's rows of the leaf (leaf ids are global:
            # every rank built the same tree): grouped histogram refinement, no row gather
            from ..parallel.order_stats import group_order_statistics
            tot = segment_sum(leaf, w, L)
            tot = coll.all_reduce_(tot.to(coll.comm_device())).to(tot.device)
            qv = group_order_statistics(diff, leaf, L, [alpha * float(t) for t in tot.cpu()], w)
            q = torch.tensor([0.0 if x != x else x for x in qv], dtype=torch.float64, device=diff.device)
            if self.dname == "huber":
                delta = self.dist.huber_delta
                r = diff - q[leaf]
                c = torch.sign(r) * torch.clamp(r.abs(), max=delta)
                s = segment_sum(leaf, w * c, L)
                s = coll.all_reduce_(s.to(coll.comm_device())).to(s.device)
                q = q + s / tot.clamp(min=1e-300)
            return q
        order = torch.argsort(diff)
        leaf_s = leaf[order]
        order2 = torch.argsort(leaf_s, stable=True)
        idx = order[order2]
        ls, ds, ws = leaf[idx], diff[idx], w[idx]
        tot = segment_sum(ls, ws, L)
        cw = torch.cumsum(ws, 0)
        start = torch.cumsum(tot, 0) - tot
        within = cw - start[ls]
        target = alpha * tot[ls]
        hit = (within >= target) & (ws > 0)
        big = torch.iinfo(torch.long).max
        pos = torch.where(hit, torch.arange(ls.numel(), device=ds.device), torch.full_like(ls, big))
        first = torch.full((L,), big, dtype=torch.long, device=ds.device).scatter_reduce_(0, ls, pos, reduce="amin")
        q = torch.where(first < big, ds[first.clamp(max=ls.numel() - 1)], torch.zeros(L, dtype=torch.float64, device=ds.device))
        if self.dname == "huber":
            delta = self.dist.huber_delta
            r = diff - q[leaf]
            c = torch.sign(r) * torch.clamp(r.abs(), max=delta)
            s = segment_sum(leaf, w * c, L)
            q = q + s / tot.clamp(min=1e-300)
        return q

    def _update(self, t, k):
        leaf = self.builder.leaf_of_row
        if self._fused():
            self._pending = (self._vals, leaf)   # applied by the next fused step (or _flush_pending)
            return
        vals = self._vals
        bw = float(self.p.get("pred_noise_bandwidth") or 0.0)
        if bw:
            # GBM.java pred_noise_bandwidth: the TRAINING margin gets each leaf's value times a factor
            # 1 + N(0, bw) drawn per (tree, class, leaf); the stored tree keeps the clean values
            if bw < 0:
                raise ValueError("pred_noise_bandwidth must be >= 0")
            g = torch.Generator(device="cpu").manual_seed(((0xDECAF + self.seed) * (0xFAAAAAAB + k * 1000 + t)) & 0x7FFFFFFF)
            noise = 1.0 + bw * torch.randn(vals.numel(), generator=g, dtype=torch.float64)
            vals = (vals.double() * noise.to(vals.device)).float()
        self.f[:, k] += vals[leaf.long()]

    def _finish(self, model, built):
        self._flush_pending()

    def _training_metrics(self, model):
        self._flush_pending()
        f = self.f
        y, w = self.y, self.w
        if self.K > 1:
            return mm.multinomial_metrics(y, torch.softmax(f, 1), w, self.info.response_domain)
        if self.dname in ("bernoulli", "quasibinomial", "modified_huber"):
            return mm.binomial_metrics(y, torch.sigmoid(f[:, 0]), w, self.info.response_domain)
        return mm.regression_metrics(y, self.dist.linkinv(f[:, 0]), w, self.dist)
