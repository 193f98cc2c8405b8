"""Naive Bayes (reference: ``hex/naivebayes/NaiveBayes.java``, ``NaiveBayesModel.java``).

Sufficient statistics are per-class device reductions: class priors, per-class categorical level
counts (Laplace smoothing ``laplace``) and per-class Gaussian mean/sd of numerics (``min_sdev``,
``eps_sdev``, ``min_prob``, ``eps_prob`` thresholds as in H2O). Scoring sums log-likelihoods
on device and normalises with log-sum-exp.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from .. import metrics as mm
from ..parallel import collectives as coll
from .base import DataInfo, Model, make_key
from ..ops.segment import segment_sum

NB_DEFAULTS = dict(laplace=0.0, min_sdev=0.001, eps_sdev=0.0, min_prob=0.001, eps_prob=0.0, compute_metrics=True, seed=-1)


class NaiveBayesModel(Model):
    algo = "naivebayes"

    def _predict_tensor(self, X, offset=None):
        X = X.to(self.device)
        K = self.nclasses
        N = X.shape[1]
        ll = torch.log(torch.as_tensor(self.prior, dtype=torch.float64, device=X.device))[None, :].repeat(N, 1)
        p = self.params
        for j in range(self.info.F):
            x = X[j].double()
            na = torch.isnan(x)
            if self.info.iscat[j]:
                tab = torch.as_tensor(self.cond[j], dtype=torch.float64, device=X.device)   # [K, L]
                L = tab.shape[1]
                code = torch.nan_to_num(x, nan=0).long().clamp(0, max(L - 1, 0))
                pr = tab[:, code].T
                pr = torch.where(pr <= float(p["eps_prob"]), torch.full_like(pr, float(p["min_prob"])), pr)
                ll += torch.where(na[:, None], torch.zeros_like(pr), torch.log(pr))
            else:
                mu = torch.as_tensor(self.cond[j][0], dtype=torch.float64, device=X.device)
                sd = torch.as_tensor(self.cond[j][1], dtype=torch.float64, device=X.device)
                sd = torch.where(sd <= float(p["eps_sdev"]), torch.full_like(sd, float(p["min_sdev"])), sd)
                z = (x[:, None] - mu[None, :]) / sd[None, :]
                lp = -0.5 * z * z - torch.log(sd[None, :]) - 0.5 * math.log(2 * math.pi)
                ll += torch.where(na[:, None], torch.zeros_like(lp), lp)
        return torch.softmax(ll, 1).float()

    def to_state(self):
        s = super().to_state()
        s["prior"] = list(self.prior)
        s["cond"] = [np.asarray(c).tolist() for c in self.cond]
        return s

    def _restore(self, s):
        super()._restore(s)
        self.prior = s["prior"]
        self.cond = [np.asarray(c) for c in s["cond"]]


class NaiveBayesTrainer:
    def __init__(self, params):
        p = dict(NB_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        t0 = time.time()
        dev = X.device
        N = X.shape[1]
        K = len(info.response_domain)
        w = torch.ones(N, dtype=torch.float64, device=dev) if w is None else w.double()
        ok = ~torch.isnan(y)
        w = torch.where(ok, w, torch.zeros_like(w))
        yl = torch.nan_to_num(y, nan=0).long()
        red = coll.all_reduce_ if coll.is_dist() else (lambda t: t)
        cnt = red(segment_sum(yl, w, K))
        lap = float(self.p["laplace"])
        prior = (cnt + lap) / (cnt.sum() + K * lap)
        cond = []
        for j in range(info.F):
            x = X[j].double()
            na = torch.isnan(x)
            wj = torch.where(na, torch.zeros_like(w), w)
            if info.iscat[j]:
                L = len(info.domains[j])
                code = torch.nan_to_num(x, nan=0).long().clamp(0, max(L - 1, 0))
                tab = red(segment_sum(yl * L + code, wj, K * L)).view(K, L)
                tab = (tab + lap) / (tab.sum(1, keepdim=True) + L * lap).clamp(min=1e-300)
                cond.append(tab.cpu().numpy())
            else:
                xz = torch.where(na, torch.zeros_like(x), x)
                s0 = red(segment_sum(yl, wj, K))
                s1 = red(segment_sum(yl, wj * xz, K))
                s2 = red(segment_sum(yl, wj * xz * xz, K))
                mu = s1 / s0.clamp(min=1e-300)
                var = (s2 - s0 * mu * mu) / (s0 - 1).clamp(min=1e-300)
                cond.append(np.stack([mu.cpu().numpy(), var.clamp(min=0).sqrt().cpu().numpy()]))
        model = NaiveBayesModel(model_key or make_key("naivebayes"), self.p, info)
        model.device = dev
        model.prior = prior.cpu().tolist()
        model.cond = cond
        model.output["apriori"] = dict(zip(info.response_domain, model.prior))
        model.output["pcond"] = {info.x[j]: np.asarray(c).tolist() for j, c in enumerate(cond)}
        model.output["training_metrics"] = model.metrics_for(X, y, w.float())
        if valid is not None:
            Xv, yv, wv, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv, ov)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
