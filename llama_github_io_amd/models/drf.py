"""Distributed Random Forest and Extremely Randomized Trees (reference: ``hex/tree/drf/DRF.java``,
``DRFModel.java``; ``histogram_type='Random'`` = XRT: random split points per histogram,
``DHistogram.makeRandomSplitPoints``).

Per iteration one tree per class (one tree for binomial/regression, ``binomial_double_trees`` builds
two), each grown on the device engine with squared-error splits of the class indicator over a
row sample (``sample_rate`` 0.632 without replacement) and ``mtries`` columns re-drawn at every
node (``k_cols`` of the split reducer). Leaves store the weighted mean of the target; a forest
predicts the average over trees (class probabilities renormalised). Training metrics are
out-of-bag, as in H2O: each tree adds its leaf values to the rows it did not sample.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import metrics as mm
from ..ops import tree as T
from .shared_tree import SharedTreeModel, SharedTreeTrainer

DRF_DEFAULTS = dict(ntrees=50, max_depth=20, min_rows=1.0, mtries=-1, sample_rate=0.632, nbins=20,
                    binomial_double_trees=False, col_sample_rate_per_tree=1.0, min_split_improvement=1e-5,
                    histogram_type="AUTO", distribution="AUTO")


class DRFModel(SharedTreeModel):
    algo = "drf"

    def _trees_per_iter(self):
        return self.output.get("trees_per_iter", 1)

    def _predict_tensor(self, X, offset=None):
        s = self.forest.predict_raw(X)
        n = max(1, self.ntrees_built())
        cat = self.model_category
        if cat == "Regression":
            return s[:, 0] / n
        if cat == "Binomial":
            if self.output.get("double_trees"):
                p = s / n
                p = p / p.sum(1, keepdim=True).clamp(min=1e-30)
                return p
            p1 = (s[:, 0] / n).clamp(0, 1)
            return torch.stack([1 - p1, p1], 1)
        p = s.clamp(min=0)
        tot = p.sum(1, keepdim=True)
        return torch.where(tot > 0, p / tot.clamp(min=1e-30), torch.full_like(p, 1.0 / p.shape[1]))


class DRFTrainer(SharedTreeTrainer):
    algo = "drf"
    mode = T.MODE_SE
    model_cls = DRFModel

    def __init__(self, params):
        p = dict(DRF_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None or k not in p})
        super().__init__(p)

    def fit(self, X, y, w, offset, info, valid=None, model_key=None):
        self.nclass = len(info.response_domain) if info.response_domain else 1
        self.double = self.nclass == 2 and bool(self.p.get("binomial_double_trees"))
        self.K = self.nclass if (self.nclass > 2 or self.double) else 1
        return super().fit(X, y, w, offset, info, valid, model_key)

    def _trees_per_iter(self):
        return self.K

    def _hist_packed(self):
        return self.p.get("weights_column") is None and bool(((self.w == 0) | (self.w == 1)).all())

    def _k_cols(self, F):
        m = int(self.p.get("mtries", -1))
        if m == -2:
            return 0
        if m <= 0:
            m = max(1, int(math.sqrt(F))) if self.nclass > 1 else max(1, F // 3)
        return 0 if m >= F else m

    def _init_model(self, model):
        N, dev = self.N, self.dev
        model.output["trees_per_iter"] = self.K
        model.output["double_trees"] = self.double
        if self.nclass > 1:
            yl = torch.nan_to_num(self.y, nan=-1).long()
            self.yk = torch.zeros(N, self.K, device=dev)
            if self.K == 1:
                self.yk[:, 0] = (yl == 1).float()
            else:
                ok = yl >= 0
                self.yk[ok, yl[ok]] = 1.0
        else:
            self.yk = self.y[:, None]
        self.yok = ~torch.isnan(self.y)
        self.oob = torch.zeros(N, self.K, dtype=torch.float64, device=dev)
        self.oob_n = torch.zeros(N, dtype=torch.float64, device=dev)
        self.aux = torch.empty(N, 4, dtype=torch.float32, device=dev)

    def _prepare(self, t, k):
        if k == 0:
            ws = self._row_sample(float(self.p["sample_rate"]), t)
            self.ws = torch.where(self.yok, ws, torch.zeros_like(ws))
            self.inbag = self.ws > 0
        yk = torch.nan_to_num(self.yk[:, k], nan=0.0)
        a = self.aux
        a[:, 0] = self.ws
        a[:, 1] = self.ws * yk
        a[:, 2] = self.ws * yk
        a[:, 3] = self.ws
        return a

    def _leaf_values(self, ls, t, k):
        v = torch.where(ls[:, 1] > 0, ls[:, 0] / ls[:, 1].clamp(min=1e-300), torch.zeros_like(ls[:, 0]))
        self._vals = v.float()
        return self._vals

    def _update(self, t, k):
        leaf = self.builder.leaf_of_row.long()
        out = ~self.inbag & (self.w > 0)
        self.oob[:, k] += torch.where(out, self._vals[leaf].double(), torch.zeros_like(self.oob[:, k]))
        if k == self.K - 1:
            self.oob_n += out.double()

    def _training_metrics(self, model):
        has = self.oob_n > 0
        if not bool(has.any()):
            return None
        y, w = self.y[has], self.w[has]
        s = self.oob[has] / self.oob_n[has, None]
        if self.nclass == 1:
            return mm.regression_metrics(y, s[:, 0].float(), w)
        if self.nclass == 2 and not self.double:
            return mm.binomial_metrics(y, s[:, 0].clamp(0, 1).float(), w, self.info.response_domain)
        p = s.clamp(min=0)
        p = p / p.sum(1, keepdim=True).clamp(min=1e-30)
        if self.nclass == 2:
            return mm.binomial_metrics(y, p[:, 1].float(), w, self.info.response_domain)
        return mm.multinomial_metrics(y, p.float(), w, self.info.response_domain)
