"""Aggregator (reference: ``hex/aggregator/Aggregator.java``, ``AggregatorModel.java``).

Leader clustering of rows in the standardized (one-hot) space: a row within ``radius`` of an
existing exemplar is absorbed (its count added), otherwise it becomes a new exemplar. The radius
is tuned by bisection on a sample so the exemplar count lands within ``rel_tol_num_exemplars`` of
``target_num_exemplars``; the full pass then streams rows in chunks, using the fused HIP nearest-
center kernel for the chunk-vs-exemplar distances. Output: the aggregated frame (exemplar rows +
``counts``) and the row -> exemplar mapping.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from ..ops.dense import kmeans_assign
from .base import DataInfo, Model, make_key
from .datainfo import Expander
from ..ops.segment import segment_sum

AGG_DEFAULTS = dict(target_num_exemplars=5000, rel_tol_num_exemplars=0.5, transform="NORMALIZE",
                    categorical_encoding="AUTO", save_mapping_frame=False, num_iteration_without_new_exemplar=500,
                    seed=-1)


def _leader(Z, r2, chunk=8192):
    """Greedy leader clustering; returns exemplar row indices and per-row exemplar id."""
    N = Z.shape[0]
    ex_idx = [0]
    C = Z[0:1].clone()
    assign = torch.empty(N, dtype=torch.long, device=Z.device)
    for s in range(0, N, chunk):
        blk = Z[s:s + chunk]
        a, d = kmeans_assign(blk, C)
        far = torch.nonzero(d > r2).flatten()
        while far.numel():
            j = int(far[0])
            ex_idx.append(s + j)
            C = torch.cat([C, blk[j:j + 1]], 0)
            dn = ((blk[far] - blk[j]) ** 2).sum(1)
            newk = C.shape[0] - 1
            upd = dn <= r2
            a[far[upd]] = newk
            d[far[upd]] = dn[upd]
            far = far[~upd]
        assign[s:s + chunk] = a
    return torch.as_tensor(ex_idx, device=Z.device), assign


class AggregatorModel(Model):
    algo = "aggregator"

    def __init__(self, key, params, info):
        super().__init__(key, params, info)
        self.output["model_category"] = "Clustering"

    @property
    def model_category(self):
        return "Clustering"

    def aggregated_frame(self):
        from ..core import dkv
        return dkv.get(self.output["output_frame"])

    def _predict_tensor(self, X, offset=None):
        raise NotImplementedError("Aggregator has no predict; use aggregated_frame")


class AggregatorTrainer:
    def __init__(self, params):
        p = dict(AGG_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None
        self.frame = None   # set by the builder hook to build the output frame with original values

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        t0 = time.time()
        p = self.p
        dev = X.device
        ex = Expander(info, standardize=str(p["transform"]).upper() != "NONE", use_all_factor_levels=True).fit(X)
        Z = ex.transform(X)
        N = Z.shape[0]
        target = int(p["target_num_exemplars"])
        tol = float(p["rel_tol_num_exemplars"])
        if N <= target:
            ex_rows, assign = torch.arange(N, device=dev), torch.arange(N, device=dev)
        else:
            g = torch.Generator().manual_seed(17)
            ns = min(N, 20000)
            samp = Z[torch.randperm(N, generator=g)[:ns].to(dev)]
            dim = Z.shape[1]
            lo, hi = 0.0, float(dim) * 16
            want = target * ns / N
            r2 = hi / 4
            for _ in range(30):   # bisection on the squared radius
                e, _ = _leader(samp, r2)
                if e.numel() > want:
                    lo = r2
                else:
                    hi = r2
                if abs(e.numel() - want) <= tol * want:
                    break
                r2 = (lo + hi) / 2
            ex_rows, assign = _leader(Z, r2)
            dim_eff = max(1.0, min(float(Z.shape[1]), 8.0))
            for _ in range(4):   # the sample extrapolation can miss: correct the radius on the full pass
                n_ex = ex_rows.numel()
                if abs(n_ex - target) <= tol * target:
                    break
                r2 *= (n_ex / target) ** (2.0 / dim_eff)
                ex_rows, assign = _leader(Z, r2)
        counts = segment_sum(assign, torch.ones(N, dtype=torch.float64, device=dev), ex_rows.numel())
        model = AggregatorModel(model_key or make_key("aggregator"), p, info)
        model.device = dev
        model.output["exemplar_rows"] = ex_rows.cpu().tolist()
        model.output["counts"] = counts.cpu().tolist()
        model.output["num_exemplars"] = int(ex_rows.numel())
        from ..frame import Column, H2OFrame
        cols = []
        for j, n in enumerate(info.x):
            v = X[j][ex_rows]
            if info.iscat[j]:
                codes = torch.where(torch.isnan(v), torch.full_like(v, -1), v).to(torch.int32)
                cols.append(Column(n, "enum", codes, list(info.domains[j])))
            else:
                cols.append(Column(n, "real", v.double()))
        cols.append(Column("counts", "int", counts))
        fr = H2OFrame._from_columns(cols)
        model.output["output_frame"] = fr.frame_id
        if p["save_mapping_frame"]:
            mf = H2OFrame._from_columns([Column("exemplar_assignment", "int", assign.double())])
            model.output["mapping_frame"] = mf.frame_id
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
