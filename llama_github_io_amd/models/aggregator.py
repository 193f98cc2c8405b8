"""Aggregator (reference: ``hex/aggregator/Aggregator.java``, ``AggregatorModel.java``).

Leader clustering of rows in the standardized (one-hot) space: a row within ``radius`` of an
existing exemplar is absorbed (its count added), otherwise it becomes a new exemplar. The radius
is tuned by bisection on a sample so the exemplar count lands within ``rel_tol_num_exemplars`` of
``target_num_exemplars``; the full pass runs the leader pass per row chunk, using the fused HIP nearest-
center kernel for the chunk-vs-exemplar distances, and merges the chunks' exemplar lists in chunk order
by the same leader rule (counts added) — the reference's map per chunk + reduce of exemplar lists
(``Aggregator.java`` AggregateTask / ``Exemplar.addExemplars``). Output: the aggregated frame (exemplar
rows + ``counts``) and the row -> exemplar mapping.

Chunks are fixed blocks of GLOBAL row ids, so the answer never depends on how rows are sharded: a chunk
that straddles a shard boundary is completed on the rank holding its first row (one all-to-all moving at
most one chunk of rows per boundary), the bisection sample is drawn by a counter-based per-row RNG, and
only exemplar lists travel (all-gather, model-sized); the mapping of moved rows goes back the same way.
"""
from __future__ import annotations

import contextlib
import os
import time

import numpy as np
import torch

from ..ops.dense import kmeans_assign
from ..parallel import collectives as coll, dframe
from .base import DataInfo, Model, make_key
from .datainfo import Expander
from ..ops.segment import segment_sum

AGG_DEFAULTS = dict(target_num_exemplars=5000, rel_tol_num_exemplars=0.5, transform="NORMALIZE",
                    categorical_encoding="AUTO", save_mapping_frame=False, num_iteration_without_new_exemplar=500,
                    seed=-1)
CHUNK = 1 << 16          # rows per leader chunk (global row ids); H2O_AGG_CHUNK overrides


def _leader(Z, r2, chunk=8192):
    """Greedy leader clustering; returns exemplar row indices and per-row exemplar id."""
    N = Z.shape[0]
    if N == 0 or r2 < 0:      # r2 < 0: every row is its own exemplar
        return torch.arange(N, device=Z.device), torch.arange(N, device=Z.device)
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
        sharded = coll.is_dist()
        CH = int(os.environ.get("H2O_AGG_CHUNK", CHUNK))
        ex = Expander(info, standardize=str(p["transform"]).upper() != "NONE", use_all_factor_levels=True).fit(
            X, reduce=coll.all_reduce_ if sharded else None)
        Z = ex.transform(X).float()
        n_loc = Z.shape[0]
        start, N = coll.exclusive_offset(n_loc)
        gid = torch.arange(start, start + n_loc, dtype=torch.float64, device=dev)
        # complete the chunks that straddle shard boundaries on the rank holding their first row
        payload = torch.cat([gid[:, None], Z.double(), X.T.double()], 1)
        offs = None
        if sharded:
            cnt = coll.all_gather_object(n_loc)
            offs = torch.tensor(np.cumsum([0] + cnt), dtype=torch.float64, device=dev)
            first = (torch.div(gid, CH, rounding_mode="floor") * CH)
            dest = torch.searchsorted(offs, first.contiguous(), right=True) - 1
            payload = coll.exchange_rows(payload, dest)
        gids, Zc, Xc = payload[:, 0], payload[:, 1:1 + Z.shape[1]].float(), payload[:, 1 + Z.shape[1]:]
        chunk = torch.div(gids, CH, rounding_mode="floor").long()
        target = int(p["target_num_exemplars"])
        tol = float(p["rel_tol_num_exemplars"])
        if N <= target:
            r2 = -1.0
        else:
            ns = min(N, 20000)
            u = coll.row_uniform(17, 5, start, n_loc, dev)
            samp = Z[u < ns / N]
            if sharded:
                samp = coll.all_gather_cat(samp.to(coll.comm_device()), bounded=True).to(dev)
            ns = max(samp.shape[0], 1)
            lo, hi = 0.0, float(Z.shape[1]) * 16
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
        res = self._pass(Zc, gids, Xc, chunk, r2)
        if N > target:
            dim_eff = max(1.0, min(float(Z.shape[1]), 8.0))
            for _ in range(4):   # the sample extrapolation can miss: correct the radius on the full pass
                n_ex = res[0].shape[0]
                if abs(n_ex - target) <= tol * target:
                    break
                r2 *= (n_ex / target) ** (2.0 / dim_eff)
                res = self._pass(Zc, gids, Xc, chunk, r2)
        ex_gid, ex_x, counts, assign = res
        if sharded:
            # the mapping of rows completed on another rank goes back to the rank that holds them
            home = torch.searchsorted(offs, gids.contiguous(), right=True) - 1
            back = coll.exchange_rows(torch.stack([gids, assign.double()], 1), home)
            assign = torch.empty(n_loc, dtype=torch.long, device=dev)
            assign[(back[:, 0] - start).long()] = back[:, 1].long()
        model = AggregatorModel(model_key or make_key("aggregator"), p, info)
        model.device = dev
        model.output["exemplar_rows"] = ex_gid.long().cpu().tolist()
        model.output["counts"] = counts.cpu().tolist()
        model.output["num_exemplars"] = int(ex_gid.numel())
        from ..frame import Column, H2OFrame
        cols = []
        with dframe.shard_ctx(None):     # exemplars: the same (model-sized) frame on every rank
            for j, n in enumerate(info.x):
                v = ex_x[:, j]
                if info.iscat[j]:
                    codes = torch.where(torch.isnan(v), torch.full_like(v, -1), v).to(torch.int32)
                    cols.append(Column(n, "enum", codes, list(info.domains[j])))
                else:
                    cols.append(Column(n, "real", v.double()))
            cols.append(Column("counts", "int", counts))
            fr = H2OFrame._from_columns(cols)
        model.output["output_frame"] = fr.frame_id
        if p["save_mapping_frame"]:
            with dframe.shard_ctx(dframe.make_shard(n_loc)) if sharded else contextlib.nullcontext():
                mf = H2OFrame._from_columns([Column("exemplar_assignment", "int", assign.double())])
            model.output["mapping_frame"] = mf.frame_id
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model

    @staticmethod
    def _pass(Zc, gids, Xc, chunk, r2):
        """Leader pass per chunk, then the chunks' exemplars merged in chunk order by the leader rule.
        Returns (exemplar global row ids, exemplar X rows, counts, merged exemplar id of each local row)."""
        dev = Zc.device
        lead_z, lead_x, lead_g, lead_c, lead_k = [], [], [], [], []
        assign_local = torch.empty(Zc.shape[0], dtype=torch.long, device=dev)
        base = 0
        for k in torch.unique(chunk).tolist():
            idx = torch.nonzero(chunk == k).flatten()
            e, a = _leader(Zc[idx], r2)
            cnt = torch.bincount(a, minlength=e.numel()).double()
            assign_local[idx] = a + base
            base += e.numel()
            lead_z.append(Zc[idx[e]].double()); lead_x.append(Xc[idx[e]]); lead_g.append(gids[idx[e]]); lead_c.append(cnt)
            lead_k.append(torch.full((e.numel(),), float(k), dtype=torch.float64, device=dev))
        D = Zc.shape[1]
        cat = lambda parts, width: torch.cat(parts) if parts else torch.zeros((0,) + width, dtype=torch.float64,
                                                                             device=dev)
        L = torch.cat([cat(lead_k, ())[:, None], cat(lead_g, ())[:, None], cat(lead_c, ())[:, None],
                       cat(lead_z, (D,)), cat(lead_x, (Xc.shape[1],))], 1)
        my_first = 0
        if coll.is_dist():
            sizes = coll.all_gather_object(L.shape[0])
            my_first = int(sum(sizes[:coll.rank()]))
            L = coll.all_gather_cat(L.to(coll.comm_device()), bounded=True).to(dev)
        # chunks are owned by increasing ranks in global order, so rank order is chunk order
        e, a = _leader(L[:, 3:3 + D].float(), r2) if L.shape[0] else (torch.zeros(0, dtype=torch.long, device=dev),
                                                              torch.zeros(0, dtype=torch.long, device=dev))
        counts = torch.zeros(e.numel(), dtype=torch.float64, device=dev).index_add_(0, a, L[:, 2])
        assign = a[my_first + assign_local] if Zc.shape[0] else assign_local
        return L[e, 1], L[e, 3 + D:], counts, assign
