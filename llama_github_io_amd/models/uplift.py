"""Uplift Distributed Random Forest (reference: ``hex/tree/uplift/UpliftDRF.java``,
``UpliftDRFModel.java``, ``Divergence.java``, ``KLDivergence.java``, ``EuclideanDistance.java``,
``ChiSquaredDivergence.java``; AUUC from ``hex/AUUC.java``).

Trees are grown level-wise on device from the shared global binning: per active node, feature and
bin the four sufficient statistics (n_treat, y_treat, n_ctrl, y_ctrl) are one ``index_add_``;
a cumulative sum over bins gives every threshold's left/right treatment and control response
rates and the divergence gain ``p_L·D(L) + p_R·D(R) − D(parent)`` with
D(pt, pc) = m(pt, pc) + m(1−pt, 1−pc) for the chosen metric (KL, Euclidean, ChiSquared).
Columns are sampled per node (``mtries``), rows per tree (``sample_rate``). Leaves keep P(y=1|T)
and P(y=1|C); the forest predicts ``uplift_predict``, ``p_y1_with_treatment``,
``p_y1_without_treatment`` (averages over trees). Training metrics: AUUC (qini, lift, gain).
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from ..ops.binning import apply_binning, fit_binning_rows
from ..parallel import collectives as coll
from ..ops.forest import Forest, Tree
from ..ops.tree import NA_BIN
from ..ops.segment import segment_sum
from .base import DataInfo, Model, make_key

UPLIFT_DEFAULTS = dict(ntrees=50, max_depth=20, min_rows=10.0, mtries=-2, sample_rate=0.632, nbins=20,
                       treatment_column="treatment", uplift_metric="AUTO", auuc_type="AUTO", auuc_nbins=-1, seed=-1)
ZERO = 1e-6


def _metric(kind, a, b):
    if kind == "kl":
        return a * torch.log2(torch.where(a > 0, a, torch.ones_like(a)) / torch.where(b > 0, b, torch.full_like(b, ZERO))) * (a > 0)
    if kind == "chisquared":
        return (a - b) ** 2 / torch.where(b > 0, b, torch.full_like(b, ZERO))
    return (a - b) ** 2


def _D(kind, pt, pc):
    return _metric(kind, pt, pc) + _metric(kind, 1 - pt, 1 - pc)


def _merge(t):
    if not coll.is_dist():
        return t
    return coll.all_reduce_(t.contiguous().to(coll.comm_device())).to(t.device)


def auuc(uplift, y, treat, nbins=1000, auuc_type="AUTO"):
    """Qini / lift / gain AUUC (AUUC.java); ``AUUC`` is the ``auuc_type`` curve (AUTO = qini) averaged
    over ``nbins`` thresholds. Thresholds are the uplift values at ``nbins`` evenly spaced descending
    ranks (exact order statistics — also over row shards); each threshold's treatment / control counts
    and responses are those of the rows scoring at or above it (ties included), merged by all-reduce."""
    from ..parallel.order_stats import order_statistics
    nbins = 1000 if nbins is None or int(nbins) <= 0 else int(nbins)
    u = uplift.double()
    N = int(coll.all_reduce_scalar(float(u.numel()))) if coll.is_dist() else u.numel()
    idx = torch.linspace(0, N - 1, min(nbins, N), dtype=torch.float64).long().clamp_(0, N - 1)
    thr = torch.tensor(order_statistics(u, (N - idx).tolist()), dtype=torch.float64, device=u.device)   # descending
    asc = thr.flip(0)
    # rows contribute to every threshold <= their uplift: bucket = #thresholds <= u, then suffix sums
    j = torch.searchsorted(asc, u, right=True)
    y, t = y.double(), treat.double()
    stats = torch.stack([t, 1 - t, y * t, y * (1 - t)], 1)
    m = idx.numel()
    c = _merge(segment_sum(j, stats, m + 1))
    S = torch.flip(torch.cumsum(torch.flip(c, [0]), 0), [0])[1:]         # S[k-1] = rows with >= k thresholds below
    S = S.flip(0)                                                      # descending threshold order
    nt, nc, yt, yc = S[:, 0], S[:, 1], S[:, 2], S[:, 3]
    qini = yt - yc * nt / nc.clamp(min=1)
    lift = yt / nt.clamp(min=1) - yc / nc.clamp(min=1)
    gain = lift * (nt + nc)
    curves = dict(qini=qini, lift=lift, gain=gain)
    kind = str(auuc_type or "AUTO").lower()
    kind = "qini" if kind == "auto" else kind
    if kind not in curves:
        raise ValueError(f"auuc_type must be AUTO, qini, lift or gain, got {auuc_type!r}")
    return dict(qini=float(qini.mean()), lift=float(lift.mean()), gain=float(gain.mean()), auuc_type=kind,
                auuc_nbins=int(idx.numel()), AUUC=float(curves[kind].mean()),
                auuc_table={k: v.cpu().tolist() for k, v in curves.items()})


class UpliftDRFModel(Model):
    algo = "upliftdrf"

    def _predict_tensor(self, X, offset=None):
        n = max(1, len(self.f_t))
        pt = self.f_t.predict_raw(X.to(self.device))[:, 0] / n
        pc = self.f_c.predict_raw(X.to(self.device))[:, 0] / n
        return torch.stack([pt - pc, pt, pc], 1).float()

    @property
    def model_category(self):
        return "BinomialUplift"

    def prediction_names(self):
        return ["uplift_predict", "p_y1_with_treatment", "p_y1_without_treatment"]


class UpliftDRFTrainer:
    def __init__(self, params):
        p = dict(UPLIFT_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from .shared_tree import resolve_seed
        t0 = time.time()
        p = self.p
        tc = p["treatment_column"]
        if tc not in info.x:
            raise ValueError(f"treatment_column {tc} must be a (categorical) column of the frame")
        jt = info.x.index(tc)
        treat = torch.nan_to_num(X[jt]).double()
        keep = [j for j in range(info.F) if j != jt]
        sub = DataInfo([info.x[j] for j in keep], np.asarray(info.iscat)[keep], [info.domains[j] for j in keep],
                       info.response, info.response_domain)
        Xs = X[keep].contiguous()
        F, N = Xs.shape
        dev = X.device
        seed = resolve_seed(p["seed"])
        gen = torch.Generator().manual_seed(seed & 0x7FFFFFFF)
        # row-sharded: global binning (sampled rows only), global-index in-bag draws, node statistics and
        # histograms all-reduced -> every rank grows the single-process trees
        b = fit_binning_rows(Xs, sub.iscat, sub.nlevels, max_bins=max(int(p["nbins"]), 2) * 4, seed=seed)
        row0 = coll.row_offset(N) if coll.is_dist() else 0
        bins = apply_binning(b, Xs)[:, :F].long()                      # [N, F]
        yv = torch.nan_to_num(y).double()
        kind = str(p["uplift_metric"]).lower()
        kind = "kl" if kind == "auto" else kind
        mt = int(p["mtries"])
        kcols = F if mt in (-2, 0) or mt >= F else (max(1, int(math.sqrt(F))) if mt == -1 else mt)
        f_t, f_c = Forest(n_classes_out=1), Forest(n_classes_out=1)
        min_rows = float(p["min_rows"])
        for t in range(int(p["ntrees"])):
            inbag = coll.row_uniform(seed, 7000 + t, row0, N, dev) < float(p["sample_rate"])
            tree_t, tree_c = self._grow(bins, b, yv, treat, inbag, int(p["max_depth"]), min_rows, kcols, kind, gen, F)
            f_t.add(tree_t)
            f_c.add(tree_c)
            if self.job is not None:
                self.job.set_progress((t + 1) / int(p["ntrees"]))
        model = UpliftDRFModel(model_key or make_key("upliftdrf"), p, sub)
        model.device = dev
        model.f_t, model.f_c = f_t, f_c
        model.output["model_category"] = "BinomialUplift"
        P = model._predict_tensor(Xs)
        model.output["training_metrics"] = auuc(P[:, 0], yv, treat, p.get("auuc_nbins"), p.get("auuc_type"))
        model.output["training_metrics"]["model_category"] = "BinomialUplift"
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model

    def _grow(self, bins, b, y, treat, inbag, max_depth, min_rows, kcols, kind, gen, F):
        N = bins.shape[0]
        dev = bins.device
        node = torch.where(inbag, torch.zeros(N, dtype=torch.long, device=dev), torch.full((N,), -1, dtype=torch.long, device=dev))
        recs = [dict(feat=-1, thr=0.0, na_left=0, left=-1, right=-1, pt=0.0, pc=0.0)]
        level = [0]
        stats = torch.stack([treat, treat * y, 1 - treat, (1 - treat) * y], 1)     # [N, 4]
        for d in range(max_depth + 1):
            A = len(level)
            act = node >= 0
            rows = torch.nonzero(act).flatten()
            nd = node[rows]
            tot = _merge(segment_sum(nd, stats[rows], A))
            pt_n = tot[:, 1] / tot[:, 0].clamp(min=1)
            pc_n = tot[:, 3] / tot[:, 2].clamp(min=1)
            for i, gid in enumerate(level):
                recs[gid]["pt"], recs[gid]["pc"] = float(pt_n[i]), float(pc_n[i])
            if d == max_depth or int(coll.all_reduce_scalar(float(rows.numel()))) == 0:
                break
            idx = (nd[:, None] * F + torch.arange(F, device=dev)[None, :]) * 256 + bins[rows]
            H = torch.zeros(A * F * 256, 4, dtype=torch.float64, device=dev)
            H.index_add_(0, idx.reshape(-1), stats[rows].repeat_interleave(F, 0))
            H = _merge(H).view(A, F, 256, 4)
            L = torch.cumsum(H[:, :, :NA_BIN], 2)                   # left = bins < t+1
            R = tot[:, None, None, :] - L
            nL = L[..., 0] + L[..., 2]
            nR = R[..., 0] + R[..., 2]
            ok = (L[..., 0] >= 1) & (L[..., 2] >= 1) & (R[..., 0] >= 1) & (R[..., 2] >= 1) & (nL >= min_rows) & (nR >= min_rows)
            ptL, pcL = L[..., 1] / L[..., 0].clamp(min=1), L[..., 3] / L[..., 2].clamp(min=1)
            ptR, pcR = R[..., 1] / R[..., 0].clamp(min=1), R[..., 3] / R[..., 2].clamp(min=1)
            n = (nL + nR).clamp(min=1)
            gain = (nL / n) * _D(kind, ptL, pcL) + (nR / n) * _D(kind, ptR, pcR) - _D(kind, pt_n, pc_n)[:, None, None]
            gain = torch.where(ok, gain, torch.full_like(gain, -1e300))
            if kcols < F:
                keys = torch.rand(A, F, generator=gen).to(dev)
                allowed = keys.argsort(1).argsort(1) < kcols
                gain = torch.where(allowed[:, :, None], gain, torch.full_like(gain, -1e300))
            flat = gain.view(A, -1)
            best, arg = flat.max(1)
            bf = arg // (NA_BIN)
            bt = arg % (NA_BIN) + 1                                  # bins < bt go left
            nxt_level = []
            new_node = torch.full_like(node, -1)
            for i, gid in enumerate(level):
                if float(best[i]) <= 1e-12:
                    continue
                f, tb = int(bf[i]), int(bt[i])
                e = b.edges[f]
                thr = float(e[tb - 1]) if e is not None and tb - 1 < len(e) else float(tb) - 0.5
                lid, rid = len(recs), len(recs) + 1
                recs.append(dict(feat=-1, thr=0.0, na_left=0, left=-1, right=-1, pt=0.0, pc=0.0))
                recs.append(dict(feat=-1, thr=0.0, na_left=0, left=-1, right=-1, pt=0.0, pc=0.0))
                recs[gid].update(feat=f, thr=thr, left=lid, right=rid)
                m = node == i
                gl = bins[:, f] < tb
                new_node = torch.where(m & gl, torch.full_like(node, len(nxt_level)), new_node)
                new_node = torch.where(m & ~gl, torch.full_like(node, len(nxt_level) + 1), new_node)
                nxt_level += [lid, rid]
            node = new_node
            level = nxt_level
            if not level:
                break

        def mk(val_key):
            n = len(recs)
            return Tree(feat=np.array([r["feat"] for r in recs], np.int32), thr=np.array([r["thr"] for r in recs], np.float32),
                        bin=np.zeros(n, np.int32), na_left=np.zeros(n, np.int8), is_cat=np.zeros(n, np.int8),
                        cat_bits=[None] * n, cat_nbits=np.zeros(n, np.int32),
                        left=np.array([r["left"] for r in recs], np.int32), right=np.array([r["right"] for r in recs], np.int32),
                        value=np.array([r[val_key] if r["feat"] < 0 else 0.0 for r in recs], np.float32),
                        cover=np.zeros(n), gain=np.zeros(n))
        return mk("pt"), mk("pc")
