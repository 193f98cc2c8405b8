"""Single Decision Tree, binary classification (reference: ``hex/tree/dt/DT.java``, ``DTModel.java``,
``CompressedDT.java``, ``binning/BinningStrategy.java`` (EQUAL_WIDTH), ``binning/FeatureBins.java``,
``mrtasks/FeaturesLimitsMRTask.java``, ``mrtasks/CountBinsSamplesCountsMRTask.java``).

The reference algorithm, level-synchronous on the device:

* every node re-bins every feature over the node's OWN value range: real limits ``(min - 1e-6, max]`` of the
  node's rows (``FeaturesLimitsMRTask``), 10 equal-width bins whose inner boundaries are rounded half-up to
  2 decimals, the first bin's lower edge pushed 1e-4 steps below the minimum and the last edge = the max
  (``BinningStrategy.EQUAL_WIDTH``); a row belongs to bin ``(lo, hi]``;
* the split criterion is the weighted binary entropy (natural log) of the class-0 frequency on each side,
  minimised over (feature, bin) with ``min_rows`` rows required on both sides; ties keep the first bin /
  the first feature (``DT.findBestSplit``);
* a node is a leaf at ``max_depth``, when a class has ``<= min_rows`` rows, when no split qualifies, or
  when the entropy decrease is below 1e-6 (``DT.buildNextNode``);
* leaves predict the majority class (ties -> class 0) and P(class 0) = count0 / count (``makeLeafFromNode``);
  scoring sends ``x <= threshold`` left (``CompressedDT.predictRowStartingFromNode``).

All (node, feature) histograms of a level are built with one ``bincount`` per feature over rows grouped by
node, so a level costs O(N * F) device work whatever the number of nodes. Nodes keep the reference's heap
numbering (children of i are 2i+1, 2i+2). Row membership follows the parent/child partition (the reference
re-evaluates the limit conjunction, which differs only when a rounded inner threshold exceeds the node's
maximum).
"""
from __future__ import annotations

import time
from decimal import ROUND_HALF_UP, Decimal

import numpy as np
import torch

from ..parallel import collectives as coll
from .base import DataInfo, Model, make_key


def _red(t: torch.Tensor, op=None) -> torch.Tensor:
    """All-reduce over the row shards (no-op in one process): DT's MRTasks (limits, bin counts)."""
    if not coll.is_dist():
        return t
    return coll.all_reduce_(t.contiguous().to(coll.comm_device()), op).to(t.device)

EPSILON = 1e-6            # DT.EPSILON (limits)
MIN_IMPROVEMENT = 1e-6    # DT.MIN_IMPROVEMENT
NUM_BINS = 10             # BinningStrategy.EQUAL_WIDTH.NUM_BINS
PREC_EPS = 2.0 ** -53     # commons-math Precision.EPSILON


def _round2(v: float) -> float:
    """``new BigDecimal(v).setScale(2, HALF_UP).doubleValue()`` (exact decimal expansion of the double)."""
    return float(Decimal(v).quantize(Decimal("0.01"), rounding=ROUND_HALF_UP))


def bin_edges(rmin: float, rmax: float):
    """EQUAL_WIDTH bins of one feature over real limits (rmin, rmax]: list of (lo, hi) or None (constant)."""
    step = (rmax - rmin) / NUM_BINS
    if step == 0:
        return None
    vals = []
    v = rmin
    while v <= rmax:
        vals.append(v)
        v += step
    if len(vals) < 2:
        return None
    bins = [[_round2(vals[i]), _round2(vals[i + 1])] for i in range(len(vals) - 1)]
    bins[0][0] = rmin - 0.0001 * (vals[1] - vals[0])
    bins[-1][1] = rmax
    return bins


def _entropy(p0):
    """DT.entropyBinarySplit (vectorised): -(p log p + (1-p) log(1-p)), terms below Precision.EPSILON dropped."""
    q = 1.0 - p0
    a = torch.where(p0 < PREC_EPS, torch.zeros_like(p0), p0 * torch.log(p0.clamp(min=1e-300)))
    b = torch.where(q < PREC_EPS, torch.zeros_like(q), q * torch.log(q.clamp(min=1e-300)))
    return -(a + b)


class DTModel(Model):
    algo = "dt"

    def __init__(self, key, params, info):
        super().__init__(key, params, info)
        self.tree = {}     # heap index -> (is_leaf, feature | decision, threshold | P(class 0))

    def _arrays(self, dev):
        idx = sorted(self.tree)
        n = (max(idx) + 1) if idx else 1
        leaf = torch.ones(n, dtype=torch.bool)
        a = torch.zeros(n, dtype=torch.float64)
        b = torch.zeros(n, dtype=torch.float64)
        for i in idx:
            lf, x1, x2 = self.tree[i]
            leaf[i], a[i], b[i] = bool(lf), float(x1), float(x2)
        return leaf.to(dev), a.to(dev), b.to(dev)

    def _predict_tensor(self, X, offset=None):
        dev = X.device
        leaf, a, b = self._arrays(dev)
        N = X.shape[1]
        node = torch.zeros(N, dtype=torch.long, device=dev)
        Xd = X.double()
        for _ in range(int(self.params.get("max_depth", 20)) + 1):
            lf = leaf[node]
            if bool(lf.all()):
                break
            f = a[node].long().clamp(min=0, max=X.shape[0] - 1)
            x = Xd.gather(0, f[None, :])[0]
            t = b[node]
            go_left = (x < t) | ((x - t).abs() <= PREC_EPS)
            nxt = torch.where(go_left, 2 * node + 1, 2 * node + 2)
            node = torch.where(lf, node, nxt.clamp(max=leaf.numel() - 1))
        p0 = b[node]
        return torch.stack([p0, 1.0 - p0], 1).float()

    def default_threshold(self):
        # the label is the leaf's majority class (count1 > count0), not an F1-optimal threshold
        return 0.5 + 1e-12

    def rules(self):
        """CompressedDT.getListOfRules: one text rule per leaf (``(x<f> <= t) and ... -> (decision, P0)``)."""
        out = []

        def walk(i, rule):
            lf, x1, x2 = self.tree[i]
            if lf:
                out.append(f"{rule} -> ({float(x1)}, {float(x2)})")
                return
            pre = rule + " and " if rule else rule
            walk(2 * i + 1, pre + f"(x{float(x1)} <= {float(x2)})")
            walk(2 * i + 2, pre + f"(x{float(x1)} > {float(x2)})")
        if self.tree:
            walk(0, "")
        return out

    def to_state(self):
        s = super().to_state()
        s["tree"] = [[int(k), int(v[0]), float(v[1]), float(v[2])] for k, v in sorted(self.tree.items())]
        return s

    def _restore(self, s):
        super()._restore(s)
        self.tree = {int(k): (int(lf), x1, x2) for k, lf, x1, x2 in s["tree"]}


class DTTrainer:
    algo = "dt"
    model_cls = DTModel

    def __init__(self, params):
        p = dict(max_depth=20, min_rows=10)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def _checks(self, X, info):
        errs = []
        if int(self.p["max_depth"]) < 1:
            errs.append("Max depth has to be at least 1")
        bad = _red(torch.tensor([float(torch.isnan(X).any()), float(torch.isinf(X).any())], dtype=torch.float64))
        if bad[0] > 0:
            errs.append("NaNs are not supported yet")
        if bad[1] > 0:
            errs.append("Infs are not supported")
        if any(int(c) for c in np.asarray(info.iscat).reshape(-1)):
            errs.append("Categorical features are not supported yet")
        if info.response_domain is None:
            errs.append("Only categorical response is supported")
        elif len(info.response_domain) != 2:
            errs.append("Only binary response is supported")
        if errs:
            raise ValueError("Illegal argument(s) for DT model: " + "; ".join(errs))

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        t0 = time.time()
        self._checks(X, info)
        p = self.p
        D, min_rows = int(p["max_depth"]), int(p["min_rows"])
        dev = X.device
        F, N = X.shape
        Xd = X.double()
        yc = torch.nan_to_num(y, nan=0).long().clamp(0, 1)
        model = DTModel(model_key or make_key("dt"), p, info)
        model.device = dev
        # root: rows within the initial limits (v.min - EPSILON, v.max]
        import torch.distributed as dist
        big = torch.finfo(torch.float64).max
        lo0 = _red(Xd.min(1).values if N else torch.full((F,), big, dtype=torch.float64, device=dev),
                   dist.ReduceOp.MIN) - EPSILON
        hi0 = _red(Xd.max(1).values if N else torch.full((F,), -big, dtype=torch.float64, device=dev), dist.ReduceOp.MAX)
        member = ((Xd > lo0[:, None]) & (Xd <= hi0[:, None])).all(0)
        node_of_row = torch.where(member, torch.zeros(N, dtype=torch.long, device=dev),
                                  torch.full((N,), -1, dtype=torch.long, device=dev))
        level = [0]          # heap indices of this level's nodes (position = local node id)
        for depth in range(D + 1):
            K = len(level)
            if K == 0:
                break
            ok = node_of_row >= 0
            cnt = _red(torch.bincount(node_of_row[ok] * 2 + yc[ok], minlength=2 * K).double()).reshape(K, 2).cpu().numpy()
            stop = (depth >= D) | (cnt[:, 0] <= min_rows) | (cnt[:, 1] <= min_rows)
            best = self._best_splits(Xd, yc, node_of_row, K, ~stop, min_rows) if (~stop).any() else {}
            nxt, route = [], np.full((K, 3), -1.0)
            for k, hidx in enumerate(level):
                c0, c1 = int(cnt[k, 0]), int(cnt[k, 1])
                b = best.get(k)
                if not stop[k] and b is not None:
                    parent = float(_entropy(torch.tensor(c0 / max(c0 + c1, 1), dtype=torch.float64)))
                    if abs(parent - b[2]) >= MIN_IMPROVEMENT:
                        model.tree[hidx] = (0, b[0], b[1])
                        route[k] = (b[0], b[1], len(nxt))
                        nxt += [2 * hidx + 1, 2 * hidx + 2]
                        continue
                tot = max(c0 + c1, 1)
                model.tree[hidx] = (1, 1 if c1 > c0 else 0, c0 / tot)
            if not nxt:
                break
            # route rows of split nodes: left child iff x_f <= threshold; leaves drop out
            rt = torch.as_tensor(route, device=dev)
            nr = node_of_row.clamp(min=0)
            f = rt[nr, 0].long()
            split = ok & (f >= 0)
            x = Xd.gather(0, f.clamp(min=0)[None, :])[0]
            left = x <= rt[nr, 1]
            child = rt[nr, 2].long() + (~left).long()
            node_of_row = torch.where(split, child, torch.full_like(node_of_row, -1))
            level = nxt
        model.output["training_metrics"] = model.metrics_for(X, y, None)
        if valid is not None:
            Xv, yv, wv, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, None)
        model.output["rules"] = model.rules()
        model.output["nodes_count"] = len(model.tree)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model

    @staticmethod
    def _best_splits(Xd, yc, node_of_row, K, active, min_rows):
        """Best (feature, threshold, criterion) per active node of a level (DT.findBestSplit)."""
        dev = Xd.device
        F, N = Xd.shape
        act = torch.as_tensor(active, device=dev)
        ok = node_of_row >= 0
        rows = torch.nonzero(ok & act[node_of_row.clamp(min=0)]).squeeze(1)
        if int(coll.all_reduce_scalar(float(rows.numel()))) == 0:
            return {}
        nd = node_of_row[rows]
        Xr = Xd[:, rows]
        yr = yc[rows]
        # real limits of each node's rows (FeaturesLimitsMRTask: min - EPSILON, max)
        big = torch.finfo(torch.float64).max
        mn = torch.full((F, K), big, dtype=torch.float64, device=dev).scatter_reduce(
            1, nd[None, :].expand(F, -1), Xr, "amin", include_self=True)
        mx = torch.full((F, K), -big, dtype=torch.float64, device=dev).scatter_reduce(
            1, nd[None, :].expand(F, -1), Xr, "amax", include_self=True)
        import torch.distributed as dist
        mn, mx = _red(mn, dist.ReduceOp.MIN), _red(mx, dist.ReduceOp.MAX)
        mn_h, mx_h = (mn - EPSILON).cpu().numpy(), mx.cpu().numpy()
        NB = NUM_BINS + 1
        lo = np.full((K, F, NB), np.inf)
        hi = np.full((K, F, NB), np.inf)
        nbins = np.zeros((K, F), np.int64)
        for k in np.nonzero(active)[0]:
            for f in range(F):
                bins = bin_edges(float(mn_h[f, k]), float(mx_h[f, k]))
                if bins is None:
                    continue
                nb = len(bins)
                nbins[k, f] = nb
                lo[k, f, :nb] = [b_[0] for b_ in bins]
                hi[k, f, :nb] = [b_[1] for b_ in bins]
        lo_t = torch.as_tensor(lo, device=dev)
        hi_t = torch.as_tensor(hi, device=dev)
        hs_t = torch.cummax(hi_t, 2).values          # search keys (a rounded inner edge may exceed the max)
        counts = torch.zeros(K, F, NB, 2, dtype=torch.float64, device=dev)
        for f in range(F):
            x = Xr[f]
            H = hs_t[nd, f]                        # [n, NB] upper edges of the row's node
            b = torch.searchsorted(H, (x - PREC_EPS)[:, None]).squeeze(1)   # first bin with x <= hi (+ tolerance)
            bc = b.clamp(max=NB - 1)
            inb = (b < NB) & (x > lo_t[nd, f, bc])
            key = ((nd * F + f) * NB + bc) * 2 + yr
            counts.view(-1).index_add_(0, key[inb], torch.ones(int(inb.sum()), dtype=torch.float64, device=dev))
        c = _red(counts)                             # [K, F, NB, 2]
        left = c.cumsum(2)
        tot = c.sum(2, keepdim=True)
        right = tot - left
        lc, lc0 = left.sum(3), left[..., 0]
        rc, rc0 = right.sum(3), right[..., 0]
        n = lc + rc
        crit = (_entropy(lc0 / lc.clamp(min=1)) * lc + _entropy(rc0 / rc.clamp(min=1)) * rc) / n.clamp(min=1)
        valid_bin = torch.arange(NB, device=dev)[None, None, :] < torch.as_tensor(nbins, device=dev)[:, :, None]
        valid_bin &= (lc >= min_rows) & (rc >= min_rows)
        crit = torch.where(valid_bin, crit, torch.full_like(crit, float("inf")))
        # first minimal bin per (node, feature), then first strictly smaller feature
        bmin, barg = crit.min(2)
        fbest, farg = bmin.min(1)
        fb, fa, ba = fbest.cpu().numpy(), farg.cpu().numpy(), barg.cpu().numpy()
        out = {}
        for k in np.nonzero(active)[0]:
            if not np.isfinite(fb[k]):
                continue
            f = int(fa[k])
            bi = int(ba[k, f])
            out[int(k)] = (f, float(hi[k, f, bi]), float(fb[k]))
        return out
