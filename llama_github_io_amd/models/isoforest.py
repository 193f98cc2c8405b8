"""Isolation Forest and Extended Isolation Forest (reference: ``hex/tree/isofor/IsolationForest.java``,
``IsolationForestModel.java``, ``hex/tree/isoforextended/ExtendedIsolationForest.java``,
``hex/genmodel/algos/isoforextended/ExtendedIsolationForestMojoModel.java``).

Isolation Forest runs on the device tree engine in random mode: every tree samples ``sample_size``
rows (or ``sample_rate``), each node draws one column per split (``mtries``) and a random threshold
inside the node's occupied bin range; a leaf stores its depth. The score is H2O's: the summed path
length is normalised by the training min/max, ``predict = (max - len) / (max - min)``, and
``mean_length = len / ntrees``; with ``contamination`` a 0/1 flag column is prepended.

Extended Isolation Forest uses random hyperplanes (``extension_level`` non-zero normal components),
so it cannot reuse axis-aligned histograms: trees are grown from the 256-row sample on the host
(tiny) and scored on device by projecting all rows on every node normal with one GEMM per tree
and walking the levels with gathers. Score ``s = 2^(-E[h(x)] / c(sample_size))``.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import metrics as mm
from ..ops import tree as T
from ..parallel import collectives as coll
from .base import DataInfo, Model, make_key
from .shared_tree import SharedTreeModel, SharedTreeTrainer

IF_DEFAULTS = dict(ntrees=50, max_depth=8, min_rows=1.0, sample_size=256, sample_rate=-1.0, mtries=-1,
                   contamination=-1.0, min_split_improvement=0.0, histogram_type="Random")


def c_factor(n):
    """Average path length of an unsuccessful BST search (``averagePathLengthOfUnsuccessfulSearch``)."""
    n = np.asarray(n, dtype=np.float64)
    out = np.where(n > 2, 2.0 * (np.log(np.maximum(n - 1, 1)) + 0.5772156649) - 2.0 * (n - 1) / np.maximum(n, 1),
                   np.where(n == 2, 1.0, 0.0))
    return out


class IsolationForestModel(SharedTreeModel):
    algo = "isolationforest"

    def _predict_tensor(self, X, offset=None):
        s = self.forest.predict_raw(X)[:, 0].double()
        n = max(1, len(self.forest))
        mn, mx = self.output["min_path_length"], self.output["max_path_length"]
        score = (mx - s) / (mx - mn) if mx > mn else torch.ones_like(s)
        cols = [score.float(), (s / n).float()]
        thr = self.output.get("default_threshold")
        if thr is not None:
            cols.insert(0, (score >= thr).float())
        return torch.stack(cols, 1)

    @property
    def model_category(self):
        return "AnomalyDetection"

    def prediction_names(self):
        base = ["predict", "mean_length"]
        return (["predict", "score", "mean_length"] if self.output.get("default_threshold") is not None else base)


class IsolationForestTrainer(SharedTreeTrainer):
    algo = "isolationforest"
    mode = T.MODE_RANDOM
    model_cls = IsolationForestModel

    def __init__(self, params):
        p = dict(IF_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None or k not in p})
        super().__init__(p)

    def _split_params(self):
        return T.SplitParams(min_w=float(self.p["min_rows"]), min_split_improvement=0.0, mode=T.MODE_RANDOM,
                             random_split=True)

    def _k_cols(self, F):
        m = int(self.p.get("mtries", -1))
        if m in (-1, 1):
            return 1 if F > 1 else 0
        if m == -2 or m >= F:
            return 0
        return m

    def fit(self, X, y, w, offset, info, valid=None, model_key=None):
        info2 = DataInfo(info.x, info.iscat, info.domains, None, None, info.weights, None, None)
        self.label = y
        self.label_info = info
        N = X.shape[1]
        yy = torch.zeros(N, device=X.device)
        model = super().fit(X, yy, w, offset, info2, None, model_key)
        if valid is not None and valid[1] is not None:
            # validation_response_column: binomial metrics of the normalised anomaly score against the labels
            Xv, yv = valid[0], valid[1]
            P = model._predict_tensor(Xv)
            ok = ~torch.isnan(yv)
            dom = self.p.get("_valid_domain") or ["0", "1"]
            model.output["validation_metrics"] = mm.binomial_metrics(yv[ok], P[ok, -2], None, dom)
        return model

    def _init_model(self, model):
        model.output["model_category"] = "AnomalyDetection"
        self.aux = torch.zeros(self.N, 4, dtype=torch.float32, device=self.dev)
        # rows of the WHOLE frame (row-sharded: every rank samples its rows at the same global rate with the
        # global-index row RNG, and the histograms are all-reduced -> the same trees on every rank)
        self.N_glob = int(coll.all_reduce_scalar(self.N)) if coll.is_dist() else self.N

    def _prepare(self, t, k):
        rate = float(self.p.get("sample_rate", -1))
        if rate <= 0:
            rate = min(1.0, float(self.p["sample_size"]) / max(1, self.N_glob))
        ws = self._row_sample(rate, t)
        a = self.aux
        a[:, 0] = ws
        a[:, 3] = ws
        return a

    def _leaf_values(self, ls, t, k):
        return torch.zeros(ls.shape[0], dtype=torch.float32, device=ls.device)

    def _finish(self, model, built):
        for tree in model.forest.trees:
            depth = np.zeros(tree.n_nodes, dtype=np.float32)
            for i in range(tree.n_nodes):
                if tree.feat[i] >= 0:
                    depth[tree.left[i]] = depth[i] + 1
                    depth[tree.right[i]] = depth[i] + 1
            tree.value = np.where(tree.feat < 0, depth, 0).astype(np.float32)
        model.forest._flat.clear()
        s = model.forest.predict_raw(self.X)[:, 0]
        mn, mx = float(s.min()), float(s.max())
        if coll.is_dist():
            import torch.distributed as dist
            mn = coll.all_reduce_scalar(mn, op=dist.ReduceOp.MIN)
            mx = coll.all_reduce_scalar(mx, op=dist.ReduceOp.MAX)
        model.output["min_path_length"] = int(mn)
        model.output["max_path_length"] = int(mx)
        cont = float(self.p.get("contamination", -1))
        if cont > 0:
            from ..parallel.order_stats import global_quantile
            mn, mx = model.output["min_path_length"], model.output["max_path_length"]
            score = (mx - s.double()) / max(mx - mn, 1)
            model.output["default_threshold"] = global_quantile(score, 1 - cont)

    def _training_metrics(self, model):
        P = model._predict_tensor(self.X)
        m = mm.anomaly_metrics(P[:, -2])
        if self.label is not None and self.label_info.response_domain is not None:
            m["label_AUC"] = mm.binomial_metrics(self.label, P[:, -2], None, self.label_info.response_domain)["AUC"]
        return m


# ================================================================================================
class ExtendedIsolationForestModel(Model):
    algo = "extendedisolationforest"

    def __init__(self, key, params, info):
        super().__init__(key, params, info)
        self.output["model_category"] = "AnomalyDetection"
        self.trees = []

    @property
    def model_category(self):
        return "AnomalyDetection"

    def prediction_names(self):
        return ["anomaly_score", "mean_length"]

    def _path_lengths(self, X):
        Xr = torch.nan_to_num(X.T.double(), nan=0.0)
        N = Xr.shape[0]
        tot = torch.zeros(N, dtype=torch.float64, device=Xr.device)
        for tr in self.trees:
            nrm = torch.as_tensor(tr["normal"], device=Xr.device)          # [nodes, F]
            off = torch.as_tensor(tr["offset"], device=Xr.device)          # [nodes]
            left = torch.as_tensor(tr["left"], device=Xr.device).long()
            right = torch.as_tensor(tr["right"], device=Xr.device).long()
            leafv = torch.as_tensor(tr["value"], device=Xr.device)
            proj = Xr @ nrm.T - off                                         # one GEMM per tree
            node = torch.zeros(N, dtype=torch.long, device=Xr.device)
            for _ in range(int(tr["depth"]) + 1):
                isleaf = left[node] < 0
                go_left = proj.gather(1, node[:, None]).squeeze(1) <= 0
                nxt = torch.where(go_left, left[node], right[node])
                node = torch.where(isleaf, node, nxt)
            tot += leafv[node]
        return tot / max(1, len(self.trees))

    def _predict_tensor(self, X, offset=None):
        h = self._path_lengths(X)
        c = float(c_factor(self.output["sample_size"]))
        score = torch.pow(2.0, -h / c)
        return torch.stack([score.float(), h.float()], 1)

    def to_state(self):
        s = super().to_state()
        s["trees"] = [{k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in t.items()} for t in self.trees]
        return s

    def _restore(self, s):
        super()._restore(s)
        self.trees = [{k: (np.asarray(v) if isinstance(v, list) else v) for k, v in t.items()} for t in s["trees"]]


class ExtendedIsolationForestTrainer:
    def __init__(self, params):
        p = dict(ntrees=100, sample_size=256, extension_level=0, seed=-1)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p

    def fit(self, X, y, w, offset, info, valid=None, model_key=None):
        from .shared_tree import resolve_seed
        p = self.p
        seed = resolve_seed(p["seed"])
        rng = np.random.default_rng(seed & 0xFFFFFFFF)
        F, N = X.shape
        ext = int(p["extension_level"])
        if ext < 0 or ext > F - 1:
            raise ValueError(f"extension_level must be in [0, {F - 1}]")
        # row-sharded: the sample is drawn over GLOBAL row ids (same RNG on every rank); each rank contributes
        # its sampled rows and only those S rows are exchanged (the trees are identical on every rank)
        dist_ = coll.is_dist()
        row0 = coll.row_offset(N) if dist_ else 0
        Ng = int(coll.all_reduce_scalar(N)) if dist_ else N
        S = int(min(p["sample_size"], Ng))
        limit = int(math.ceil(math.log2(max(S, 2))))
        Xh = torch.nan_to_num(X, nan=0.0).T.double()
        model = ExtendedIsolationForestModel(model_key or make_key("eif"), p, info)
        model.device = X.device
        model.output["sample_size"] = S
        for t in range(int(p["ntrees"])):
            gidx = rng.choice(Ng, S, replace=False)
            if dist_:
                mine = np.nonzero((gidx >= row0) & (gidx < row0 + N))[0]
                loc = torch.as_tensor(gidx[mine] - row0, device=X.device)
                part = torch.cat([torch.as_tensor(mine, dtype=torch.float64, device=X.device)[:, None],
                                  Xh.index_select(0, loc)], 1)
                dev_c = coll.comm_device()
                allp = coll.all_gather_cat(part.to(dev_c), 0, bounded=True).cpu().numpy()
                xs = allp[np.argsort(allp[:, 0], kind="stable"), 1:]
            else:
                idx = torch.as_tensor(gidx, device=X.device)
                xs = Xh.index_select(0, idx).cpu().numpy()
            model.trees.append(_grow_eif(xs, limit, ext, rng))
        model.output["ntrees"] = len(model.trees)
        P = model._predict_tensor(X)
        model.output["training_metrics"] = mm.anomaly_metrics(P[:, 0])
        return model


def _grow_eif(xs, limit, ext, rng):
    F = xs.shape[1]
    normal, offset, left, right, value, nrows = [], [], [], [], [], []

    def node(rows, depth):
        i = len(normal)
        normal.append(np.zeros(F)); offset.append(0.0); left.append(-1); right.append(-1); value.append(0.0)
        nrows.append(0)
        n = rows.shape[0]
        if depth >= limit or n <= 1:
            value[i] = depth + float(c_factor(n))
            nrows[i] = n
            return i
        nv = rng.normal(size=F)
        zero = rng.choice(F, F - ext - 1, replace=False) if F - ext - 1 > 0 else []
        nv[list(zero)] = 0.0
        lo, hi = rows.min(0), rows.max(0)
        pt = rng.uniform(lo, hi)
        normal[i] = nv
        offset[i] = float(pt @ nv)
        gl = rows @ nv - offset[i] <= 0
        left[i] = node(rows[gl], depth + 1)
        right[i] = node(rows[~gl], depth + 1)
        return i

    node(xs, 0)
    return dict(normal=np.asarray(normal), offset=np.asarray(offset), left=np.asarray(left, dtype=np.int64),
                right=np.asarray(right, dtype=np.int64), value=np.asarray(value), nrows=np.asarray(nrows, dtype=np.int64),
                depth=limit)
