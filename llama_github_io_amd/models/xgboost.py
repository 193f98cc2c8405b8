"""XGBoost-compatible booster (reference: ``h2o-extensions/xgboost/src/main/java/hex/tree/xgboost/
XGBoost.java``, ``XGBoostModel.java`` parameter mapping, native libxgboost ``hist`` updater).

The H2O extension calls libxgboost; here the same model is grown by the framework's own device
histogram engine in Newton mode: per-row gradient/hessian of the objective, split gain
``G_L²/(H_L+λ) + G_R²/(H_R+λ) - G²/(H+λ)`` with L1 soft-thresholding (``reg_alpha``) and
``gamma`` (min split loss), ``min_child_weight`` on hessian sums, leaf weight ``-G/(H+λ)`` times
``eta`` (clamped by ``max_delta_step``). ``booster='dart'`` drops trees per iteration
(``rate_drop``, ``skip_drop``, normalize_type tree); ``booster='gblinear'`` runs shotgun coordinate
descent on the expanded design matrix.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from .. import metrics as mm
from ..ops import tree as T
from ..ops.binning import WIDE_MAX_BINS
from .base import Model
from .datainfo import Expander
from .shared_tree import SharedTreeModel, SharedTreeTrainer

XGB_DEFAULTS = dict(ntrees=50, max_depth=6, min_rows=1.0, min_child_weight=None, learn_rate=0.3, eta=None,
                    sample_rate=1.0, subsample=None, col_sample_rate=1.0, colsample_bylevel=None,
                    col_sample_rate_per_tree=1.0, colsample_bytree=None, reg_lambda=1.0, reg_alpha=0.0, gamma=0.0,
                    min_split_improvement=None, max_bins=256, max_delta_step=0.0, max_abs_leafnode_pred=None,
                    booster="gbtree", tree_method="auto", grow_policy="depthwise", distribution="AUTO",
                    tweedie_power=1.5, rate_drop=0.0, skip_drop=0.0, one_drop=False, normalize_type="tree",
                    sample_type="uniform", scale_pos_weight=1.0, max_leaves=0, calibrate_model=False)


def _alias(p):
    for a, b in (("eta", "learn_rate"), ("subsample", "sample_rate"), ("colsample_bylevel", "col_sample_rate"),
                 ("colsample_bytree", "col_sample_rate_per_tree"), ("min_child_weight", "min_rows"),
                 ("min_split_improvement", "gamma"), ("max_abs_leafnode_pred", "max_delta_step")):
        if p.get(a) is not None:
            p[b] = p[a]
    return p


def grad_hess(obj, y, f, k=None, probs=None, tweedie_power=1.5, max_delta_step=0.7):
    if obj == "gaussian":
        return f - y, torch.ones_like(f)
    if obj == "bernoulli":
        p = torch.sigmoid(f)
        return p - y, (p * (1 - p)).clamp(min=1e-16)
    if obj == "multinomial":
        p = probs[:, k]
        return p - y, (2 * p * (1 - p)).clamp(min=1e-16)
    if obj == "poisson":
        ef = torch.exp(f)
        return ef - y, torch.exp(f + max_delta_step)
    if obj == "gamma":
        e = y * torch.exp(-f)
        return 1 - e, e
    if obj == "tweedie":
        r = tweedie_power
        a, b = torch.exp((1 - r) * f), torch.exp((2 - r) * f)
        return -y * a + b, -y * (1 - r) * a + (2 - r) * b
    raise ValueError(f"XGBoost objective for distribution {obj} not supported")


class XGBoostModel(SharedTreeModel):
    algo = "xgboost"

    def _trees_per_iter(self):
        return self.forest.K if self.forest is not None else 1

    def _predict_tensor(self, X, offset=None):
        if self.output.get("booster") == "gblinear":
            Z = self.expander.transform(X)
            f = Z @ self.beta.to(Z.device).T + self.bias.to(Z.device)
        else:
            f = self.forest.predict_raw(X) + torch.as_tensor(self.init_f, dtype=torch.float32, device=X.device)
        if offset is not None:
            f = f + offset.float()[:, None]
        d = self.output["distribution"]
        if d == "bernoulli":
            p1 = torch.sigmoid(f[:, 0])
            return torch.stack([1 - p1, p1], 1)
        if d == "multinomial":
            return torch.softmax(f, 1)
        if d in ("poisson", "gamma", "tweedie"):
            return torch.exp(f[:, 0])
        return f[:, 0]

    def to_state(self):
        s = super().to_state() if self.forest is not None else Model.to_state(self)
        if self.output.get("booster") == "gblinear":
            s["beta"] = self.beta.cpu().tolist()
            s["bias"] = self.bias.cpu().tolist()
            s["expander"] = self.expander.to_state()
        return s

    def _restore(self, s):
        if "forest" in s:
            super()._restore(s)
        else:
            Model._restore(self, s)
        if "beta" in s:
            self.beta = torch.tensor(s["beta"])
            self.bias = torch.tensor(s["bias"])
            self.expander = Expander.from_state(self.info, s["expander"])


class XGBoostTrainer(SharedTreeTrainer):
    algo = "xgboost"
    mode = T.MODE_NEWTON
    model_cls = XGBoostModel

    def __init__(self, params):
        p = dict(XGB_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None or k not in p})
        p = _alias(p)
        super().__init__(p)

    # xgboost's hist bins come from max_bins alone (H2O's nbins_top_level is not an XGBoost parameter)
    _adaptive_top_level = False

    def _split_params(self):
        p = self.p
        return T.SplitParams(min_w=float(p["min_rows"]), min_split_improvement=0.0, lam=float(p["reg_lambda"]),
                             alpha=float(p["reg_alpha"]), gamma=float(p["gamma"]), mode=T.MODE_NEWTON)

    def fit(self, X, y, w, offset, info, valid=None, model_key=None):
        d = str(self.p.get("distribution") or "AUTO").lower()
        if d == "auto":
            d = "gaussian" if info.response_domain is None else ("bernoulli" if len(info.response_domain) == 2 else "multinomial")
        self.obj = d
        self.K = len(info.response_domain) if d == "multinomial" else 1
        if str(self.p.get("booster")).lower() == "gblinear":
            return self._fit_linear(X, y, w, offset, info, valid, model_key)
        tm = str(self.p.get("tree_method") or "auto").lower()
        if tm not in ("auto", "exact", "approx", "hist"):
            raise ValueError(f"tree_method must be one of auto, exact, approx, hist; got {tm!r}")
        self.tree_method = tm
        # hist / approx / auto: histogram splits on global quantile bins (approx's per-tree sketch is the
        # same cut set up to resampling); exact: every distinct value of every numeric column is a split
        # candidate, i.e. one bin per distinct value of the WHOLE column
        if tm != "exact":
            self.p["max_bins"] = min(int(self.p.get("max_bins", 256)), 255)
        return super().fit(X, y, w, offset, info, valid, model_key)

    def _max_bins(self):
        # exact: one bin per distinct value, up to the wide-column capacity (4 engine columns, 1016 edges)
        if getattr(self, "tree_method", "auto") == "exact":
            return WIDE_MAX_BINS
        return super()._max_bins()

    def _binning_sample(self):
        if getattr(self, "tree_method", "auto") == "exact":
            return 1 << 62           # edges from every row, not a sample
        return super()._binning_sample()

    def _check_binning(self, b):
        if getattr(self, "tree_method", "auto") != "exact":
            return
        # exact greedy splits are the histogram splits when no bin merges two distinct values: at most 1016
        # distinct values per numeric column (254 per engine column, wide columns beyond, ops/binning.py)
        Xn = self.X
        for j in range(b.F):
            if b.iscat[j] or (j > 0 and b.orig(j) == b.orig(j - 1)):
                continue
            f = b.orig(j)
            col = Xn[f][~torch.isnan(Xn[f])]
            nd = int(torch.unique(col).numel()) if col.numel() else 0
            if nd > WIDE_MAX_BINS:
                raise ValueError(f"tree_method='exact': column {self.info.x[f]!r} has {nd} distinct values; the "
                                 f"exact split search of this engine handles at most {WIDE_MAX_BINS} per column "
                                 "(use 'hist')")

    def _trees_per_iter(self):
        return self.K

    def _wrap_builder(self, builder):
        gp = str(self.p.get("grow_policy") or "depthwise").lower()
        if gp not in ("depthwise", "lossguide"):
            raise ValueError(f"grow_policy must be depthwise or lossguide, got {gp!r}")
        L = int(self.p.get("max_leaves") or 0)
        if L < 0:
            raise ValueError("max_leaves must be >= 0")
        # xgboost's hist driver honours max_leaves under both policies (depthwise: shallowest nodes
        # first; lossguide: largest loss change first). Without a leaf limit both expand every
        # positive-gain node up to max_depth, i.e. the level-wise tree itself
        return T.BestFirstBuilder(builder, L, by_depth=gp == "depthwise") if L > 0 else builder

    def _k_cols(self, F):
        # colsample_bylevel (H2O col_sample_rate) x colsample_bynode: the engine draws a fresh column sample
        # for every node (XGBoost samples bynode from the level's sample: the expected size is the product)
        r = float(self.p.get("col_sample_rate", 1.0)) * float(self.p.get("colsample_bynode") or 1.0)
        return 0 if r >= 1.0 else max(1, int(math.floor(F * r + 0.5)))

    def _base_score(self):
        if self.obj in ("bernoulli", "multinomial"):
            return 0.0
        if self.obj in ("poisson", "gamma", "tweedie"):
            return math.log(0.5)
        return 0.5

    def _init_model(self, model):
        N, K, dev = self.N, self.K, self.dev
        model.output["distribution"] = self.obj
        model.output["booster"] = str(self.p.get("booster", "gbtree")).lower()
        init = np.full(K, self._base_score())
        model.init_f = init.tolist()
        self.f = torch.tensor(init, dtype=torch.float32, device=dev).repeat(N, 1).contiguous()
        if self.offset is not None:
            self.f += self.offset[:, None]
        if K > 1:
            self.yk = torch.nn.functional.one_hot(torch.nan_to_num(self.y, nan=0).long(), K).float()
        self.yok = ~torch.isnan(self.y)
        # [4, N] planes on the device (the histogram passes stream only the hessian / gradient planes)
        self.aux = (torch.empty(4, N, dtype=torch.float32, device=dev) if dev.type == "cuda"
                    else torch.empty(N, 4, dtype=torch.float32, device=dev))
        self.dart = model.output["booster"] == "dart"
        self.tree_rows = []   # dart: per tree (k, vals, leaf)
        self.tree_w = []
        spw = float(self.p.get("scale_pos_weight", 1.0))
        if self.obj == "bernoulli" and spw != 1.0:
            self.w = torch.where(self.y == 1, self.w * spw, self.w)

    def _dart_drop(self, t):
        p = self.p
        self.dropped = []
        if not self.tree_rows or float(p.get("rate_drop", 0)) <= 0:
            return
        rng = np.random.default_rng((self.seed + 31 * t) & 0xFFFFFFFF)
        if rng.random() < float(p.get("skip_drop", 0)):
            return
        n_iter = len(self.tree_rows) // self.K
        tw = np.asarray(self.tree_w[:n_iter], dtype=np.float64)
        weighted = str(p.get("sample_type") or "uniform").lower() == "weighted"
        # gbm::Dart::DropTrees: uniform, or in proportion to the trees' current weights
        prob = float(p["rate_drop"]) * n_iter * tw / tw.sum() if weighted else float(p["rate_drop"])
        drop = np.nonzero(rng.random(n_iter) < prob)[0].tolist()
        if not drop and p.get("one_drop"):
            drop = [int(rng.choice(n_iter, p=tw / tw.sum()))] if weighted else [int(rng.integers(n_iter))]
        self.dropped = drop
        for it in drop:
            for k in range(self.K):
                kk, vals, leaf = self.tree_rows[it * self.K + k]
                self.f[:, kk] -= self.tree_w[it] * vals[leaf.long()]

    # ---- fused HIP row step (gbm_kernels.hip k_gbm_step, D_XGB_LOGISTIC / D_GAUSSIAN): the previous tree's
    # margin update, the gradient / hessian planes and the fixed-point scale maxima in ONE pass over the rows
    # (the torch path is ~10 elementwise kernels over N rows per tree); leaves by k_leaf_values
    _FUSED_OBJ = {"bernoulli": 10, "gaussian": 0}

    def _hist_packed(self):
        # one LDS atomic per (row, feature): squared error rows weigh exactly 1 (count|wY word); logistic hessians
        # go in the 32/32 fixed-point FPACK word (2 = tree.build packed mode; H2O_XGB_FPACK=0: two 64-bit atomics)
        if not self._fused():
            return False
        if self.obj == "gaussian":
            return True
        return 2 if os.environ.get("H2O_XGB_FPACK", "1") != "0" else False

    def _num_plane(self):
        # both fused objectives store num == w * z only in plane 1 (h2o_gbm_step skip bit 2)
        return 1 if self._fused() else 2

    def _fused(self):
        if getattr(self, "_fused_ok", None) is None:
            self._fused_ok = bool(
                self.dev.type == "cuda" and self.K == 1 and self.obj in self._FUSED_OBJ and not self.dart
                and str(self.p.get("booster", "gbtree")).lower() != "gblinear"
                and float(self.p.get("sample_rate", 1.0)) >= 1.0 and bool(self.yok.all())
                and bool((self.w == 1).all()))
        return self._fused_ok

    def _amax_for_build(self):
        if not self._fused():
            return None
        if not hasattr(self, "_amax"):
            self._amax = torch.zeros(4 * T.AMAX_SHARDS, dtype=torch.int32, device=self.dev)
        return self._amax

    def _leaf_native(self, t, k):
        if not self._fused():
            return None
        p = self.p
        self._vals = self.builder.leaf_values_view()
        lr = float(p["learn_rate"])
        mds = float(p.get("max_delta_step") or 0)
        return (0, lr, 0.0, lr * mds if mds > 0 else float("inf"), float(p["reg_lambda"]), float(p["reg_alpha"]))

    def _flush_pending(self):
        pend = getattr(self, "_pending", None)
        if pend is not None:
            from ..ops import _native as nat
            vals, leaf = pend
            nat.call("h2o_add_leaf", self.N, self.f.data_ptr(), 1, vals.data_ptr(), leaf.data_ptr(), nat.stream_ptr(self.dev))
            self._pending = None

    def _prepare(self, t, k):
        if self._fused():
            from ..ops import _native as nat
            self._amax_for_build()
            pv, pl = self._pending if getattr(self, "_pending", None) is not None else (None, None)
            nat.call("h2o_gbm_step", self.N, self.row0, self._FUSED_OBJ[self.obj], self.y.data_ptr(), 0,
                     self.f.data_ptr(), 0 if pv is None else pv.data_ptr(), 0 if pl is None else pl.data_ptr(),
                     1.0, 0, 0.0, self.aux.data_ptr(), self._amax.data_ptr(), 4, nat.stream_ptr(self.dev))
            self._pending = None
            return self.aux
        if k == 0:
            if self.dart:
                self._dart_drop(t)
            ws = self._row_sample(float(self.p["sample_rate"]), t)
            self.ws = torch.where(self.yok, ws, torch.zeros_like(ws))
            if self.K > 1:
                self.probs = torch.softmax(self.f, 1)
        y = torch.nan_to_num(self.yk[:, k] if self.K > 1 else self.y, nan=0.0)
        g, h = grad_hess(self.obj, y, self.f[:, k], k, getattr(self, "probs", None), float(self.p["tweedie_power"]))
        a = self.aux
        if self._aux_soa():
            torch.mul(self.ws, h, out=a[0])
            torch.mul(self.ws, g, out=a[1]).neg_()
            a[2].copy_(a[1])
            a[3].copy_(a[0])
        else:
            a[:, 0] = self.ws * h
            a[:, 1] = -self.ws * g
            a[:, 2] = -self.ws * g
            a[:, 3] = self.ws * h
        return a

    def _aux_soa(self):
        return self.dev.type == "cuda"

    def _leaf_values(self, ls, t, k):
        p = self.p
        G, H = ls[:, 0], ls[:, 1]
        al = float(p["reg_alpha"])
        if al > 0:
            G = torch.sign(G) * (G.abs() - al).clamp(min=0)
        v = G / (H + float(p["reg_lambda"])).clamp(min=1e-300)
        v = torch.where(H > 0, v, torch.zeros_like(v))
        mds = float(p.get("max_delta_step") or 0)
        if mds > 0:
            v = v.clamp(-mds, mds)
        self._vals = (float(p["learn_rate"]) * v).float()
        return self._vals

    def _update(self, t, k):
        leaf = self.builder.leaf_of_row
        if self._fused():
            self._pending = (self._vals, leaf)   # applied by the next fused step (or _flush_pending)
            return
        if self.dart:
            # gbm::Dart::NormalizeTrees (leaf values already carry eta; lr = eta / trees per iteration):
            #   tree:   new trees weigh 1 / (k + lr), dropped trees are scaled by k / (k + lr)
            #   forest: new trees weigh 1 / (1 + lr), dropped trees are scaled by 1 / (1 + lr)
            nd = len(self.dropped)
            lr = float(self.p["learn_rate"]) / self.K
            forest = str(self.p.get("normalize_type") or "tree").lower() == "forest"
            if not nd:
                wnew, scale = 1.0, 1.0
            elif forest:
                wnew = scale = 1.0 / (1.0 + lr)
            else:
                wnew, scale = 1.0 / (nd + lr), nd / (nd + lr)
            self.tree_rows.append((k, self._vals.clone(), leaf.clone()))
            if k == 0:
                self.tree_w.append(wnew)
            self.f[:, k] += wnew * self._vals[leaf.long()]
            if k == self.K - 1 and nd:
                for it in self.dropped:
                    for kk in range(self.K):
                        _, vals, lf = self.tree_rows[it * self.K + kk]
                        self.f[:, kk] += self.tree_w[it] * scale * vals[lf.long()]
                    self.tree_w[it] *= scale
        else:
            self.f[:, k] += self._vals[leaf.long()]

    def _finish(self, model, built):
        self._flush_pending()
        if self.dart:
            # fold the dart weights into the stored leaf values
            for i, tree in enumerate(model.forest.trees):
                it = i // self.K
                if it < len(self.tree_w):
                    tree.value = (tree.value * self.tree_w[it]).astype(np.float32)
            model.forest._flat.clear()

    def _training_metrics(self, model):
        self._flush_pending()
        f, y, w = self.f, self.y, self.w
        if self.obj == "multinomial":
            return mm.multinomial_metrics(y, torch.softmax(f, 1), w, self.info.response_domain)
        if self.obj == "bernoulli":
            return mm.binomial_metrics(y, torch.sigmoid(f[:, 0]), w, self.info.response_domain)
        pred = torch.exp(f[:, 0]) if self.obj in ("poisson", "gamma", "tweedie") else f[:, 0]
        return mm.regression_metrics(y, pred, w)

    # ---- gblinear: elastic-net shotgun coordinate descent on Newton statistics
    def _fit_linear(self, X, y, w, offset, info, valid, model_key):
        from .base import make_key
        dev = X.device
        N = X.shape[1]
        w = torch.ones(N, device=dev) if w is None else w.float()
        y = y.float()
        ok = ~torch.isnan(y)
        w = torch.where(ok, w, torch.zeros_like(w))
        y = torch.nan_to_num(y, nan=0.0)
        ex = Expander(info, standardize=False, use_all_factor_levels=True).fit(X, w)
        Z = ex.transform(X)
        P = Z.shape[1]
        K = self.K
        beta = torch.zeros(K, P, device=dev)
        bias = torch.full((K,), self._base_score(), device=dev)
        lam, al, eta = float(self.p["reg_lambda"]), float(self.p["reg_alpha"]), float(self.p["learn_rate"])
        yk = torch.nn.functional.one_hot(y.long(), K).float() if K > 1 else None
        for t in range(int(self.p["ntrees"])):
            f = Z @ beta.T + bias
            if offset is not None:
                f = f + offset[:, None]
            probs = torch.softmax(f, 1) if K > 1 else None
            for k in range(K):
                g, h = grad_hess(self.obj, yk[:, k] if K > 1 else y, f[:, k], k, probs, float(self.p["tweedie_power"]))
                g, h = g * w, h * w
                bias[k] -= eta * g.sum() / h.sum().clamp(min=1e-12)
                G = Z.T @ g + lam * beta[k]
                H = (Z * Z).T @ h + lam
                bk = beta[k]
                num = G - H * bk
                step = torch.where(bk - G / H > 0, -(G + al) / H, -(G - al) / H)
                step = torch.maximum(step, -bk) if al > 0 else step
                step = torch.where((bk == 0) & ((G.abs() <= al)), torch.zeros_like(step), step)
                beta[k] = bk + eta * step
                del num
        model = XGBoostModel(model_key or make_key("xgboost"), self.p, info)
        model.device = dev
        model.output["distribution"] = self.obj
        model.output["booster"] = "gblinear"
        model.beta, model.bias, model.expander = beta, bias, ex
        model.output["coefficients"] = {n: beta[:, i].tolist() for i, n in enumerate(ex.names)}
        model.output["training_metrics"] = model.metrics_for(X, y, w, offset) if info.response else None
        if valid is not None:
            Xv, yv, wv, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv, ov)
        return model
