"""Shared driver for histogram-tree algorithms (reference: ``hex/tree/SharedTree.java``,
``hex/tree/SharedTreeModel.java``).

Responsibilities: bin the training matrix once (``ops.binning``), own the device tree builder
(``ops.tree``), run the per-tree loop with row/column sampling, keep the forest, score periodically
(scoring history, ``ScoreKeeper`` early stopping), and build variable importances from split gains.
Algorithm subclasses provide ``_prepare`` (per-row histogram/leaf statistics), ``_leaf_values`` and
``_update`` (prediction bookkeeping).
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch

from .. import metrics as mm
from ..ops import tree as T
from ..ops.binning import WIDE_MAX_BINS, Binning, apply_binning, fit_binning, sample_rows
from ..ops.forest import Forest, Tree, levels_to_tree
from ..parallel import collectives as coll
from .base import DataInfo, Model, ScoreKeeper, make_key, model_category, variable_importance

SHARED_TREE_DEFAULTS = dict(
    ntrees=50, max_depth=5, min_rows=10.0, nbins=20, nbins_top_level=1024, nbins_cats=1024,
    histogram_type="AUTO", seed=-1, sample_rate=1.0, col_sample_rate_per_tree=1.0,
    min_split_improvement=1e-5, score_each_iteration=False, score_tree_interval=0,
    stopping_rounds=0, stopping_metric="AUTO", stopping_tolerance=1e-3, max_runtime_secs=0.0,
    weights_column=None, offset_column=None, fold_column=None, nfolds=0, ignored_columns=None,
    monotone_constraints=None, checkpoint=None, categorical_encoding="AUTO", max_bins=255,
    calibrate_model=False, build_tree_one_node=False, check_constant_response=True,
)


_CANCEL_EVERY = 4     # trees between cancellation checks of a REST job


def resolve_seed(seed) -> int:
    if seed is None or int(seed) == -1:
        from ..parallel import collectives as coll
        return coll.shared_entropy(1 << 62)
    return int(seed)


def interaction_map(constraints, names):
    """GlobalInteractionConstraints: [F, F] map (row f = union of the constraint sets containing f) and the
    root's allowed features (every column named in some set; unlisted columns are never split on)."""
    F = len(names)
    m = np.zeros((F, F), dtype=np.uint8)
    for group in constraints:
        group = [group] if isinstance(group, str) else list(group)
        idx = []
        for c in group:
            if c not in names:
                raise ValueError(f"interaction_constraints: column {c!r} is not a predictor")
            idx.append(names.index(c))
        for i in idx:
            m[i, idx] = 1
    return m, m.any(1).astype(np.uint8)


class SharedTreeModel(Model):
    def __init__(self, key, params, info):
        super().__init__(key, params, info)
        self.forest: Forest | None = None
        self.binning: Binning | None = None
        self.init_f = 0.0

    def ntrees_built(self):
        return len(self.forest) // max(1, self._trees_per_iter()) if self.forest else 0

    def _trees_per_iter(self):
        return 1

    def _raw(self, X, offset=None, ntrees=None):
        t1 = None if ntrees is None else ntrees * self._trees_per_iter()
        raw = self.forest.predict_raw(X, 0, t1)
        return raw

    def predict_leaf_node_assignment(self, X: torch.Tensor) -> torch.Tensor:
        _, leaves = self.forest.predict_raw(X.to(self.device), return_leaves=True)
        return leaves

    def update_tree_weights(self, frame, weights_column):
        """Recompute every node's weight (``cover``, used by TreeSHAP and the tree API) from the rows of
        ``frame`` weighted by ``weights_column`` (Model.UpdateAuxTreeWeights)."""
        X, _ = frame.model_matrix(self.info, device=self.device)
        w = frame._col(weights_column).as_float().double().to(self.device)
        _, leaves = self.forest.predict_raw(X, return_leaves=True)
        warn = None
        base = 0
        for t, tree in enumerate(self.forest.trees):
            lv = leaves[:, t].long() - base          # flattened node ids -> this tree's ids
            base += tree.n_nodes
            cover = torch.zeros(tree.n_nodes, dtype=torch.float64, device=self.device).index_add_(0, lv, w)
            cover = cover.cpu().numpy()
            for i in range(tree.n_nodes - 1, -1, -1):     # children are appended after their parent
                if tree.feat[i] >= 0:
                    cover[i] = cover[tree.left[i]] + cover[tree.right[i]]
            if warn is None and (cover == 0).any():
                warn = (t, self.forest.tree_class[t])
            tree.cover = cover.astype(tree.cover.dtype if hasattr(tree.cover, "dtype") else np.float64)
        self.forest._flat = {}
        if warn is not None:
            return (f"Some of the updated nodes have zero weights (eg.: tree #{warn[0] + 1}, "
                    f"class #{warn[1] + 1}).")
        return "OK"

    def to_state(self):
        s = super().to_state()
        s["forest"] = dict(trees=[t.to_state() for t in self.forest.trees], tree_class=self.forest.tree_class,
                           K=self.forest.K)
        s["binning"] = self.binning.to_state() if self.binning is not None else None
        s["init_f"] = self.init_f
        return s

    def _restore(self, s):
        super()._restore(s)
        fs = s["forest"]
        self.forest = Forest([Tree.from_state(t) for t in fs["trees"]], fs["tree_class"], fs["K"])
        self.binning = Binning.from_state(s["binning"]) if s.get("binning") else None
        self.init_f = s["init_f"]


class SharedTreeTrainer:
    """Generic per-tree loop. ``X`` is float32 [F, N] column-major on the training device."""

    algo = "sharedtree"
    mode = T.MODE_SE
    model_cls = SharedTreeModel

    def __init__(self, params: dict):
        p = dict(SHARED_TREE_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None or k not in p})
        self.p = p

    # ---- hooks
    def _aux_soa(self) -> bool:
        """The trainer's _prepare returns the row statistics as [4, N] planes (else [N, 4] rows)."""
        return False

    def _num_plane(self) -> int:
        return 2

    def _unit_weights(self) -> bool:
        """Every row weight of the current tree is exactly 1 (no weights, no row sampling)."""
        return False

    def _max_bins(self) -> int:
        """Data bins per numeric feature of the global binning (above 255: wide engine columns)."""
        p = self.p
        max_bins = int(min(255, max(int(p.get("max_bins") or 255), 2)))
        ht_ = str(p.get("histogram_type", "AUTO")).lower().replace("_", "")
        if (self._adaptive_top_level and ht_ in ("auto", "uniformadaptive", "random", "roundrobin", "uniformrobust")
                and "nbins_top_level" in p):
            # DHistogram's root resolution: nbins_top_level (default 1024) bins; above 255 the numeric
            # features are binned wide (several engine columns each, ops/binning.py)
            max_bins = int(min(WIDE_MAX_BINS, max(int(p.get("nbins_top_level") or 1024), int(p.get("nbins") or 20))))
        return max_bins

    def _binning_sample(self) -> int:
        """Rows of the quantile-edge sample (fit_binning); subclasses needing exact edges raise it."""
        return 1 << 20

    def _check_binning(self, b) -> None:
        """Hook: refuse a binning that cannot express the requested split semantics."""

    def _split_params(self) -> T.SplitParams:
        sp = T.SplitParams(min_w=float(self.p["min_rows"]), min_split_improvement=float(self.p["min_split_improvement"]),
                           mode=self.mode)
        ht = str(self.p.get("histogram_type", "AUTO")).lower().replace("_", "")
        if ht not in T.HIST_TYPES:
            raise ValueError(f"histogram_type {self.p.get('histogram_type')!r} is not one of "
                             "AUTO, UniformAdaptive, Random, QuantilesGlobal, RoundRobin, UniformRobust")
        if T.HIST_TYPES[ht] != T.HT_QUANTILES and getattr(self, "binning", None) is not None:
            # DHistogram: nbins_top_level bins at the root, halved per level down to nbins, laid out as the
            # type's split points (uniform / random / SE-guided / per-histogram round robin) over the
            # global bin edges — see _lattice in ops/tree.py
            sp.adapt_nbins = int(self.p.get("nbins") or 20)
            sp.adapt_top = int(self.p.get("nbins_top_level") or 1024)
            sp.edges = self._edge_table()
            sp.hist_type = T.HIST_TYPES[ht]
            sp.vrange = getattr(self, "_vrange", None)
            sp.parent_range = os.environ.get("H2O_HIST_PARENT_RANGE", "1") != "0"
        return sp

    def _value_range_table(self, X):
        """[F_engine, 2] float32: every column's exact (min, max) over ALL rows (all ranks), the range of the
        reference's root histogram (DHistogram.initialHist: the column's rollup min / max)."""
        Xf = X.float()
        nan = torch.isnan(Xf)
        mn = torch.where(nan, torch.full_like(Xf, float("inf")), Xf).amin(1) if Xf.shape[1] else \
            torch.full((Xf.shape[0],), float("inf"), device=Xf.device)
        mx = torch.where(nan, torch.full_like(Xf, float("-inf")), Xf).amax(1) if Xf.shape[1] else \
            torch.full((Xf.shape[0],), float("-inf"), device=Xf.device)
        if coll.is_dist():
            coll.all_reduce_min_(mn)
            coll.all_reduce_max_(mx)
        vr = torch.stack([mn, mx], 1).cpu().numpy().astype(np.float32)
        vm = self.binning.vmap
        return vr if vm is None else vr[np.asarray(vm)]

    def _edge_table(self):
        tab = np.full((self.binning.F, 255), np.inf, dtype=np.float32)
        for f, e in enumerate(self.binning.edges):
            if e is not None and len(e):
                tab[f, :min(len(e), 255)] = e[:255]
        return tab

    def _k_cols(self, F_ok: int) -> int:
        return 0

    def _level_k_cols(self, F: int):
        """k_cols, or its per-level schedule when col_sample_rate_change_per_level != 1
        (DTree.actual_mtries: min(max(1, int(k * change^depth)), F))."""
        k = self._k_cols(F)
        ch = float(self.p.get("col_sample_rate_change_per_level") or 1.0)
        if not 0.0 < ch <= 2.0:
            raise ValueError("col_sample_rate_change_per_level must be > 0 and <= 2.0")
        if ch == 1.0:
            return k
        base = k if k > 0 else F
        D = int(self.p["max_depth"]) if int(self.p["max_depth"]) > 0 else 32
        return [min(max(1, int(base * ch ** d)), F) for d in range(D + 1)]

    def _trees_per_iter(self) -> int:
        return 1

    # H2O's SharedTree binning: nbins_top_level root resolution for the adaptive histogram types
    # (XGBoost bins by its own max_bins instead)
    _adaptive_top_level = True

    # ---- main
    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None) -> SharedTreeModel:
        t_start = time.time()
        p = self.p
        dev = X.device
        F, N = X.shape
        self.dev, self.F, self.N, self.info = dev, F, N, info
        self.seed = resolve_seed(p["seed"])
        self.row0 = coll.row_offset(N)            # global index of this rank's first row (0 unsharded)
        self.category = model_category(info)
        self.w = torch.ones(N, dtype=torch.float32, device=dev) if w is None else w.float().to(dev)
        self.offset = None if offset is None else offset.float().to(dev)
        self.y = y.float().to(dev)
        self.X = X
        # ---- binning (QuantilesGlobal on the whole training set, shared by every tree)
        max_bins = self._max_bins()
        bsample = self._binning_sample()
        if coll.is_dist():
            # every rank must bin identically, and exactly like the single-process run: the quantile
            # sample is drawn on GLOBAL row indices (fit_binning's own rule), each rank contributes the
            # sampled rows it owns, and the edges come from the gathered sample
            n_glob = coll.exclusive_offset(N)[1]
            Xl = sample_rows(X, bsample, self.seed, self.row0, n_glob)
            # (a sample of <= the binning sample size, not the frame: tree_method="exact" samples every row)
            Xs = coll.all_gather_cat(Xl.contiguous(), dim=1, bounded=bsample < (1 << 40))
            self.binning = fit_binning(Xs, info.iscat, info.nlevels, max_bins=max_bins, seed=self.seed,
                                       max_cat_bins=int(p.get("nbins_cats") or 1024), presampled=True)
        else:
            self.binning = fit_binning(X, info.iscat, info.nlevels, max_bins=max_bins, seed=self.seed,
                                       max_cat_bins=int(p.get("nbins_cats") or 1024), sample=bsample)
        self._check_binning(self.binning)
        ht = str(p.get("histogram_type", "AUTO")).lower().replace("_", "")
        self._vrange = self._value_range_table(X) if T.HIST_TYPES.get(ht, 0) != T.HT_QUANTILES else None
        bins = apply_binning(self.binning, X, planar=X.is_cuda)
        mono = None
        if p.get("monotone_constraints"):
            mono = np.zeros(F, dtype=np.int32)
            for k, v in dict(p["monotone_constraints"]).items():
                if k in info.x:
                    mono[info.x.index(k)] = int(v)
        max_depth = int(p["max_depth"]) if int(p["max_depth"]) > 0 else 32
        node_cap = int(p.get("node_cap", 1 << 14))
        bn = self.binning
        self.builder = T.make_builder(bins, bn.F, bn.nbins, bn.iscat, bn.expand(mono), max_depth,
                                      self._split_params(), node_cap=node_cap)
        if bn.vmap is not None:
            self.builder.set_feature_groups(bn.vmap, getattr(bn, "n_low", 0), getattr(bn, "n_mid", 0))
            if bn.cat_groups:
                self.builder.set_cat_groups(bn.gcat())
        if p.get("interaction_constraints"):
            icm, root = interaction_map(p["interaction_constraints"], info.x)
            if bn.vmap is not None:
                icm, root = icm[np.ix_(bn.vmap, bn.vmap)], root[bn.vmap]
            self.builder.set_interaction_constraints(icm, root)
        self.builder = self._wrap_builder(self.builder)
        model = self.model_cls(model_key or make_key(self.algo), p, info)
        model.binning = self.binning
        model.device = dev
        self.model = model
        self._init_model(model)
        K = self._trees_per_iter()
        forest = Forest(n_classes_out=self._forest_k())
        model.forest = forest
        ntrees = int(p["ntrees"])
        interval = int(p.get("score_tree_interval") or 0)
        if p.get("score_each_iteration"):
            interval = 1
        keeper = ScoreKeeper(p.get("stopping_rounds", 0), p.get("stopping_metric", "AUTO"),
                             p.get("stopping_tolerance", 1e-3), self.category)
        need_sync = valid is not None or keeper.k > 0 or interval > 0
        if keeper.k > 0 and interval == 0:
            interval = max(1, min(5, ntrees // 10 or 1))
        gen = torch.Generator(device=dev)
        gen.manual_seed(self.seed & 0x7FFFFFFFFFFF)
        self.gen = gen
        rng = np.random.default_rng(self.seed & 0xFFFFFFFF)
        handles = []
        gains = np.zeros(F, dtype=np.float64)
        start = self._apply_checkpoint(model, forest, gains)
        history = []
        max_rt = float(p.get("max_runtime_secs") or 0)
        self.valid = valid
        built = start
        hprof = os.environ.get("H2O_HOST_PROF") == "1"    # host seconds per phase (launch-bound diagnosis)
        ht = dict(prepare=0.0, build=0.0, update=0.0, drain=0.0, loop=0.0, build_max=0.0)
        # H2O_TREE_GC=0: no cyclic garbage collection inside the tree loop (A/B of host stalls between trees)
        import gc
        gc_was = gc.isenabled()
        if os.environ.get("H2O_TREE_GC", "1") == "0":
            gc.disable()
        for t in range(start, ntrees):
            tl0 = time.perf_counter()
            feat_ok = self.binning.expand(self._tree_feature_mask(rng, F))
            for k in range(K):
                h0 = time.perf_counter()
                aux = self._prepare(t, k)
                h1 = time.perf_counter()
                kw = {}
                am = self._amax_for_build()
                if am is not None:
                    kw["amax_bits"] = am
                if self.dev.type == "cuda":
                    kw["packed"] = self._hist_packed()
                    kw["soa"] = aux.dim() == 2 and aux.shape[0] == 4 and aux.shape[1] == self.N and self._aux_soa()
                    kw["unit"] = self._unit_weights()
                    if kw["soa"]:
                        kw["num_plane"] = self._num_plane()
                    ln = self._leaf_native(t, k)
                    if ln is not None:
                        kw["leaf_native"] = ln
                h = self.builder.build(aux, feat_ok, self._level_k_cols(F), seed=(self.seed * 1000003 + t * 97 + k) & ((1 << 63) - 1),
                                       leaf_fn=lambda ls, t=t, k=k: self._leaf_values(ls, t, k), **kw)
                h2 = time.perf_counter()
                self._update(t, k)
                handles.append((h, k))
                h3 = time.perf_counter()
                if t >= start + 2:                   # skip first-launch module loads / allocations
                    ht["prepare"] += h1 - h0
                    ht["build"] += h2 - h1
                    ht["build_max"] = max(ht["build_max"], h2 - h1)
                    ht["update"] += h3 - h2
            built = t + 1
            if not need_sync:
                h0 = time.perf_counter()
                self._drain(handles, forest, gains, ready_only=True)   # overlap host decode with GPU work
                if t >= start + 2:
                    ht["drain"] += time.perf_counter() - h0
            if t >= start + 2:
                ht["loop"] += time.perf_counter() - tl0
            if need_sync:
                self._drain(handles, forest, gains)
                if interval and (built % interval == 0 or built == ntrees):
                    ev = self._score_event(model, built, t_start)
                    history.append(ev)
                    mref = ev.get("_valid") or ev.get("_train")
                    if mref is not None and keeper.add(mref):
                        break
            ck_dir = p.get("in_training_checkpoints_dir")
            if ck_dir and built % max(1, int(p.get("in_training_checkpoints_tree_interval") or 1)) == 0:
                self._drain(handles, forest, gains)       # snapshot of the model so far, resumable via checkpoint=
                self._save_in_training(model, built, ck_dir)
            if max_rt > 0 and coll.agree(time.time() - t_start > max_rt):
                break
            job = getattr(self, "job", None)
            if job is not None:                  # SharedTree.doScoringAndSaveModel: progress + stop_requested per tree
                job.worked = job.work * built / max(ntrees, 1)
                if (built - start) % _CANCEL_EVERY == 0:
                    job.check_cancelled()        # (REST cloud: a collective; every rank checks at the same trees)
        self._drain(handles, forest, gains)
        if gc_was:
            gc.enable()
        if hprof and built > start + 2:
            n = (built - start - 2) * K
            print("[host-prof] us/tree " + " ".join(f"{k}={v / (1 if k.endswith('_max') else n) * 1e6:.1f}"
                                                    for k, v in ht.items()), flush=True)
        if need_sync and (not history or history[-1]["number_of_trees"] != built):
            history.append(self._score_event(model, built, t_start))
        self._finish(model, built)
        model.output["scoring_history"] = [{k: v for k, v in e.items() if not k.startswith("_")} for e in history]
        model.output["variable_importances"] = variable_importance(info.x, gains)
        model.output["ntrees"] = built
        model.output["model_summary"] = self._summary(forest, built)
        model.output["training_metrics"] = self._training_metrics(model)
        if valid is not None:
            Xv, yv, wv, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv, ov)
        if not model.output["scoring_history"]:
            # SharedTree always scores the final model (doScoringAndSaveModel(finalScoring=true)): one history
            # row from the final metrics, no extra pass
            ev = dict(timestamp=time.time(), duration=time.time() - t_start, number_of_trees=built)
            for src, pre in (("training_metrics", "training_"), ("validation_metrics", "validation_")):
                mt = model.output.get(src)
                for k in ("RMSE", "logloss", "AUC", "pr_auc", "mean_per_class_error", "mae", "mean_residual_deviance"):
                    if mt is not None and hasattr(mt, "get") and mt.get(k) is not None:
                        ev[pre + k.lower()] = mt[k]
            model.output["scoring_history"] = [ev]
        model.output["start_time"] = int(t_start * 1000)
        model.output["run_time_ms"] = int((time.time() - t_start) * 1000)
        model.output["end_time"] = model.output["start_time"] + model.output["run_time_ms"]
        return model

    def _forest_k(self):
        return self._trees_per_iter()

    def _tree_feature_mask(self, rng, F):
        r = float(self.p.get("col_sample_rate_per_tree", 1.0))
        if r >= 1.0:
            return None
        k = max(1, int(math.floor(F * r + 0.5)))
        ok = np.zeros(F, dtype=np.int32)
        ok[rng.choice(F, size=k, replace=False)] = 1
        return torch.from_numpy(ok).to(self.dev)

    def _drain(self, handles, forest, gains, ready_only=False):
        """Move built trees (in build order) from the builder into the forest; ``handles`` is consumed
        in place. ``ready_only`` takes only trees whose device->host snapshot has already landed."""
        if not handles:
            return
        levels = self.builder.pop_levels(ready_only=ready_only)
        done = handles[:len(levels)]
        del handles[:len(levels)]
        for (h, k), tl in zip(done, levels):
            forest.add_levels(tl, self.binning, k)     # flattened lazily (Forest.trees)
            vm = self.binning.vmap
            for d in tl.decs:
                fe = d["feat"]
                m = fe >= 0
                np.add.at(gains, fe[m] if vm is None else vm[fe[m]], np.maximum(d["gain"][m], 0.0))

    def _summary(self, forest: Forest, built):
        dl = forest.depth_leaves()
        depths = [d for d, _ in dl] or [0]
        leaves = [n for _, n in dl] or [0]
        return dict(number_of_trees=built, number_of_internal_trees=len(forest), min_depth=int(min(depths)),
                    max_depth=int(max(depths)), mean_depth=float(np.mean(depths)), min_leaves=int(min(leaves)),
                    max_leaves=int(max(leaves)), mean_leaves=float(np.mean(leaves)))

    def _score_event(self, model, built, t_start):
        ev = dict(timestamp=time.time(), duration=time.time() - t_start, number_of_trees=built)
        tm = self._training_metrics(model)
        ev["_train"] = tm
        if tm is not None:
            for k in ("RMSE", "logloss", "AUC", "pr_auc", "mean_per_class_error", "mae", "mean_residual_deviance"):
                if k in tm:
                    ev["training_" + k.lower()] = tm[k]
        if self.valid is not None:
            Xv, yv, wv, ov = self.valid
            vm = model.metrics_for(Xv, yv, wv, ov)
            ev["_valid"] = vm
            for k in ("RMSE", "logloss", "AUC", "pr_auc", "mean_per_class_error", "mae", "mean_residual_deviance"):
                if vm is not None and k in vm:
                    ev["validation_" + k.lower()] = vm[k]
        return ev

    # ---- checkpoint / resume (hex/tree/SharedTree.java checkpoint handling)
    def _apply_checkpoint(self, model, forest, gains) -> int:
        """Continue from ``checkpoint`` (model or key): copy its trees, restore the training margin, return
        the number of iterations already built. ntrees must exceed the checkpoint's."""
        ck = self.p.get("checkpoint")
        if not ck:
            return 0
        from ..core import dkv
        prev = dkv.get(ck) if isinstance(ck, str) else getattr(ck, "_model", ck)
        if prev is None or getattr(prev, "forest", None) is None:
            raise ValueError(f"checkpoint {ck} is not a tree model of this kind")
        if prev.info.x != self.info.x:
            raise ValueError("checkpoint model was trained on different predictors")
        K = self._trees_per_iter()
        for t, c in zip(prev.forest.trees, prev.forest.tree_class):
            forest.add(t, c)
            m = t.feat >= 0
            np.add.at(gains, t.feat[m], np.maximum(t.gain[m], 0.0))
        done = len(prev.forest.trees) // max(K, 1)
        if done >= int(self.p["ntrees"]):
            raise ValueError(f"ntrees ({self.p['ntrees']}) must be larger than the checkpoint's ({done})")
        self._restore_margin(model, prev)
        return done

    def _save_in_training(self, model, built, ck_dir):
        import copy
        from ..persist import save_model
        snap = copy.copy(model)
        snap.key = f"{model.key}.{built}"
        snap.output = dict(model.output, ntrees=built)
        self._finish_snapshot(snap)
        save_model(snap, ck_dir, force=True)

    def _finish_snapshot(self, snap):
        pass

    def _restore_margin(self, model, prev):
        if hasattr(self, "f"):
            raw = prev.forest.predict_raw(self.X)
            model.init_f = prev.init_f
            init = torch.as_tensor(prev.init_f, dtype=torch.float32, device=self.dev).reshape(1, -1)
            self.f.copy_(raw + init + (self.offset[:, None] if self.offset is not None else 0))

    # defaults, overridden
    def _wrap_builder(self, builder):
        return builder

    def _amax_for_build(self):
        return None

    def _leaf_native(self, t, k):
        """Optional (log_link, scale, kclamp, max_abs) for device-side closed-form leaf values."""
        return None

    def _hist_packed(self) -> bool:
        """True when every histogram row weight (aux.x) is a 0/1 (or small integer) count."""
        return False

    def _init_model(self, model):
        pass

    def _finish(self, model, built):
        pass

    def _training_metrics(self, model):
        return None

    def _prepare(self, t, k):
        raise NotImplementedError

    def _leaf_values(self, leafsum, t, k):
        raise NotImplementedError

    def _update(self, t, k):
        pass

    def _row_sample(self, rate: float, t: int):
        """Bernoulli(rate) row sample keyed by (seed, tree, GLOBAL row index): identical however the
        rows are sharded."""
        spc = self.p.get("sample_rate_per_class")
        if spc:
            # sample_rate_per_class: one rate per response class (SharedTree.java sample_rate_per_class)
            if self.info.response_domain is None or len(spc) != len(self.info.response_domain):
                raise ValueError("sample_rate_per_class needs one rate per response class")
            rates = torch.tensor([float(v) for v in spc], dtype=torch.float64, device=self.dev)
            cls = torch.nan_to_num(self.y, nan=0).long().clamp(0, len(spc) - 1)
            m = coll.row_uniform(self.seed, 1000 + t, self.row0, self.N, self.dev) < rates[cls]
            return self.w * m.float()
        if rate >= 1.0:
            return self.w
        m = coll.row_uniform(self.seed, 1000 + t, self.row0, self.N, self.dev) < rate
        return self.w * m.float()
