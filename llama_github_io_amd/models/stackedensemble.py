"""Stacked Ensemble (reference: ``hex/ensemble/StackedEnsemble.java``, ``StackedEnsembleModel.java``,
``Metalearners.java``).

Base models must share the fold assignment and keep their cross-validation holdout predictions;
the level-one frame is [holdout predictions of each base model] (p1 for binomial, all class
probabilities for multinomial, the prediction for regression) and the metalearner (default GLM
with non-negative weights, or GBM/DRF/DeepLearning/naive-bayes-free choice) is trained on it.
Scoring stacks the base models' predictions on the new data and applies the metalearner.
"""
from __future__ import annotations

import numpy as np
import torch

from ..core import dkv
from .base import DataInfo, Model, make_key


def builder_train(algo, params, x, y, frame, model_id):
    from .builder import train
    return train(algo, params, x, y, frame, None, None, model_id)


def _level_one(models, X, offset, category):
    cols = []
    for m in models:
        P = m.score_tensor(X, offset)
        if category == "Binomial":
            cols.append(P[:, 1:2].float())
        elif category == "Multinomial":
            cols.append(P.float())
        else:
            cols.append(P.reshape(-1, 1).float())
    return torch.cat(cols, 1).T.contiguous()   # [F', N] like every trainer input


class StackedEnsembleModel(Model):
    algo = "stackedensemble"

    def __init__(self, key, params, info):
        super().__init__(key, params, info)
        self.base_keys = []
        self.meta = None

    def base_models(self):
        return [dkv.get(k) for k in self.base_keys]

    def _predict_tensor(self, X, offset=None):
        L1 = _level_one(self.base_models(), X, offset, self.model_category)
        if self.output.get("metalearner_transform") == "logit":
            L1 = _logit(L1)
        return self.meta.score_tensor(L1)

    def metalearner(self):
        return self.meta

    def to_state(self):
        s = super().to_state()
        s["base_models"] = [m.to_state() | {"__class__": type(m).__module__ + ":" + type(m).__name__}
                            for m in self.base_models()]
        s["meta"] = self.meta.to_state() | {"__class__": type(self.meta).__module__ + ":" + type(self.meta).__name__}
        return s

    def _restore(self, s):
        super()._restore(s)
        from ..persist import _from_state
        bms = [_from_state(dict(b)) for b in s["base_models"]]
        for b in bms:
            dkv.put(b.key, b)
        self.base_keys = [b.key for b in bms]
        self.meta = _from_state(dict(s["meta"]))


def _logit(P):
    p = P.double().clamp(1e-15, 1 - 1e-15)
    return torch.log(p / (1 - p)).float()


class StackedEnsembleTrainer:
    def __init__(self, params):
        p = dict(base_models=[], metalearner_algorithm="AUTO", metalearner_params=None, metalearner_nfolds=0,
                 metalearner_fold_assignment="AUTO", metalearner_fold_column=None, metalearner_transform="NONE",
                 keep_levelone_frame=False, seed=-1, blending_frame=None)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from .builder import REGISTRY  # noqa: F401
        from .base import model_category
        self._train_y, self._train_w = y, w
        keys = []
        for b in self.p["base_models"]:
            if isinstance(b, str):
                keys.append(b)
            else:
                k = getattr(b, "model_id", None) or getattr(b, "key", None)
                if k is None and hasattr(b, "_model"):
                    k = b._model.key
                keys.append(k)
        models = []
        for k in keys:
            v = dkv.get(k)
            if v is None:
                continue
            if hasattr(v, "models") and hasattr(v, "grid_id"):   # a Grid: take all its models
                models += list(v.models)
            else:
                models.append(v)
        if not models:
            raise ValueError("StackedEnsemble needs base_models")
        cat = model_category(info)
        from ..parallel import collectives as coll, dframe
        blend = self.p.get("blending_frame")
        if blend is not None:
            # blending mode (StackedEnsemble.java StackedEnsembleBlendingDriver): the level-one frame is the
            # base models' predictions on the blending frame, whose response trains the metalearner; the base
            # models need no cross-validation
            if isinstance(blend, str):
                blend = dkv.get(blend)
            if blend is None or not hasattr(blend, "model_matrix"):
                raise ValueError("blending_frame must be a frame (or a frame key)")
            cols_ = []
            for m in models:
                fr = m._adapt(blend)
                Xb, ob = fr.model_matrix(m.info, device=X.device)
                cols_.append(_level_one([m], Xb, ob, cat))
            L1 = torch.cat(cols_, 0).contiguous()
            y = blend.response_tensor(info, device=X.device)
            w = blend.weights_tensor(info, device=X.device)
            return self._finish(models, L1, y, w, X, info, cat, valid, model_key, ytrain=(X, None, None, offset),
                                l1_sharded=getattr(blend, "_shard", None) is not None)
        holds = []
        for m in models:
            h = getattr(m, "cv_holdout", None)
            if h is None:
                raise ValueError(f"base model {m.key} has no cross-validation holdout predictions "
                                 "(train it with nfolds>1 and keep_cross_validation_predictions=True)")
            if getattr(m, "cv_holdout_sharded", False) and not coll.is_dist():
                h = dframe.gather_tensor(h.cpu() if coll.comm_device().type == "cpu" else h).to(X.device)
            if cat == "Binomial":
                holds.append(h[:, 1:2].float())
            elif cat == "Multinomial":
                holds.append(h.float())
            else:
                holds.append(h.reshape(-1, 1).float())
        L1 = torch.cat(holds, 1).T.contiguous().to(X.device)
        return self._finish(models, L1, y, w, X, info, cat, valid, model_key, ytrain=(X, y, w, offset),
                            l1_sharded=coll.is_dist())

    def _finish(self, models, L1, y, w, X, info, cat, valid, model_key, ytrain, l1_sharded=False):
        """Metalearner on the level-one frame L1 [F', N] with response y / weights w; the ensemble's
        training metrics are scored on the training frame ``ytrain = (X, y, w, offset)``. On a row-sharded
        cloud the level-one frame holds this rank's rows (the base models' holdouts are sharded the same
        way) and the metalearner trains sharded."""
        from ..parallel import collectives as coll, dframe
        transform = str(self.p.get("metalearner_transform") or "NONE").lower()
        if transform == "logit":
            if cat not in ("Binomial", "Multinomial"):
                raise ValueError("metalearner_transform=Logit needs a categorical response")
            L1 = _logit(L1)
        names = []
        for m in models:
            if cat == "Multinomial":
                names += [f"{m.key}/{d}" for d in info.response_domain]
            else:
                names.append(m.key)
        algo = str(self.p["metalearner_algorithm"]).lower()
        mp = dict(self.p["metalearner_params"] or {})
        if algo in ("auto", "glm"):
            algo = "glm"
            mp.setdefault("non_negative", True)
            if "lambda" not in mp:
                mp.setdefault("lambda_", 0.0)
            if cat == "Binomial":
                mp.setdefault("family", "binomial")
        elif algo == "naivebayes":
            algo = "naivebayes"
        mp.setdefault("seed", self.p.get("seed", -1))
        # the metalearner is a regular model trained on the level-one frame (StackedEnsemble.java
        # buildMetalearner): with metalearner_nfolds it is cross-validated there, so the ensemble's
        # cross-validation metrics are out-of-fold twice over (base holdouts -> metalearner holdouts)
        from ..frame import Column, H2OFrame
        with dframe.shard_ctx(dframe.make_shard(L1.shape[1]) if l1_sharded else None):
            cols = [Column(n, "real", L1[i].double()) for i, n in enumerate(names)]
            if info.response_domain is not None:
                yc = torch.nan_to_num(y.float(), nan=-1).to(torch.int32)
                cols.append(Column(info.response, "enum", yc, list(info.response_domain)))
            else:
                cols.append(Column(info.response, "real", y.double()))
            wname = None
            if w is not None:
                wname = "__se_weights"
                cols.append(Column(wname, "real", w.double()))
            fold_col = self.p.get("metalearner_fold_column")
            if fold_col:
                raise ValueError("metalearner_fold_column: pass the fold ids as metalearner_params['fold_column'] "
                                 "of a column present in the level-one frame")
            l1_frame = H2OFrame._from_columns(cols)
        nf = int(self.p.get("metalearner_nfolds") or 0)
        if nf > 1:
            fa = str(self.p.get("metalearner_fold_assignment") or "AUTO")
            mp.update(nfolds=nf, fold_assignment="Random" if fa.upper() == "AUTO" else fa,
                      keep_cross_validation_predictions=True)
        if wname:
            mp["weights_column"] = wname
        meta = builder_train(algo, mp, names, info.response, l1_frame,
                             (model_key or make_key("se")) + "_metalearner")
        model = StackedEnsembleModel(model_key or make_key("stackedensemble"), self.p, info)
        model.device = X.device
        model.base_keys = [m.key for m in models]
        model.meta = meta
        model.output["base_models"] = model.base_keys
        model.output["metalearner"] = meta.key
        model.output["metalearner_transform"] = transform
        Xt, yt_, wt_, offset = ytrain
        if yt_ is None:                      # blending: the SE's training metrics are on the training frame
            yt_, wt_ = self._train_y, self._train_w
        y, w = yt_, wt_
        model.output["stacking_strategy"] = "blending" if self.p.get("blending_frame") is not None else "cross_validation"
        nst = int(self.p.get("score_training_samples") or 0)
        start, n_glob = coll.exclusive_offset(X.shape[1]) if coll.is_dist() else (0, X.shape[1])
        if 0 < nst < n_glob:      # score_training_samples: training metrics on a row sample of about nst rows
            from .shared_tree import resolve_seed
            u = coll.row_uniform(resolve_seed(self.p.get("seed", -1)) & 0x7FFFFFFF, 29, start, X.shape[1], X.device)
            si = torch.nonzero(u < nst / n_glob).flatten()
            model.output["training_metrics"] = model.metrics_for(X[:, si], y[si], None if w is None else w[si],
                                                                 None if offset is None else offset[si])
        else:
            model.output["training_metrics"] = model.metrics_for(X, y, w, offset)
        # out-of-fold estimate only: the metalearner's own cross-validation (never its training fit)
        model.output["cross_validation_metrics"] = meta.output.get("cross_validation_metrics")
        if self.p.get("keep_levelone_frame"):
            model.output["levelone_frame_id"] = l1_frame.frame_id
        if valid is not None:
            Xv, yv, wv, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv, ov)
        dkv.put(meta.key, meta)
        return model

    def to_state(self):  # pragma: no cover - persisted through base models' keys
        return {}
