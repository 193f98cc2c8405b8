"""Generic model: a model imported from a MOJO (reference: ``hex/generic/Generic.java``,
``GenericModel.java`` — scoring through genmodel without the original algorithm)."""
from __future__ import annotations

import math

import numpy as np
import torch

from .base import DataInfo, Model, make_key


_ALGO_BY_NAME = {"Generalized Linear Modeling": "glm", "Gradient Boosting Machine": "gbm",
                 "Distributed Random Forest": "drf", "K-means": "kmeans", "Deep Learning": "deeplearning",
                 "Isolation Forest": "isolationforest", "Word2Vec": "word2vec", "XGBoost": "xgboost",
                 "Principal Components Analysis": "pca", "Generalized Low Rank Modeling": "glrm",
                 "Stacked Ensemble": "stackedensemble", "Support Vector Machine (*Spark*)": "svm"}


class GenericModel(Model):
    algo = "generic"

    @staticmethod
    def from_mojo(path: str, model_id=None, prefix: str = "") -> "GenericModel":
        from ..mojo import algos as A
        from ..mojo.reader import _floats, parse_mojo
        from ..ops.forest import Forest
        mj = parse_mojo(path, prefix)
        ki = mj["info"]
        if mj["state"] is not None:                    # framework-native payload
            from ..persist import _from_state
            st = mj["state"]
            inner = _from_state(st)
            m = GenericModel(model_id or make_key("generic"), dict(path=path), inner.info)
            m.inner = inner
            m.output = dict(inner.output)
            m.mojo_info = ki
            return m
        cols = mj["columns"]
        sup = ki.get("supervised", "false") == "true"
        nfeat = int(ki["n_features"])
        xs = cols[:nfeat]
        doms = [mj["domains"].get(i) for i in range(nfeat)]
        iscat = np.array([1 if d is not None else 0 for d in doms], dtype=np.int32)
        # the response is the LAST column (weights / offset / fold columns may sit in between)
        resp = cols[-1] if sup and len(cols) > nfeat else None
        rdom = mj["domains"].get(len(cols) - 1) if resp else None
        info = DataInfo(xs, iscat, doms, resp, rdom)
        m = GenericModel(model_id or make_key("generic"), dict(path=path), info)
        m.mojo_info = ki
        m.inner = None
        if "algo" not in ki:          # MOJO 1.0 files name the algorithm only in full
            ki["algo"] = _ALGO_BY_NAME.get(ki.get("algorithm", ""), str(ki.get("algorithm", "")).lower())
        algo = ki["algo"]
        m.output["original_algo"] = algo
        cat = ki.get("category", "Regression")
        m.output["model_category"] = cat
        if algo in ("gbm", "drf", "isolationforest"):
            K = int(ki.get("n_trees_per_class", 1))
            n = int(ki["n_trees"])
            fr = Forest(n_classes_out=K)
            binom_drf = algo == "drf" and cat == "Binomial" and K == 1
            vmap = (lambda v: 1.0 - v) if binom_drf else (lambda v: v)
            from ..mojo.treebytes import bytes_to_tree
            for it in range(n):
                for c in range(K):
                    name = f"trees/t{c:02d}_{it:03d}.bin"
                    if name in mj["trees"]:
                        fr.add(bytes_to_tree(mj["trees"][name], vmap), c)
            m.forest = fr
            m.ntrees = n
            if ki.get("calib_method") == "platt":
                m.calibration_model = ("platt", _floats(ki["calib_glm_beta"]))
            elif ki.get("calib_method") == "isotonic":
                tx, ty = A.load_isotonic(mj["files"])
                m.calibration_model = ("isotonic", float(ki["calib_min_x"]), float(ki["calib_max_x"]), tx, ty)
        elif algo == "xgboost":
            from ..mojo import xgboost_mojo as XG
            obj, base, ncls, trees, tinfo = XG.read(mj["files"]["boosterBytes"])
            m.forest = Forest(trees, tinfo, max(ncls, 1))
            m.xgb_obj, m.xgb_base = obj, base
        elif algo == "glm":
            m.beta = torch.tensor(_floats(ki["beta"]), dtype=torch.float64)
            m.cat_offsets = [int(v) for v in _floats(ki["cat_offsets"])]
            m.use_all = ki.get("use_all_factor_levels") == "true"
            m.num_means = _floats(ki.get("num_means", "[]"))
            m.cat_modes = [int(v) for v in _floats(ki.get("cat_modes", "[]"))]
        elif algo == "kmeans":
            m.centers = torch.tensor([_floats(ki[f"center_{i}"]) for i in range(int(ki["center_num"]))], dtype=torch.float64)
            m.std = ki.get("standardize") == "true"
            if m.std:
                m.means = _floats(ki["standardize_means"])
                m.mults = _floats(ki["standardize_mults"])
                m.modes = [int(v) for v in _floats(ki["standardize_modes"])]
        elif algo == "glrm":
            m.glrm = A.load_glrm(ki, mj["files"])
            m.output["model_category"] = "DimReduction"
        elif algo == "svm":
            m.svm = dict(weights=_floats(ki["weights"]), intercept=float(ki["interceptor"]),
                         means=_floats(ki.get("means", "[]")), mean_imputation=ki.get("meanImputation") == "true",
                         threshold=float(ki.get("threshold", 0.0)), default_threshold=float(ki.get("defaultThreshold", 0.0)))
        elif algo == "deeplearning":
            m.dl = A.load_deeplearning(ki)
        elif algo == "pca":
            m.pca = A.load_pca(ki, mj["files"]["eigenvectors_raw"])
            m.output["model_category"] = "DimReduction"
        elif algo == "word2vec":
            from .word2vec import Word2VecModel
            words, V = A.load_word2vec(ki, mj["files"]["vectors"], mj["files"]["vocabulary"].decode())
            inner = Word2VecModel(m.key + "_w2v", {}, info)
            inner.words, inner.vectors = words, V
            inner.vocab = {w: i for i, w in enumerate(words)}
            m.inner = inner
            m.output["model_category"] = "WordEmbedding"
        elif algo == "isotonicregression":
            from .isotonic import IsotonicModel
            tx, ty = A.load_isotonic(mj["files"])
            inner = IsotonicModel(m.key + "_iso", dict(out_of_bounds="clip"), info)
            inner.thresholds_x, inner.thresholds_y = tx.tolist(), ty.tolist()
            m.inner = inner
        elif algo == "extendedisolationforest":
            m.eif = A.load_eif(ki, mj["files"])
            m.output["model_category"] = "AnomalyDetection"
        elif algo == "targetencoder":
            m.inner = A.load_targetencoder(ki, mj["files"], info)
            m.inner.key = m.key + "_te"
            m.output["model_category"] = "TargetEncoder"
        elif algo == "coxph":
            m.cox = A.load_coxph(ki, mj["files"])
            m.output["model_category"] = "CoxPH"
        elif algo == "stackedensemble":
            subs = {}
            for i in range(int(ki.get("submodel_count", 0))):
                key = ki[f"submodel_key_{i}"]
                subs[key] = GenericModel.from_mojo(path, key, prefix + ki[f"submodel_dir_{i}"])
            # a base model the metalearner dropped (zero coefficient) is absent from the zip: keep its
            # slot so the level-one columns line up with the metalearner's inputs (StackedEnsembleMojoModel)
            m.base = [subs.get(ki.get(f"base_model{i}")) for i in range(int(ki["base_models_num"]))]
            m.meta = subs[ki["metalearner"]]
            m.meta_transform = ki.get("metalearner_transform", "NONE")
            if m.info.response_domain is None and m.meta.info.response_domain is not None:
                m.info.response_domain = list(m.meta.info.response_domain)   # out-of-range domain entry
        elif algo == "gam":
            m.gam = A.load_gam(ki, mj["files"])
            ncen = int(ki["num_expanded_gam_columns_center"])
            normal = xs[: nfeat - ncen]
            src = [c for cs in m.gam["cols"] for c in cs if c not in normal]
            src = list(dict.fromkeys(src))
            m.gam["n_normal"] = len(normal)
            m.gam["src_index"] = [(normal + src).index(cs[0]) for cs in m.gam["cols"]]
            m.info = DataInfo(normal + src, np.concatenate([iscat[: len(normal)], np.zeros(len(src), np.int32)]),
                              doms[: len(normal)] + [None] * len(src), resp, rdom)
        elif algo == "rulefit":
            m.rulefit = A.load_rulefit(ki)
            m.glm_sub = GenericModel.from_mojo(path, m.rulefit["linear_key"],
                                               prefix + ki.get("submodel_dir_0", f"models/{m.rulefit['linear_key']}/"))
        else:
            raise NotImplementedError(f"MOJO algo {algo} not supported by this reader")
        return m

    def _calibrated(self, P):
        """CalibrationMojoHelper.calibrateClassProbabilities: Platt p = logistic(p0 * b0 + b1), isotonic
        p = interp(clip(p1)); cal_p0 = 1 - p."""
        from ..frame import Column, H2OFrame
        cm = self.calibration_model
        if cm[0] == "platt":
            b = cm[1]
            c1 = torch.sigmoid(P[:, 0].double() * b[0] + b[1])
        else:
            _, lo, hi, tx, ty = cm
            x = P[:, 1].double().clamp(lo, hi).cpu().numpy()
            c1 = torch.as_tensor(np.interp(x, tx, ty), dtype=torch.float64, device=P.device)
        return H2OFrame._from_columns([Column("cal_p0", "real", (1 - c1).contiguous()), Column("cal_p1", "real", c1)])

    def __getattr__(self, name):
        # Word2Vec / isotonic MOJOs delegate their model-specific API (find_synonyms, transform, ...)
        inner = self.__dict__.get("inner")
        if inner is not None and not name.startswith("_"):
            return getattr(inner, name)
        raise AttributeError(name)

    @property
    def model_category(self):
        return self.output.get("model_category", "Regression")

    def _align(self, X, parent_info):
        """Rows of ``X`` (parent's predictor order) re-ordered into this model's predictor order."""
        idx = [parent_info.x.index(n) for n in self.info.x]
        return X[idx]

    def default_threshold(self):
        if self.inner is not None:
            return self.inner.default_threshold()
        if self.model_category != "Binomial":
            return None
        return float(self.mojo_info.get("default_threshold", 0.5))

    def prediction_names(self):
        if self.inner is not None:
            return self.inner.prediction_names()
        if self.output.get("original_algo") == "isolationforest":
            return ["predict", "mean_length"]
        if self.output.get("original_algo") == "extendedisolationforest":
            return ["anomaly_score", "mean_length"]
        if self.output.get("original_algo") == "coxph":
            return ["lp"]
        if self.output.get("original_algo") == "glrm":
            return [f"Arch{i + 1}" for i in range(self.glrm["ncolX"])]
        if self.output.get("original_algo") == "pca":
            return [f"PC{i + 1}" for i in range(self.pca["k"])]
        return None

    def _design(self, X):
        """GLM/KMeans layout: one-hot categoricals (cats first), then numerics (GlmMojoModel)."""
        info = self.info
        cats = [j for j in range(info.F) if info.iscat[j]]
        nums = [j for j in range(info.F) if not info.iscat[j]]
        N = X.shape[1]
        use_all = getattr(self, "use_all", True)
        ncat_cols = sum(len(info.domains[j]) - (0 if use_all else 1) for j in cats)
        Z = torch.zeros(N, ncat_cols + len(nums), dtype=torch.float64, device=X.device)
        off = 0
        modes = getattr(self, "cat_modes", None) or getattr(self, "modes", None) or [0] * len(cats)
        for i, j in enumerate(cats):
            L = len(info.domains[j])
            c = X[j]
            c = torch.where(torch.isnan(c), torch.full_like(c, float(modes[i] if i < len(modes) else 0)), c).long()
            col = c - (0 if use_all else 1)
            ok = (col >= 0) & (col < L - (0 if use_all else 1))
            rows = torch.nonzero(ok).flatten()
            Z[rows, off + col[rows]] = 1
            off += L - (0 if use_all else 1)
        for i, j in enumerate(nums):
            v = X[j].double()
            mu = (getattr(self, "num_means", None) or getattr(self, "means", None) or [0.0] * len(nums))
            Z[:, off + i] = torch.where(torch.isnan(v), torch.full_like(v, mu[i] if i < len(mu) else 0.0), v)
        return Z, off

    def _xgb_matrix(self, X):
        """XGBoost MOJO input (h2o XGBoost DataInfo): each categorical one-hot over its levels plus a
        trailing NA slot at ``cat_offsets``, then the numerics. With ``sparse`` the DMatrix was sparse:
        absent entries (non-hot levels, numeric zeros) are *missing*, not 0."""
        ki = self.mojo_info
        if "cat_offsets" not in ki:
            return X
        from ..mojo.reader import _floats
        off = [int(v) for v in _floats(ki["cat_offsets"])]
        ncat, nnum = int(ki.get("cats", 0)), int(ki.get("nums", 0))
        sparse = ki.get("sparse") == "true"
        N = X.shape[1]
        P = off[-1] + nnum
        fill = float("nan") if sparse else 0.0
        D = torch.full((P, N), fill, dtype=torch.float32, device=X.device)
        ar = torch.arange(N, device=X.device)
        for c in range(ncat):
            v = X[c]
            L = off[c + 1] - off[c] - 1
            idx = torch.where(torch.isnan(v), torch.full_like(v, float(L)), v).long().clamp(0, L)
            D[off[c] + idx, ar] = 1.0
        nums = X[ncat:ncat + nnum].float()
        if sparse:
            nums = torch.where(nums == 0, torch.full_like(nums, float("nan")), nums)
        D[off[-1]:] = nums
        return D

    def kmeans_distances(self, X):
        """KMeansMojoModel.score0: Kmeans_preprocessData (NA -> mean / mode, standardise numerics) then
        KMeans_distance per center: squared difference for numerics, 0/1 mismatch for categoricals,
        scaled up by n / (non-NA count)."""
        info = self.info
        Xd = X.double().T.clone()                                   # [N, F]
        F = Xd.shape[1]
        iscat = torch.tensor([bool(info.iscat[j]) for j in range(F)], device=Xd.device)
        if self.std:
            mu = torch.tensor(self.means, dtype=torch.float64, device=Xd.device)
            mul = torch.tensor(self.mults, dtype=torch.float64, device=Xd.device)
            mode = torch.tensor([float(v) for v in self.modes], dtype=torch.float64, device=Xd.device)
            fill = torch.where(iscat, mode, mu)
            Xd = torch.where(torch.isnan(Xd), fill.expand_as(Xd), Xd)
            Xd = torch.where(iscat, Xd, (Xd - torch.nan_to_num(mu)) * mul)
        C = self.centers.to(Xd.device)                              # [K, F]
        valid = ~torch.isnan(Xd)
        diff = Xd[:, None, :] - C[None]
        term = torch.where(iscat, (diff != 0).double(), diff * diff)
        term = torch.where(valid[:, None, :], term, torch.zeros_like(term))
        D = term.sum(-1)
        pts = valid.sum(1, keepdim=True).double()
        scale = torch.where((pts > 0) & (pts < F), F / pts.clamp(min=1), torch.ones_like(pts))
        return D * scale

    def _predict_tensor(self, X, offset=None):
        if self.inner is not None:
            return self.inner._predict_tensor(X, offset)
        ki = self.mojo_info
        algo = ki["algo"]
        cat = self.model_category
        if algo == "gbm":
            f = self.forest.predict_raw(X) + float(ki.get("init_f", 0.0))
            if offset is not None:
                f = f + offset[:, None]
            d = ki.get("distribution", "gaussian")
            if d == "multinomial":
                if f.shape[1] == 1 and cat == "Binomial":      # 1-tree binomial optimisation: [f, -f]
                    f = torch.cat([f, -f], 1)
                return torch.softmax(f, 1)
            if d in ("bernoulli", "quasibinomial", "modified_huber"):
                p1 = torch.sigmoid(f[:, 0])
                return torch.stack([1 - p1, p1], 1)
            if ki.get("link_function") == "log":
                return torch.exp(f[:, 0])
            return f[:, 0]
        if algo == "xgboost":
            f = self.forest.predict_raw(self._xgb_matrix(X)) + self.xgb_base
            if offset is not None:
                f = f + offset[:, None]
            obj = self.xgb_obj
            if obj == "binary:logistic":
                p1 = torch.sigmoid(f[:, 0])
                return torch.stack([1 - p1, p1], 1)
            if obj.startswith("multi:"):
                return torch.softmax(f, 1)
            if obj in ("count:poisson", "reg:gamma", "reg:tweedie"):
                return torch.exp(f[:, 0])
            return f[:, 0]
        if algo == "drf":
            s = self.forest.predict_raw(X) / max(1, self.ntrees)
            if cat == "Regression":
                return s[:, 0]
            if cat == "Binomial" and s.shape[1] == 1:
                p1 = s[:, 0].clamp(0, 1)
                return torch.stack([1 - p1, p1], 1)
            return s / s.sum(1, keepdim=True).clamp(min=1e-30)
        if algo == "isolationforest":
            s = self.forest.predict_raw(X)[:, 0].double()
            mn, mx = float(ki["min_path_length"]), float(ki["max_path_length"])
            score = (mx - s) / (mx - mn) if mx > mn else torch.ones_like(s)
            return torch.stack([score.float(), (s / max(1, self.ntrees)).float()], 1)
        if algo == "glm":
            Z, _ = self._design(X)
            fam, link = ki["family"], ki["link"]
            nb = Z.shape[1] + 1
            B = self.beta.to(Z.device).view(-1, nb)
            eta = Z @ B[:, :-1].T + B[:, -1]
            if offset is not None:
                eta = eta + offset.double()[:, None]
            if fam == "multinomial":
                return torch.softmax(eta, 1).float()
            from .glm import Family
            mu = Family(fam, link, 0.0, float(ki.get("tweedie_link_power", 1.0))).linkinv(eta[:, 0])
            if fam in ("binomial", "quasibinomial", "fractionalbinomial"):
                return torch.stack([1 - mu, mu], 1).float()
            return mu.float()
        if algo == "gam":
            from ..mojo import algos as A
            g = self.gam
            eta = A.score_gam(g, X[: g["n_normal"]], [X[i] for i in g["src_index"]])
            if offset is not None:
                eta = eta + offset.double()
            from .glm import Family
            fam = "binomial" if g["family"] == "bernoulli" else g["family"]
            mu = Family(fam, g["link"], 0.0, g["tlp"]).linkinv(eta)
            if fam in ("binomial", "quasibinomial", "fractionalbinomial"):
                return torch.stack([1 - mu, mu], 1).float()
            return mu.float()
        if algo == "deeplearning":
            from ..mojo import algos as A
            return A.score_deeplearning(self.dl, X, cat)
        if algo == "pca":
            from ..mojo import algos as A
            return A.score_pca(self.pca, X)
        if algo == "extendedisolationforest":
            from ..mojo import algos as A
            return A.score_eif(self.eif, X)
        if algo == "coxph":
            from ..mojo import algos as A
            return A.score_coxph(self.cox, X)
        if algo == "rulefit":
            from ..mojo import algos as A
            return A.score_rulefit(self.rulefit, self.glm_sub, X, self.info)
        if algo == "stackedensemble":
            cols = []
            K = len(self.info.response_domain or []) if cat == "Multinomial" else 1
            for b in self.base:
                if b is None:
                    cols.append(torch.zeros(X.shape[1], K, dtype=torch.float64, device=X.device))
                    continue
                P = b._predict_tensor(b._align(X, self.info), offset)
                if cat == "Binomial":
                    p1 = P[:, 1:2].double()
                    if self.meta_transform == "Logit":
                        p1 = torch.logit(p1.clamp(1e-15, 1 - 1e-15))
                    cols.append(p1)
                elif cat == "Multinomial":
                    cols.append(P.double())
                else:
                    cols.append(P.reshape(-1, 1).double())
            L1 = torch.cat(cols, 1).T.contiguous().float()
            return self.meta._predict_tensor(L1, None)
        if algo == "kmeans":
            return self.kmeans_distances(X).argmin(1).float()
        if algo == "glrm":
            from ..mojo import algos as A
            return A.score_glrm(self.glrm, X)
        if algo == "svm":
            sv = self.svm
            Xd = X.double().T
            w = torch.tensor(sv["weights"], dtype=torch.float64, device=Xd.device)
            if sv["mean_imputation"] and sv["means"]:
                mu = torch.tensor(sv["means"][:Xd.shape[1]], dtype=torch.float64, device=Xd.device)
                Xd = torch.where(torch.isnan(Xd), mu.expand_as(Xd), Xd)
            pred = Xd @ w + sv["intercept"]
            if cat != "Binomial":
                return pred.float()
            thr, dthr = sv["threshold"], sv["default_threshold"]
            # SvmMojoModel.score0: preds = [label, p0, p1] built from the margin
            p1 = torch.where(pred > thr, torch.clamp(pred, min=dthr), torch.where(pred >= dthr, torch.full_like(pred, dthr - 1), pred))
            p0 = torch.where(pred > thr, p1 - 1, p1 + 1)
            self._svm_label = (pred > thr)
            return torch.stack([p0, p1], 1).float()
        raise NotImplementedError(algo)


class GenericTrainer:
    """``H2OGenericEstimator(path=...)``: 'training' imports the MOJO."""

    def __init__(self, params):
        self.p = dict(params)
        self.job = None

    def fit(self, X=None, y=None, w=None, offset=None, info=None, valid=None, model_key=None):
        path = self.p.get("path") or self.p.get("model_key")
        return GenericModel.from_mojo(path, model_key)
