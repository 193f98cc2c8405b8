"""Infogram / admissible machine learning (reference: ``h2o-admissibleml/src/main/java/hex/Infogram/
Infogram.java``, ``InfogramModel.java``, ``EstimateCMI.java``).

Core infogram (no ``protected_columns``): relevance = normalised variable importance of a model on
the top-k predictors; conditional mutual information of predictor j = mean log₂ p̂(y|all) −
mean log₂ p̂(y|all \\ j) (EstimateCMI: per-row log probability of the observed class), scaled to
[0, 1] by its maximum. Safe infogram (``protected_columns`` given): relevance from the model on
non-protected features; CMI_j = log-likelihood gain of (protected ∪ {j}) over protected only.
Admissible = relevance ≥ ``relevance_threshold`` and cmi ≥ ``cmi_threshold``. The per-feature
models are GBMs on the device tree engine (``algorithm`` may pick GLM/DRF/DeepLearning). On a row-sharded
frame the per-feature models train sharded and the log-likelihood means are merged sums.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from ..parallel import collectives as coll
from .base import DataInfo, Model, make_key


def _red(t: torch.Tensor) -> torch.Tensor:
    if not coll.is_dist():
        return t
    return coll.all_reduce_(t.contiguous().to(coll.comm_device())).to(t.device)

INFO_DEFAULTS = dict(algorithm="AUTO", algorithm_params=None, protected_columns=None, cmi_threshold=0.1,
                     relevance_threshold=0.1, total_information_threshold=-1.0, net_information_threshold=-1.0,
                     safety_index_threshold=-1.0, relevance_index_threshold=-1.0, data_fraction=1.0, top_n_features=50,
                     seed=-1)


class InfogramModel(Model):
    algo = "infogram"

    def _predict_tensor(self, X, offset=None):
        raise NotImplementedError("Infogram is an exploratory model; use get_admissible_features()")

    def get_admissible_features(self):
        return self.output["admissible_features"]

    def get_admissible_cmi(self):
        return self.output["admissible_cmi"]

    def get_admissible_relevance(self):
        return self.output["admissible_relevance"]

    def get_admissible_score_frame(self):
        from ..frame import H2OFrame
        import pandas as pd
        return H2OFrame(pd.DataFrame(self.output["table"]))


class InfogramTrainer:
    def __init__(self, params):
        p = dict(INFO_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def _train(self, cols, X, y, w, info):
        from .builder import REGISTRY
        algo = str(self.p["algorithm"]).lower()
        algo = "gbm" if algo == "auto" else algo
        sub = DataInfo([info.x[j] for j in cols], np.asarray(info.iscat)[cols], [info.domains[j] for j in cols],
                       info.response, info.response_domain)
        params = dict(self.p.get("algorithm_params") or {})
        params.setdefault("seed", self.p["seed"])
        if algo == "gbm":
            params.setdefault("ntrees", 50)
            params.setdefault("max_depth", 5)
        m = REGISTRY[algo].trainer(params).fit(X[cols].contiguous(), y, w, None, sub)
        return m

    def _loglik(self, m, X, y, cols):
        """Mean log2 likelihood of the observed responses (EstimateCMI); sums merged over the row shards."""
        P = m.score_tensor(X[cols].contiguous())
        if P.dim() == 1:                        # regression: Gaussian log-likelihood proxy
            r = (y - P).double()
            st = _red(torch.stack([(r * r).sum(), torch.tensor(float(r.numel()), dtype=torch.float64,
                                                               device=r.device)]))
            s2 = float(st[0] / st[1]) + 1e-12
            return (-0.5 * float(st[0]) / s2 / float(st[1]) - 0.5 * math.log(2 * math.pi * s2)) / math.log(2)
        py = P.double().gather(1, torch.nan_to_num(y).long()[:, None])[:, 0]
        ok = py > 0
        st = _red(torch.stack([torch.log(py[ok]).sum(), ok.double().sum()]))
        return float(st[0] / st[1]) / math.log(2)

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        t0 = time.time()
        p = self.p
        frac = float(p.get("data_fraction") or 1.0)
        if not 0 < frac <= 1:
            raise ValueError("data_fraction must be in (0, 1]")
        if frac < 1.0:      # Infogram data_fraction: the CMI / relevance models see a random row sample
            from .shared_tree import resolve_seed
            # a per-global-row draw: the same sample however the rows are sharded
            start = coll.row_offset(X.shape[1])
            keep = coll.row_uniform(resolve_seed(p.get("seed", -1)) & 0x7FFFFFFF, 23, start, X.shape[1],
                                    X.device) < frac
            X, y = X[:, keep], y[keep]
            w = None if w is None else w[keep]
        prot = [c for c in (p["protected_columns"] or []) if c in info.x]
        prot_idx = [info.x.index(c) for c in prot]
        cand = [j for j in range(info.F) if j not in prot_idx]
        base = self._train(cand, X, y, w, info)
        vi = {r[0]: r[2] for r in (base.output.get("variable_importances") or [])}
        order = sorted(cand, key=lambda j: -vi.get(info.x[j], 0.0))
        k = int(p["top_n_features"])
        top = order[:k] if k > 0 else order
        rel = np.array([vi.get(info.x[j], 0.0) for j in top])
        rel = rel / rel.max() if rel.max() > 0 else rel
        cmi_raw = []
        if prot_idx:
            ll0 = self._loglik(self._train(prot_idx, X, y, w, info), X, y, prot_idx)
            for j in top:
                cols = prot_idx + [j]
                cmi_raw.append(self._loglik(self._train(cols, X, y, w, info), X, y, cols) - ll0)
        else:
            ll_all = self._loglik(self._train(top, X, y, w, info), X, y, top)
            for j in top:
                cols = [c for c in top if c != j]
                cmi_raw.append(ll_all - self._loglik(self._train(cols, X, y, w, info), X, y, cols) if cols else ll_all)
        cmi_raw = np.maximum(np.asarray(cmi_raw), 0.0)
        cmi = cmi_raw / cmi_raw.max() if cmi_raw.max() > 0 else cmi_raw
        rth = p["relevance_index_threshold"] if prot_idx else p["total_information_threshold"]
        cth = p["safety_index_threshold"] if prot_idx else p["net_information_threshold"]
        rth = p["relevance_threshold"] if rth is None or rth < 0 else rth
        cth = p["cmi_threshold"] if cth is None or cth < 0 else cth
        adm = (rel >= rth) & (cmi >= cth)
        names = [info.x[j] for j in top]
        model = InfogramModel(model_key or make_key("infogram"), p, info)
        model.device = X.device
        model.output.update(all_predictor_names=names, relevance=rel.tolist(), cmi=cmi.tolist(), cmi_raw=cmi_raw.tolist(),
                            admissible=adm.astype(int).tolist(),
                            admissible_features=[n for n, a in zip(names, adm) if a],
                            admissible_cmi=[float(c) for c, a in zip(cmi, adm) if a],
                            admissible_relevance=[float(r) for r, a in zip(rel, adm) if a],
                            table=dict(column=names, admissible=adm.astype(int).tolist(),
                                       admissible_index=(np.sqrt(rel ** 2 + cmi ** 2) / math.sqrt(2)).tolist(),
                                       relevance=rel.tolist(), cmi=cmi.tolist(), cmi_raw=cmi_raw.tolist()))
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
