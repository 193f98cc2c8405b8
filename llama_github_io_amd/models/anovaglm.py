"""ANOVA GLM (reference: ``hex/anovaglm/ANOVAGLM.java``, ``ANOVAGLMModel.java``, ``ANOVAGLMUtils``).

Builds every main effect and interaction term up to ``highest_interaction_term`` (products of the
standardized numeric / one-hot categorical columns), fits the full GLM and, for each term, the GLM
without it (Type III), and reports per term: degrees of freedom, the deviance increase (SS) and
the F (or χ² for binomial/poisson) test p-value. Fits run on the IRLSM Gram solver.
"""
from __future__ import annotations

import itertools
import math
import time

import numpy as np
import torch

from .base import DataInfo, Model, make_key
from .datainfo import Expander

ANOVA_DEFAULTS = dict(family="AUTO", link="family_default", highest_interaction_term=2, lambda_=0.0, alpha=0.0,
                      standardize=True, type=3, save_transformed_framekeys=False, seed=-1)


class ANOVAGLMModel(Model):
    algo = "anovaglm"

    def _predict_tensor(self, X, offset=None):
        return self.full._predict_tensor(self._terms(X.to(self.device))[0], offset)

    def _terms(self, X):
        ex = self.expander
        Z = ex.transform(X)
        cols, names = [], []
        for term, idx in self.term_cols:
            for combo in idx:
                v = torch.ones(Z.shape[0], dtype=Z.dtype, device=Z.device)
                for c in combo:
                    v = v * Z[:, c]
                cols.append(v)
        return torch.stack(cols, 0), names

    def summary(self):
        return self.output["anova_table"]


class ANOVAGLMTrainer:
    def __init__(self, params):
        p = dict(ANOVA_DEFAULTS)
        if "lambda" in params:
            params = dict(params)
            params["lambda_"] = params.pop("lambda")
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from scipy import stats
        if int(self.p.get("type") or 0) not in (0, 3):
            raise ValueError("ANOVAGLM: only type 3 sums of squares are supported (type=3 or the default 0)")
        from .glm import GLMTrainer
        t0 = time.time()
        p = self.p
        from ..parallel import collectives as coll
        ex = Expander(info, standardize=True, use_all_factor_levels=False).fit(
            X, reduce=coll.all_reduce_ if coll.is_dist() else None)
        groups = []
        for j in range(info.F):
            if info.iscat[j]:
                i = ex.cats.index(j)
                groups.append(list(range(ex.cat_offsets[i], ex.cat_offsets[i] + ex.cat_sizes[i])))
            else:
                groups.append([ex.num_off + ex.nums.index(j)])
        term_cols = []
        H = int(p["highest_interaction_term"])
        for r in range(1, min(H, info.F) + 1):
            for combo in itertools.combinations(range(info.F), r):
                idx = list(itertools.product(*[groups[j] for j in combo]))
                term_cols.append((":".join(info.x[j] for j in combo), idx))
        model = ANOVAGLMModel(model_key or make_key("anovaglm"), p, info)
        model.device = X.device
        model.expander = ex
        model.term_cols = term_cols
        T, _ = model._terms(X)
        names = []
        spans = []
        k = 0
        for term, idx in term_cols:
            spans.append((term, k, k + len(idx)))
            names += [f"{term}_{i}" for i in range(len(idx))]
            k += len(idx)
        # GLM fields ANOVAGLM passes to its GLMs (ANOVAGLMUtils.buildGLMParameters; "type" and
        # "save_transformed_framekeys" are the ANOVA-only ones)
        gp = {kk: v for kk, v in p.items() if kk in ("family", "link", "lambda_", "alpha", "seed", "early_stopping", "prior",
                                                     "plug_values", "missing_values_handling", "tweedie_variance_power",
                                                     "tweedie_link_power", "theta", "solver", "max_iterations",
                                                     "non_negative", "compute_p_values") and v is not None}
        gp["standardize"] = False

        def fitg(rows):
            ginfo = DataInfo([names[i] for i in rows], np.zeros(len(rows), np.int32), [None] * len(rows), info.response,
                             info.response_domain)
            return GLMTrainer(gp).fit(T[rows].contiguous(), y, w, offset, ginfo)
        full = fitg(list(range(T.shape[0])))
        model.full = full
        fam = full.output["family"]
        dev_full = full.output["residual_deviance"]
        n = int(coll.all_reduce_scalar(float((~torch.isnan(y)).sum())))
        p_full = T.shape[0] + 1
        disp = dev_full / max(n - p_full, 1)
        table = []
        for term, a, b in spans:
            rows = [i for i in range(T.shape[0]) if not (a <= i < b)]
            red = fitg(rows) if rows else None
            dev_red = red.output["residual_deviance"] if red is not None else full.output["null_deviance"]
            ss = dev_red - dev_full
            df = b - a
            if fam in ("binomial", "poisson", "multinomial"):
                stat, pv = ss, float(stats.chi2.sf(max(ss, 0), df))
            else:
                stat = (ss / df) / max(disp, 1e-300)
                pv = float(stats.f.sf(max(stat, 0), df, max(n - p_full, 1)))
            table.append(dict(term=term, family=fam, df=df, SS=ss, F_or_chisq=stat, p_value=pv))
        model.output["anova_table"] = table
        model.output["training_metrics"] = full.output["training_metrics"]
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
