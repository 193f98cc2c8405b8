"""Model selection (reference: ``hex/modelselection/ModelSelection.java``, ``ModelSelectionModel.java``,
``ModelSelectionUtils``): best-subset style searches over GLM predictors.

``mode``: ``allsubsets`` (exhaustive), ``maxr`` (forward add + sequential replacement), ``maxrsweep``
(same search on the swept Gram), ``forward``, ``backward`` (drop the predictor with the smallest
|z| until ``min_predictor_number``; needs p-values). For gaussian models the R² of any subset comes
straight from the device Gram of [Z, y] (one MFMA Gram kernel call, then tiny solves) — no refit
per candidate; other families refit the GLM. Output: best predictors and R² (or deviance) per
subset size, plus the GLM of each best subset.
"""
from __future__ import annotations

import itertools
import time

import numpy as np
import torch

from ..ops.gram import gram
from .base import DataInfo, Model, make_key
from .datainfo import Expander

MS_DEFAULTS = dict(mode="maxr", max_predictor_number=1, min_predictor_number=1, nparallelism=0, family="AUTO",
                   p_values_threshold=0.0, seed=-1)


class ModelSelectionModel(Model):
    algo = "modelselection"

    def _predict_tensor(self, X, offset=None):
        return self.best_models[-1]._predict_tensor(X[self.best_cols[-1]].contiguous(), offset)

    def result(self):
        import pandas as pd
        from ..frame import H2OFrame
        return H2OFrame(pd.DataFrame(self.output["result"]))

    def get_best_R2_values(self):
        return [r["best_r2_value"] for r in self.output["result"]]

    def get_best_model_predictors(self):
        return [r["predictor_names"] for r in self.output["result"]]

    def coef(self, predictor_size=None):
        i = (predictor_size or len(self.best_models)) - 1
        return self.best_models[i].output["coefficients"]


# GLM parameters ModelSelection hands to every GLM it builds (ModelSelectionUtils.generateGLMParameters copies
# the shared GLM fields of the ModelSelection parameters onto each GLM)
_GLM_PASS = ("beta_constraints", "cold_start", "max_active_predictors", "prior", "remove_collinear_columns",
             "startval", "objective_epsilon", "gradient_epsilon", "early_stopping", "plug_values",
             "missing_values_handling", "standardize", "intercept", "non_negative", "max_iterations", "influence",
             "tweedie_variance_power", "tweedie_link_power", "theta", "link", "solver")


class ModelSelectionTrainer:
    def __init__(self, params):
        p = dict(MS_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def _glm(self, **kw):
        from .glm import GLMTrainer
        gp = {k: self.p[k] for k in _GLM_PASS if self.p.get(k) is not None}
        gp.update(family=self.p["family"], lambda_=0.0)
        if gp.get("influence") and not kw.get("final"):
            gp.pop("influence")                       # diagnostics only for the reported best models
        kw.pop("final", None)
        gp.update(kw)
        return GLMTrainer(gp)

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from .glm import GLMTrainer
        t0 = time.time()
        p = self.p
        mode = str(p["mode"]).lower()
        F = info.F
        kmax = min(int(p["max_predictor_number"]), F)
        gaussian = info.response_domain is None and str(p["family"]).lower() in ("auto", "gaussian")
        ok = ~torch.isnan(y)
        # R² machinery from one Gram of [1, x_1..x_F (numeric; categoricals as codes), y]
        Xc = torch.nan_to_num(X.double())
        M = torch.cat([torch.ones(1, X.shape[1], dtype=torch.float64, device=X.device), Xc, y.double()[None]], 0)[:, ok].T
        G = gram(M.float().contiguous()) if X.is_cuda else M.T @ M
        from ..parallel import collectives as coll
        if coll.is_dist():                    # Gram of every rank's rows
            G = coll.all_reduce_(G.double().contiguous().to(coll.comm_device())).to(M.device)
        yy = G[-1, -1]
        ybar = G[0, -1] / G[0, 0]
        sst = float(yy - G[0, 0] * ybar * ybar)

        def r2(cols):
            idx = [0] + [c + 1 for c in cols]
            A = G[idx][:, idx]
            b = G[idx, -1]
            beta = torch.linalg.lstsq(A, b[:, None]).solution[:, 0]
            sse = float(yy - b @ beta)
            return 1 - sse / sst

        def score(cols):
            if gaussian:
                return r2(cols)
            sub = DataInfo([info.x[j] for j in cols], np.asarray(info.iscat)[cols], [info.domains[j] for j in cols],
                           info.response, info.response_domain)
            m = self._glm().fit(X[cols].contiguous(), y, w, offset, sub)
            return -m.output["residual_deviance"]

        best = []
        if mode == "allsubsets":
            for k in range(1, kmax + 1):
                cands = [(score(list(c)), list(c)) for c in itertools.combinations(range(F), k)]
                best.append(max(cands))
        elif mode in ("maxr", "maxrsweep", "forward"):
            cur = []
            for k in range(1, kmax + 1):
                rest = [j for j in range(F) if j not in cur]
                s, j = max((score(cur + [j]), j) for j in rest)
                cur = cur + [j]
                if mode != "forward":      # sequential replacement until no swap improves
                    improved = True
                    while improved:
                        improved = False
                        for i in range(len(cur)):
                            for jj in [x for x in range(F) if x not in cur]:
                                trial = cur[:i] + [jj] + cur[i + 1:]
                                st = score(trial)
                                if st > s + 1e-12:
                                    s, cur, improved = st, trial, True
                best.append((s, list(cur)))
        elif mode == "backward":
            cur = list(range(F))
            kmin = max(1, int(p["min_predictor_number"]))
            hist = []
            while len(cur) >= kmin:
                sub = DataInfo([info.x[j] for j in cur], np.asarray(info.iscat)[cur], [info.domains[j] for j in cur],
                               info.response, info.response_domain)
                m = self._glm(compute_p_values=True, standardize=False).fit(X[cur].contiguous(), y, w, offset, sub)
                hist.append((score(cur), list(cur)))
                if len(cur) == kmin:
                    break
                thr = float(p.get("p_values_threshold") or 0.0)
                if thr > 0:
                    # ModelSelection.buildBackwardModels: stop once every predictor's p-value (intercept
                    # excluded) is at or below the threshold
                    pv = m.output.get("p_values") or {}
                    if all(v <= thr for k, v in pv.items() if not k.startswith("Intercept")):
                        break
                z = m.output["z_values"]
                j_drop = min(cur, key=lambda j: abs(z.get(info.x[j], 0.0)))
                cur = [j for j in cur if j != j_drop]
            best = sorted(hist, key=lambda h: len(h[1]))
        else:
            raise ValueError(f"unknown mode {mode}")
        model = ModelSelectionModel(model_key or make_key("modelselection"), p, info)
        model.device = X.device
        model.best_cols, model.best_models = [], []
        rows = []
        for s, cols in best:
            sub = DataInfo([info.x[j] for j in cols], np.asarray(info.iscat)[cols], [info.domains[j] for j in cols],
                           info.response, info.response_domain)
            m = self._glm(final=True).fit(X[cols].contiguous(), y, w, offset, sub)
            model.best_cols.append(cols)
            model.best_models.append(m)
            rows.append(dict(model_name=f"best {len(cols)} predictor(s) model", predictor_names=[info.x[j] for j in cols],
                             best_r2_value=float(s) if gaussian else None, deviance=m.output.get("residual_deviance"),
                             coefficient_names=list(m.output["coefficients"])))
        model.output["result"] = rows
        model.output["training_metrics"] = model.best_models[-1].output["training_metrics"]
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
