"""AutoML (reference: ``h2o-automl/src/main/java/ai/h2o/automl/AutoML.java``, ``ModelingPlans.java``,
``Leaderboard.java``, ``modeling/*StepsProvider.java``).

Modeling plan: the reference default ``ModelingPlans.TEN_LAYERED`` (trimmed by ``include_algos`` /
``exclude_algos``): priority groups 1..10 of default models (XGBoost def_1..3, GLM, DRF, XRT, GBM
def_1..5, DeepLearning), random-discrete grids (XGBoost, GBM, DeepLearning 1/2/3 hidden layers),
exploitation (GBM learning-rate annealing, XGBoost learning-rate search), the completion step (resume
the two best grids) and Stacked Ensembles closing each group. Every model gets ``nfolds`` (default 5,
Modulo fold assignment so all share folds) CV with kept holdout predictions; early stopping uses the
adaptive tolerance of the training frame. Budgets: ``max_models`` (base models), ``max_runtime_secs``
(default 3600 when neither is set, split over steps by weight), ``max_runtime_secs_per_model``.
Leaderboard sort: AUC (binomial), mean_per_class_error (multinomial), mean_residual_deviance
(regression), with the other standard columns.
"""
from __future__ import annotations

import math
import time

import numpy as np

from .core import dkv
from .core.job import Job
from .grid import _metric_of
from .models import builder


def _coll():
    from .parallel import collectives as coll
    return coll

_DEFAULT_SORT = {"Binomial": "auc", "Multinomial": "mean_per_class_error", "Regression": "mean_residual_deviance"}
_DESC = {"auc", "aucpr", "r2"}


MODEL_W, GRID_W = 10, 30          # ModelingStep DEFAULT_MODEL_TRAINING_WEIGHT / DEFAULT_GRID_TRAINING_WEIGHT


def _plan():
    """The reference default plan (``ModelingPlans.TEN_LAYERED``): (algo, step id, priority group, weight).
    Steps run group by group in this definition order; SE steps close each group."""
    steps = [("xgboost", "def_2", 1, MODEL_W), ("xgboost", "def_1", 2, MODEL_W), ("xgboost", "def_3", 3, MODEL_W),
             ("xgboost", "grid_1", 4, 3 * GRID_W), ("xgboost", "lr_search", 6, GRID_W),
             ("glm", "def_1", 1, MODEL_W),
             ("drf", "def_1", 2, MODEL_W), ("drf", "XRT", 3, MODEL_W),
             ("gbm", "def_5", 1, MODEL_W), ("gbm", "def_2", 2, MODEL_W), ("gbm", "def_3", 2, MODEL_W),
             ("gbm", "def_4", 2, MODEL_W), ("gbm", "def_1", 3, MODEL_W), ("gbm", "grid_1", 4, 2 * GRID_W),
             ("gbm", "lr_annealing", 6, MODEL_W),
             ("deeplearning", "def_1", 3, MODEL_W), ("deeplearning", "grid_1", 4, GRID_W),
             ("deeplearning", "grid_2", 5, GRID_W), ("deeplearning", "grid_3", 5, GRID_W),
             ("completion", "resume_best_grids", 10, 2 * GRID_W)]
    steps += [("stackedensemble", f"best_of_family_{g}", g, MODEL_W // 2) for g in range(1, 6)]
    steps += [("stackedensemble", f"all_{g}", g, MODEL_W) for g in range(2, 6)]
    steps += [("stackedensemble", "best_of_family_gbm", 6, MODEL_W), ("stackedensemble", "all_gbm", 7, MODEL_W),
              ("stackedensemble", "best_of_family_xglm", 8, MODEL_W), ("stackedensemble", "all_xglm", 8, MODEL_W),
              ("stackedensemble", "best_of_family", 10, MODEL_W), ("stackedensemble", "best_N", 10, MODEL_W)]
    order = {id(st): i for i, st in enumerate(steps)}
    return sorted(steps, key=lambda st: (st[2], order[id(st)]))


def _defaults(algo, sid, seed, cat):
    """Per-step model parameters of the reference steps providers (``modeling/*StepsProvider.java``)."""
    tree = dict(ntrees=10000, score_tree_interval=5, seed=seed)
    if algo == "xgboost":
        base = dict(tree, sample_rate=0.6 if sid != "def_3" else 0.8, col_sample_rate=0.8, col_sample_rate_per_tree=0.8)
        return dict(base, **{"def_1": dict(max_depth=10, min_rows=5), "def_2": dict(max_depth=15, min_rows=10),
                             "def_3": dict(max_depth=5, min_rows=3)}[sid])
    if algo == "gbm":
        base = dict(tree, sample_rate=0.8, col_sample_rate=0.8, col_sample_rate_per_tree=0.8)
        return dict(base, **{"def_1": dict(max_depth=6, min_rows=1), "def_2": dict(max_depth=7, min_rows=10),
                             "def_3": dict(max_depth=8, min_rows=10), "def_4": dict(max_depth=10, min_rows=10),
                             "def_5": dict(max_depth=15, min_rows=100)}[sid])
    if algo == "glm":
        return dict(lambda_search=True, seed=seed, family="binomial" if cat == "Binomial" else
                    ("multinomial" if cat == "Multinomial" else "gaussian"))
    if algo == "drf":
        return dict(ntrees=10000, score_tree_interval=5, seed=seed, **({"histogram_type": "Random"} if sid == "XRT" else {}))
    if algo == "deeplearning":
        return dict(hidden=[10, 10, 10], seed=seed)
    return dict(seed=seed)


def _grid_space(algo, sid):
    """Random-discrete search spaces of the grid steps (GBM/XGBoost/DeepLearning steps providers)."""
    if algo == "gbm":
        return dict(max_depth=list(range(3, 18)), min_rows=[1, 5, 10, 15, 30, 100],
                    sample_rate=[0.5, 0.6, 0.7, 0.8, 0.9, 1.0], col_sample_rate=[0.4, 0.7, 1.0],
                    col_sample_rate_per_tree=[0.4, 0.7, 1.0], min_split_improvement=[1e-4, 1e-5])
    if algo == "xgboost":
        return dict(max_depth=[3, 6, 9, 12, 15], min_rows=[0.01, 0.1, 1.0, 3.0, 5.0, 10.0, 15.0, 20.0],
                    sample_rate=[0.6, 0.8, 1.0], col_sample_rate=[0.6, 0.8, 1.0],
                    col_sample_rate_per_tree=[0.7, 0.8, 0.9, 1.0], booster=["gbtree", "dart"],
                    reg_lambda=[0.001, 0.01, 0.1, 1, 10, 100], reg_alpha=[0.001, 0.01, 0.1, 0.5, 1])
    layers = {"grid_1": 1, "grid_2": 2, "grid_3": 3}[sid]
    return dict(hidden=[[u] * layers for u in (20, 50, 100)],
                hidden_dropout_ratios=[[r] * layers for r in (0.0, 0.1, 0.2, 0.3, 0.4, 0.5)],
                rho=[0.9, 0.95, 0.99], epsilon=[1e-6, 1e-7, 1e-8, 1e-9], input_dropout_ratio=[0.0, 0.05, 0.1, 0.15, 0.2])


def _grid_base(algo, seed):
    if algo == "gbm":
        return dict(ntrees=10000, score_tree_interval=5, seed=seed)
    if algo == "xgboost":
        return dict(ntrees=10000, score_tree_interval=5, seed=seed)
    return dict(epochs=10000, adaptive_rate=True, activation="RectifierWithDropout", seed=seed)


def default_stopping_tolerance(nrows: int) -> float:
    """RandomDiscreteValueSearchCriteria.default_stopping_tolerance_for_frame."""
    return min(0.05, max(0.001, 1.0 / math.sqrt(max(nrows, 1))))


_ALGO_NAMES = {"gbm": "gbm", "drf": "drf", "xgboost": "xgboost", "glm": "glm", "deeplearning": "deeplearning",
               "stackedensemble": "stackedensemble", "completion": "completion"}
_EXPLOITATION = {"lr_annealing", "lr_search"}


def _step_alias(sid: str, alias: str) -> bool:
    """StepDefinition.Alias membership of a step id."""
    alias = alias.lower()
    if alias == "all":
        return True
    if alias == "defaults":
        return sid.startswith("def_") or sid == "XRT" or sid.startswith("best_of_family") or sid.startswith("all")
    if alias == "grids":
        return sid.startswith("grid_") or sid == "resume_best_grids"
    if alias in ("exploitation", "optionals"):
        return sid in _EXPLOITATION
    raise ValueError(f"unknown modeling step alias {alias!r}")


def custom_plan(modeling_plan) -> list:
    """``modeling_plan`` (AutoMLBuildSpec.AutoMLBuildModels.modeling_plan, h2o-py forms): a list of
    ``"GBM"`` (every step of the algo), ``("GBM", "defaults"|"grids"|"exploitation"|"all")``,
    ``("GBM", ["def_1", ("grid_1", group, weight), ...])`` or ``{"name": "GBM", "alias": ...}`` /
    ``{"name": "GBM", "steps": [{"id": "def_1", "group": 2, "weight": 10}, ...]}``. Steps keep the
    default group / weight of the TEN_LAYERED plan unless given, and run by (group, definition order)."""
    catalog = _plan()
    out = []

    def add(algo, sid, group=None, weight=None):
        for a, i, g, w in catalog:
            if a == algo and i == sid:
                out.append((a, i, g if group in (None, -1) else int(group), w if weight in (None, -1) else int(weight)))
                return
        raise ValueError(f"no modeling step {sid!r} for {algo}")

    for item in modeling_plan:
        if isinstance(item, dict):
            algo = str(item.get("name", "")).lower()
            alias, steps = item.get("alias"), item.get("steps")
        elif isinstance(item, (list, tuple)):
            algo = str(item[0]).lower()
            alias, steps = (item[1], None) if len(item) > 1 and isinstance(item[1], str) else (None, item[1] if len(item) > 1 else None)
        else:
            algo, alias, steps = str(item).lower(), "all", None
        if algo not in _ALGO_NAMES:
            raise ValueError(f"modeling_plan: unknown algo {algo!r}")
        if steps is None:
            for a, i, g, w in catalog:
                if a == algo and _step_alias(i, alias or "all"):
                    out.append((a, i, g, w))
            continue
        for st in steps:
            if isinstance(st, dict):
                add(algo, st["id"], st.get("group"), st.get("weight"))
            elif isinstance(st, (list, tuple)):
                add(algo, *st)
            else:
                add(algo, str(st))
    order = {id(st): i for i, st in enumerate(out)}
    return sorted(out, key=lambda st: (st[2], order[id(st)]))


def exploitation_weights(steps, ratio: float) -> list:
    """AutoML.distributeExplorationVsExploitationWork: exploration weights stay, the exploitation steps'
    weights are rescaled so they make up ``ratio`` of the total (0 removes them)."""
    if ratio is None or ratio < 0:
        return steps
    if ratio > 1:
        raise ValueError("`exploitation_ratio` must be between 0 and 1.")
    expl = [st for st in steps if st[1] in _EXPLOITATION]
    sum_x = sum(st[3] for st in steps if st[1] not in _EXPLOITATION and st[0] != "stackedensemble")
    sum_e = sum(st[3] for st in expl)
    if not expl or sum_e <= 0:
        return steps
    new_total = int(round(sum_x / (1.0 - ratio))) if ratio < 1 else sum_x + sum_e
    new_e = new_total - sum_x
    return [(a, i, g, int(round(w * new_e / sum_e)) if i in _EXPLOITATION else w) for a, i, g, w in steps]


class AutoML:
    def __init__(self, project_name=None, max_models=None, max_runtime_secs=None, max_runtime_secs_per_model=0,
                 nfolds=5, seed=None, sort_metric="AUTO", include_algos=None, exclude_algos=None,
                 stopping_metric="AUTO", stopping_rounds=3, stopping_tolerance=None, balance_classes=False,
                 class_sampling_factors=None, max_after_balance_size=5.0, keep_cross_validation_predictions=True,
                 keep_cross_validation_models=False, keep_cross_validation_fold_assignment=False, verbosity="warn",
                 exploitation_ratio=-1, modeling_plan=None, preprocessing=None, monotone_constraints=None,
                 export_checkpoints_dir=None):
        self.project_name = project_name or dkv.new_key("AutoML")
        self.max_models = max_models
        self.max_runtime_secs = max_runtime_secs if max_runtime_secs is not None else (0 if max_models else 3600)
        self.per_model = max_runtime_secs_per_model or 0
        self.nfolds = nfolds
        if nfolds not in (0, -1) and int(nfolds) == 1:
            raise ValueError("nfolds set to 1; use nfolds >= 2 or 0 (no cross-validation)")
        self.seed = seed if seed not in (None, -1) else _coll().shared_entropy(1 << 31)
        self.sort_metric = sort_metric
        self.include = [a.lower() for a in include_algos] if include_algos else None
        self.exclude = [a.lower() for a in exclude_algos] if exclude_algos else []
        self.stopping = dict(stopping_metric=stopping_metric, stopping_rounds=stopping_rounds,
                             stopping_tolerance=stopping_tolerance)
        # AutoMLBuildControl: class balancing and CV artefact retention go to every model that has them
        self.balance = dict(balance_classes=bool(balance_classes), class_sampling_factors=class_sampling_factors,
                            max_after_balance_size=max_after_balance_size)
        self.keep_cv = dict(keep_cross_validation_models=bool(keep_cross_validation_models),
                            keep_cross_validation_fold_assignment=bool(keep_cross_validation_fold_assignment))
        self.keep_cv_predictions = bool(keep_cross_validation_predictions)
        self.exploitation_ratio = float(exploitation_ratio if exploitation_ratio is not None else -1)
        if self.exploitation_ratio > 1:
            raise ValueError("`exploitation_ratio` must be between 0 and 1.")
        self.modeling_plan = custom_plan(modeling_plan) if modeling_plan else None
        pre = []
        for st in preprocessing or []:
            t = st.get("type") if isinstance(st, dict) else st
            t = str(t).lower().replace("_", "")
            if t != "targetencoding":
                raise ValueError(f"unknown preprocessing step {st!r} (supported: 'target_encoding')")
            pre.append("target_encoding")
        self.preprocessing = pre
        # AutoMLCustomParameters: monotone_constraints is the one allowed custom algo parameter
        self.algo_params = {"monotone_constraints": monotone_constraints} if monotone_constraints else {}
        self.export_checkpoints_dir = export_checkpoints_dir
        self.models = []
        self.event_log = []
        self.te_model = None

    def _allowed(self, algo):
        name = _ALGO_NAMES[algo]
        if self.include is not None and name not in self.include:
            return False
        return name not in self.exclude

    def _log(self, msg):
        self.event_log.append(dict(timestamp=time.time(), message=msg))

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, leaderboard_frame=None,
              blending_frame=None, fold_column=None, weights_column=None, job: Job | None = None):
        """Run the modeling plan group by group. Time budgets follow the steps' weights: a step gets
        ``remaining_time * weight / remaining_weight`` (ModelingStep weights); ``max_models`` counts
        base models only (SEs are free). Grid steps draw random-discrete points from their space until
        their share runs out, exploitation steps retrain the best GBM with learning-rate annealing and
        search the learning rate of the best XGBoost, the completion step resumes the two best grids,
        and SE steps (best-of-family / all, per group and for GBM-only and XGBoost+GLM subsets) close
        each group."""
        from .parallel import collectives as coll
        from .models import params as P_
        t0 = time.time()
        nrows = training_frame.nrows
        tol = self.stopping["stopping_tolerance"]
        tol = default_stopping_tolerance(nrows) if tol in (None, -1, "AUTO") else float(tol)
        nfolds = int(self.nfolds) if self.nfolds not in (None, -1) else 5
        if blending_frame is not None and self.nfolds in (None, -1):
            nfolds = 0          # blending mode: the SEs stack predictions on the blending frame
        common = dict(nfolds=nfolds if not fold_column else 0, fold_assignment="Modulo",
                      keep_cross_validation_predictions=True, fold_column=fold_column, weights_column=weights_column,
                      **self.keep_cv)
        if self.stopping["stopping_rounds"]:
            common.update(stopping_rounds=self.stopping["stopping_rounds"], stopping_metric=self.stopping["stopping_metric"],
                          stopping_tolerance=tol)
        self._log(f"stopping tolerance {tol:.6g} (adaptive on {nrows} rows)" if self.stopping["stopping_tolerance"] in
                  (None, -1, "AUTO") else f"stopping tolerance {tol} (user)")
        cat = self._category(training_frame, y)
        self.blending_frame = blending_frame
        if self.preprocessing:
            training_frame, validation_frame, x, common = self._target_encoding(
                training_frame, validation_frame, x, y, fold_column, weights_column, nfolds, common)
        plan = self.modeling_plan if self.modeling_plan is not None else _plan()
        steps = [st for st in plan if st[0] in ("completion", "stackedensemble") or self._allowed(st[0])]
        steps = exploitation_weights(steps, self.exploitation_ratio)
        total_w = float(sum(st[3] for st in steps)) or 1.0
        used_w = 0.0
        rng = np.random.default_rng(self.seed)
        self._grids = {}
        n_base = lambda: sum(1 for m in self.models if m.algo != "stackedensemble")  # noqa: E731

        def time_left():
            return self.max_runtime_secs - (time.time() - t0) if self.max_runtime_secs > 0 else float("inf")

        def models_left():
            return (self.max_models - n_base()) if self.max_models else 1 << 30

        def can_go(ignore_count=False):
            return coll.agree(time_left() > 0 and (ignore_count or models_left() > 0))

        def algo_params(algo):
            """build-control and custom parameters, for the algos whose schema has them"""
            sch = P_.schema(algo) or {}
            extra = {}
            if cat in ("Binomial", "Multinomial") and self.balance["balance_classes"]:
                extra.update({k: v for k, v in self.balance.items() if k in sch and v is not None})
            extra.update({k: v for k, v in self.algo_params.items() if k in sch})
            return extra

        def run(algo, name, p, share, exploit=False):
            if algo != "stackedensemble" and not can_go(exploit and self.exploitation_ratio > 0):
                return None
            p = dict(p, **common, **algo_params(algo))
            if self.per_model:
                p["max_runtime_secs"] = self.per_model
            elif self.max_runtime_secs > 0:
                p["max_runtime_secs"] = coll.broadcast_object(max(1.0, min(share, time_left())))
            mid = f"{name}_AutoML_{self.project_name}"
            try:
                m = builder.train(algo, p, x, y, training_frame, validation_frame, job, mid)
                self._register(m, mid)
                return m
            except Exception as e:  # noqa: BLE001 - AutoML logs and moves on (EventLog)
                self._log(f"{mid} failed: {e!r}")
                return None

        counters = {}
        last_group = 0
        self.executed_steps = []      # (algo family, step id, group, weight) of the steps that built models
        self.training_frame_ref = training_frame      # predict_time_per_row_ms without a leaderboard frame
        self.start_epoch = t0
        for algo, sid, group, w in steps:
            share = (time_left() * w / max(total_w - used_w, 1e-9)) if self.max_runtime_secs > 0 else float("inf")
            used_w += w
            if w <= 0:             # ModelingStep.canRun: no work allocated (e.g. exploitation_ratio=0)
                continue
            if algo == "stackedensemble":
                # SEs do not count against the budget: they close every group that trained base models
                # (and the final group always runs)
                if (self._allowed("stackedensemble") and len(self.models) >= 2 and self.models[0].info.response
                        and (group <= last_group or group == 10)):
                    n_se = len(self.models)
                    self._se_step(sid, x, y, training_frame, validation_frame, job)
                    if len(self.models) > n_se:
                        self.executed_steps.append(("StackedEnsemble", sid, group, w))
                continue
            if not can_go(sid in _EXPLOITATION and self.exploitation_ratio > 0):
                continue
            n_before = len(self.models)
            fam = dict(gbm="GBM", xgboost="XGBoost", glm="GLM", drf="DRF", deeplearning="DeepLearning").get(algo, algo)
            if algo == "completion":
                self._resume_best_grids(run, rng, share)
                continue
            if sid.startswith("def_") or sid == "XRT":
                counters[fam] = counters.get(fam, 0) + 1
                name = "XRT_1" if sid == "XRT" else f"{fam}_{counters[fam]}"
                run(algo, name, _defaults(algo, sid, self.seed, cat), share)
            elif sid.startswith("grid_"):
                cap = None if not self.max_models else max(1, int(round(models_left() * w / max(total_w - used_w + w, 1e-9))))
                self._grid_step(algo, fam, sid, run, rng, share, cap)
            elif sid == "lr_annealing":
                best = self._best_of(["gbm"])
                if best is not None:
                    p = {k: v for k, v in best.params.items() if k in _defaults("gbm", "def_1", self.seed, cat)}
                    run("gbm", "GBM_lr_annealing_selection_model_1", dict(p, learn_rate_annealing=0.99), share, exploit=True)
            elif sid == "lr_search":
                best = self._best_of(["xgboost"])
                if best is not None:
                    base = {k: v for k, v in best.params.items() if k in _defaults("xgboost", "def_1", self.seed, cat)}
                    sti = int(base.get("score_tree_interval") or 5)
                    for j, lr in enumerate((0.5, 0.2, 0.1, 0.05, 0.02, 0.01, 0.005, 0.002, 0.001, 0.0005)):
                        if not can_go(self.exploitation_ratio > 0):
                            break
                        run("xgboost", f"XGBoost_lr_search_selection_model_{j + 1}",
                            dict(base, learn_rate=lr, score_tree_interval=(j + 1) * sti), share / 10, exploit=True)
            if len(self.models) > n_before:
                last_group = group
                self.executed_steps.append((fam if algo != "completion" else "completion", sid, group, w))
        self.stop_epoch = time.time()
        self.leaderboard_frame = leaderboard_frame
        if not self.keep_cv_predictions:
            # the holdout predictions were kept for the SEs only (AutoML keep_cross_validation_predictions=False)
            for m in self.models:
                fid = m.output.pop("cross_validation_holdout_predictions_frame_id", None) if isinstance(m.output, dict) else None
                if fid:
                    dkv.remove(fid)
        dkv.put(self.project_name, self)
        return self

    def _register(self, m, mid):
        if self.te_model is not None and m.algo != "stackedensemble":
            m.preprocessors = [self.te_model]       # predict / score raw frames through the TE preprocessor
            m.output["preprocessors"] = [self.te_model.key]
        self.models.append(m)
        self._log(f"built {mid}")
        if self.export_checkpoints_dir:
            import os
            from .persist import save_model
            os.makedirs(self.export_checkpoints_dir, exist_ok=True)
            save_model(m, self.export_checkpoints_dir, force=True)

    def _target_encoding(self, fr, valid, x, y, fold_column, weights_column, nfolds, common):
        """preprocessing=["target_encoding"] (ai/h2o/automl/preprocessing/TargetEncoding.java): encode the
        categorical predictors with cardinality >= 25 whose rows-per-level exceed the blending inflection
        point (5); with CV the encoder uses KFold leakage handling on the user fold column or a Modulo fold
        column ``<y>_te_fold``, which the models then train on (nfolds=0). Models keep the encoder as a
        preprocessor, so predictions on raw frames are encoded the same way."""
        from .frame import Column
        from .models import builder as B  # noqa: N812
        names = list(x) if x is not None else [n for n in fr.names if n not in (y, fold_column, weights_column)]
        te_cols = []
        for n in names:
            if fr.type(n) == "enum":
                card = len(fr._col(n).domain or [])
                if card >= 25 and fr.nrows / max(card, 1) > 5:
                    te_cols.append(n)
        if not te_cols:
            self._log("target_encoding: no categorical column qualifies (cardinality >= 25)")
            return fr, valid, x, common
        tp = dict(blending=True, inflection_point=5, smoothing=10, noise=0.0, keep_original_categorical_columns=False,
                  seed=self.seed)
        train = fr
        fcol = fold_column
        if common.get("nfolds", 0) > 1 or fold_column:
            tp["data_leakage_handling"] = "KFold"
            if not fcol:
                fcol = f"{y}_te_fold"
                import torch
                from .frame import engine_device
                n = fr.nrows
                folds = torch.arange(n, dtype=torch.float64, device=engine_device()) % nfolds   # Modulo
                train = fr.cbind(type(fr)._from_columns([Column(fcol, "int", folds)]))
            tp["fold_column"] = fcol
        self.te_model = B.train("targetencoder", tp, te_cols + ([fcol] if fcol else []), y, train, None, None,
                                f"TargetEncoding_AutoML_{self.project_name}")
        self._log(f"target_encoding: encoded {te_cols} (experimental in the reference: no MOJO for these models)")
        enc = self.te_model.transform(train, as_training=True)
        x2 = [n for n in names if n not in te_cols] + [n for n in enc.names if n.endswith("_te")]
        common = dict(common)
        if fcol:
            common.update(fold_column=fcol, nfolds=0)
        v2 = self.te_model.transform(valid) if valid is not None else None
        return enc, v2, x2, common


    @staticmethod
    def _category(fr, y):
        if y is None:
            return "Regression"
        if fr.type(y) == "enum":
            return "Binomial" if len(fr._col(y).domain) == 2 else "Multinomial"
        return "Regression"

    def _grid_step(self, algo, fam, sid, run, rng, share, cap=None):
        """Random-discrete grid search (RandomDiscreteValueSearchCriteria) within the step's time share
        (or, under a model-count budget, its weight share of the remaining models)."""
        space = _grid_space(algo, sid)
        g = self._grids.setdefault((algo, sid), dict(n=0, space=space, algo=algo, fam=fam, sid=sid, seen=set()))
        t_end = time.time() + share
        tries = 0
        while time.time() < t_end and tries < 200:
            tries += 1
            hp = {k: v[int(rng.integers(len(v)))] for k, v in space.items()}
            key = repr(sorted(hp.items()))
            if key in g["seen"]:
                continue
            g["seen"].add(key)
            g["n"] += 1
            m = run(algo, f"{fam}_{sid}_model_{g['n']}", dict(_grid_base(algo, self.seed), **hp), max(1.0, t_end - time.time()))
            if m is None and (self.max_models and sum(1 for x in self.models if x.algo != "stackedensemble") >= self.max_models):
                break
            if cap is not None and g["n"] >= cap:
                break

    def _resume_best_grids(self, run, rng, share):
        """completion step: keep searching the two grids whose best model ranks highest."""
        if not self._grids:
            return
        cat = self.models[0].model_category if self.models else "Regression"
        metric = self._sort_key(cat)

        def best_of(gk):
            fam, sid = self._grids[gk]["fam"], self._grids[gk]["sid"]
            ms = [m for m in self.models if m.key.startswith(f"{fam}_{sid}_model_")]
            vals = [_metric_of(m, metric) for m in ms]
            vals = [v for v in vals if not math.isnan(v)]
            if not vals:
                return float("nan")
            return max(vals) if metric in _DESC else min(vals)
        ranked = sorted(self._grids, key=lambda k: (math.isnan(best_of(k)),
                                                   -best_of(k) if metric in _DESC else best_of(k)))
        for gk in ranked[:2]:
            g = self._grids[gk]
            self._grid_step(g["algo"], g["fam"], g["sid"], run, rng, share / 2,
                            None if not self.max_models else g["n"] + 1)

    def _best_of(self, algos):
        cat = self.models[0].model_category if self.models else "Regression"
        metric = self._sort_key(cat)
        best, bv = None, float("nan")
        for m in self.models:
            if m.algo in algos:
                v = _metric_of(m, metric)
                if best is None or self._better(v, bv, metric):
                    best, bv = m, v
        return best

    def _se_step(self, sid, x, y, fr, valid, job):
        """StackedEnsembleStepsProvider: best_of_family_* (best model of each family) and all_* (every
        base model so far); ``_gbm`` restricts to GBMs, ``_xglm`` to XGBoost + GLM, ``best_N`` to the top
        20. A SE is only built when its base set differs from every SE built before."""
        cat = self.models[0].model_category
        metric = self._sort_key(cat)
        blend = getattr(self, "blending_frame", None)
        base = [m for m in self.models if m.algo != "stackedensemble" and
                (blend is not None or getattr(m, "cv_holdout", None) is not None)]
        if sid.endswith("_gbm"):
            base = [m for m in base if m.algo == "gbm"]
        elif sid.endswith("_xglm"):
            base = [m for m in base if m.algo in ("xgboost", "glm")]
        if sid.startswith("best_of_family"):
            best = {}
            for m in base:
                fam = "xrt" if m.key.startswith("XRT") else m.algo
                v = _metric_of(m, metric)
                if fam not in best or self._better(v, best[fam][1], metric):
                    best[fam] = (m, v)
            ms, kind = [b[0] for b in best.values()], "BestOfFamily"
        elif sid == "best_N":
            ranked = sorted(base, key=lambda m: (math.isnan(_metric_of(m, metric)),
                                                 -_metric_of(m, metric) if metric in _DESC else _metric_of(m, metric)))
            ms, kind = ranked[:20], "Best20"
        else:
            ms, kind = base, "AllModels"
        if len(ms) < 2:
            return
        keyset = frozenset(m.key for m in ms)
        done = getattr(self, "_se_sets", set())
        if keyset in done:
            return
        done.add(keyset)
        self._se_sets = done
        n = sum(1 for m in self.models if m.algo == "stackedensemble" and f"_{kind}_" in m.key) + 1
        suffix = {"_gbm": "_GBM", "_xglm": "_XGBoost_GLM"}.get(sid[sid.rfind("_"):], "") if not sid[-1].isdigit() else ""
        mid = f"StackedEnsemble_{kind}{suffix}_{n}_AutoML_{self.project_name}"
        try:
            # StackedEnsembleStepsProvider.setMetalearnerParameters: the metalearner is cross-validated
            # with the AutoML nfolds, and its out-of-fold metrics are what the leaderboard ranks
            sp = dict(base_models=[m.key for m in ms], seed=self.seed, keep_levelone_frame=True)
            if blend is not None:
                sp["blending_frame"] = blend
            else:
                sp.update(metalearner_nfolds=self.nfolds, metalearner_fold_assignment="Modulo")
            if cat in ("Binomial", "Multinomial"):
                sp["metalearner_transform"] = "Logit"
            se = builder.train("stackedensemble", sp, x, y, fr, valid, job, mid)
            self._register(se, mid)
        except Exception as e:  # noqa: BLE001
            self._log(f"{mid} failed: {e!r}")

    def _sort_key(self, cat):
        s = str(self.sort_metric).lower()
        return _DEFAULT_SORT.get(cat, "mse") if s == "auto" else s

    @staticmethod
    def _better(a, b, metric):
        if math.isnan(b):
            return True
        return a > b if metric in _DESC else a < b

    def leaderboard_rows(self):
        if not self.models:
            return [], []
        cat = self.models[0].model_category
        key = self._sort_key(cat)
        cols = {"Binomial": ["auc", "logloss", "aucpr", "mean_per_class_error", "rmse", "mse"],
                "Multinomial": ["mean_per_class_error", "logloss", "rmse", "mse"],
                "Regression": ["mean_residual_deviance", "rmse", "mse", "mae", "rmsle"]}.get(cat, ["mse"])
        if key in cols:
            cols.remove(key)
        cols = [key] + cols
        lb = self.leaderboard_frame
        rows = []
        for m in self.models:
            if lb is not None:
                perf = m.model_performance(lb)
                vals = {c: _metric_of_dict(perf, c) for c in cols}
            else:
                vals = {c: _metric_of(m, c) for c in cols}
            rows.append(dict(model_id=m.key, **vals))
        desc = key in _DESC
        rows.sort(key=lambda r: (math.isnan(r[key]), -r[key] if desc else r[key]))
        return rows, ["model_id"] + cols

    @property
    def leader(self):
        rows, _ = self.leaderboard_rows()
        return dkv.get(rows[0]["model_id"]) if rows else None


def _metric_of_dict(perf, metric):
    key = {"auc": "AUC", "aucpr": "pr_auc", "logloss": "logloss", "mse": "MSE", "rmse": "RMSE", "mae": "mae",
           "rmsle": "rmsle", "mean_per_class_error": "mean_per_class_error",
           "mean_residual_deviance": "mean_residual_deviance"}.get(metric, metric)
    v = perf.get(key) if perf else None
    if v is None and key == "mean_residual_deviance" and perf:
        v = perf.get("MSE")
    return float("nan") if v is None else float(v)


def leaderboard_frame(models, frame=None, sort_metric="AUTO"):
    """``makeLeaderboard`` (h2o-automl ``Leaderboard.java``): rank arbitrary models on a frame (or their
    own training/cross-validation metrics) with the AutoML leaderboard columns."""
    import numpy as np
    import torch
    from .frame import Column, H2OFrame, engine_device
    lb = AutoML.__new__(AutoML)
    lb.models = list(models)
    lb.sort_metric = sort_metric
    lb.leaderboard_frame = frame
    rows, cols = lb.leaderboard_rows()
    out = [Column("model_id", "string", strings=np.array([r["model_id"] for r in rows], dtype=object))]
    for c in cols[1:]:
        out.append(Column(c, "real", torch.tensor([r[c] for r in rows], dtype=torch.float64, device=engine_device())))
    return H2OFrame._from_columns(out)
