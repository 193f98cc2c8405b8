"""ModelBuilder front-end: frame -> tensors -> trainer, cross-validation, model registry (reference:
``hex/ModelBuilder.java`` (init/validation, ``computeCrossValidation``, fold assignment),
``hex/CVModelBuilder.java``, ``hex/ModelBuilderHelper.java``, ``water/api/ModelBuildersHandler.java``).

Every algorithm registers an :class:`AlgoSpec` (trainer class, supervised?, defaults). ``train``
resolves predictors/response/special columns exactly like ``ModelBuilder.init`` (ignored columns,
constant columns dropped, response domain, weights/offset/fold columns), builds the ``[F, N]``
float32 device matrix, runs N-fold CV when asked (fold models + holdout predictions -> the
``cross_validation_metrics`` and ``cross_validation_metrics_summary``), then trains the main model.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import metrics as mm
from ..core import dkv
from ..core.job import Job
from .base import DataInfo, Model, make_key

REGISTRY: dict = {}


@dataclass
class AlgoSpec:
    name: str
    trainer: type
    supervised: bool = True
    defaults: dict = field(default_factory=dict)
    classification_only: bool = False
    regression_only: bool = False
    needs_response_optional: bool = False   # e.g. isolation forest accepts an optional label


# Trainers that reduce their sufficient statistics over row-sharded tensors (histograms, Gram, centroid
# sums, gradients, class counts, exact order statistics, all-to-all range partitions): under a multi-rank
# cloud they train on the local shard. That is every trainer that reads rows; the rest (grep, generic)
# get the gathered rows and run replicated (identical on every rank).
DISTRIBUTED = {"gbm", "drf", "xgboost", "glm", "kmeans", "deeplearning", "naivebayes", "pca", "quantile",
               "isolationforest", "extendedisolationforest", "svd", "targetencoder", "gam", "anovaglm",
               "modelselection", "upliftdrf", "dt", "glrm", "rulefit", "word2vec", "isotonicregression",
               "coxph", "aggregator", "psvm", "infogram", "stackedensemble"}


def register(name, trainer, supervised=True, defaults=None, **kw):
    REGISTRY[name] = AlgoSpec(name, trainer, supervised, dict(defaults or {}), **kw)


COMMON = ("nfolds", "fold_assignment", "fold_column", "keep_cross_validation_predictions", "keep_cross_validation_models",
          "keep_cross_validation_fold_assignment", "weights_column", "offset_column", "ignored_columns",
          "ignore_const_cols", "model_id", "training_frame", "validation_frame", "response_column", "x", "y",
          "custom_metric_func", "calibrate_model", "calibration_frame", "calibration_method")


def _resolve_names(fr, cols):
    if cols is None:
        return None
    if isinstance(cols, (str, int)):
        cols = [cols]
    out = []
    for c in cols:
        out.append(fr.names[c] if isinstance(c, int) else c)
    return out


def _classification_requested(algo, params) -> bool:
    d = str(params.get("distribution") or "").lower()
    fam = str(params.get("family") or "").lower()
    return d in ("bernoulli", "multinomial", "quasibinomial", "modified_huber") or fam in ("binomial", "multinomial",
                                                                                           "quasibinomial", "ordinal",
                                                                                           "fractionalbinomial")


def prepare(algo: str, params: dict, x=None, y=None, training_frame=None):
    """Resolve columns and build the DataInfo (``ModelBuilder.init``)."""
    spec = REGISTRY[algo]
    fr = training_frame
    y = _resolve_names(fr, y)
    y = y[0] if y else None
    # the target encoder reads its fold column as data (KFold leakage handling), it does no CV of its own
    special = {params.get("weights_column"), params.get("offset_column"),
               params.get("fold_column") if algo != "targetencoder" else None, y}
    special.discard(None)
    ignored = set(_resolve_names(fr, params.get("ignored_columns")) or [])
    if x is None:
        xs = [n for n in fr.names if n not in special and n not in ignored]
    else:
        xs = [n for n in _resolve_names(fr, x) if n not in special]
    xs = [n for n in xs if fr.type(n) != "string" or algo in ("word2vec", "targetencoder")]
    if params.get("ignore_const_cols", True) and fr.nrows > 1:
        keep = []
        sharded = fr._shard is not None
        for n in xs:
            c = fr._col(n)
            if c.type == "enum":
                v = c.data
                u = torch.unique(v)
                if sharded:                      # distinct codes over every shard
                    from ..parallel import dframe
                    u = torch.unique(dframe.gather_tensor(u.cpu(), bounded=True))
                if int(u.numel()) > 1:
                    keep.append(n)
            elif c.type == "string":
                keep.append(n)
            else:
                from ..parallel import dframe
                m = dframe.moments(c.values(), sharded)     # compressed columns stay encoded
                if m["n"] > 0 and (m["max"] != m["min"] or m["nas"] > 0):
                    keep.append(n)
        xs = keep
    iscat = np.array([1 if fr.type(n) == "enum" else 0 for n in xs], dtype=np.int32)
    doms = [list(fr._col(n).domain) if fr.type(n) == "enum" else None for n in xs]
    rdom = None
    if y is not None:
        yc = fr._col(y)
        if yc.type == "enum":
            rdom = list(yc.domain)
        elif _classification_requested(algo, params) or spec.classification_only:
            from ..frame import _num_to_enum
            rdom = list(_num_to_enum(yc, fr._shard is not None).domain)
    info = DataInfo(xs, iscat, doms, y, rdom, params.get("weights_column"), params.get("offset_column"),
                    params.get("fold_column"))
    return info


def tensors(fr, info: DataInfo, device=None):
    X, offset = fr.model_matrix(info, device=device)
    yv = fr.response_tensor(info, device=X.device) if info.response else None
    w = fr.weights_tensor(info, device=X.device)
    return X, yv, w, offset


def _fold_ids(fr, info, params, n, seed):
    """Fold id of every local row (``FoldAssignment``). Assignments are defined on the GLOBAL row index,
    so a row-sharded training gets exactly the folds of the single-process run."""
    from ..parallel import dframe
    sh = fr._shard
    off, n_glob = (sh.offset, sh.n_global) if sh is not None else (0, n)
    k = int(params.get("nfolds") or 0)
    if info.fold and info.fold in fr.names:
        v = fr._col(info.fold).as_float()
        u = dframe.global_unique(v) if sh is not None else torch.unique(v[~torch.isnan(v)])
        return torch.bucketize(v, u).long(), int(u.numel())
    scheme = str(params.get("fold_assignment") or "AUTO").lower()
    if scheme == "modulo":
        return torch.arange(off, off + n) % k, k
    rng = np.random.default_rng(seed & 0xFFFFFFFF)
    if scheme == "stratified" and info.response is not None:
        yt = fr.response_tensor(info, device=torch.device("cpu"))
        yv = (dframe.gather_tensor(yt) if sh is not None else yt).numpy()
        fold = np.zeros(n_glob, dtype=np.int64)
        for cls in np.unique(yv[~np.isnan(yv)]):
            idx = np.nonzero(yv == cls)[0]
            rng.shuffle(idx)
            fold[idx] = np.arange(len(idx)) % k
        return torch.from_numpy(fold[off:off + n]), k
    return torch.from_numpy(rng.integers(0, k, n_glob)[off:off + n]), k


def _seed_of(params):
    s = params.get("seed")
    if s is None or int(s) == -1:
        from ..parallel import collectives as coll
        return coll.shared_entropy(1 << 62)
    return int(s)


def train(algo: str, params: dict, x=None, y=None, training_frame=None, validation_frame=None, job: Job | None = None,
          model_id: str | None = None) -> Model:
    spec = REGISTRY[algo]
    _validate(spec, algo, params)
    p = dict(spec.defaults)
    p.update({k: v for k, v in params.items() if v is not None})
    if algo == "grep":                          # raw-text scan: no DataInfo / device tensors
        m = spec.trainer(p).fit_text(training_frame, model_id or p.get("model_id"))
        m.algo = "grep"
        dkv.put(m.key, m)
        return m
    if algo == "generic":                       # import a MOJO: no training frame involved
        m = spec.trainer(p).fit(model_key=model_id or p.get("model_id"))
        m.algo = "generic"
        dkv.put(m.key, m)
        return m
    if algo == "word2vec" and p.get("pre_trained") is not None:
        # Word2Vec pre_trained: the model is the given [word, v1..vD] frame (no training)
        m = spec.trainer(p).from_pretrained(p["pre_trained"], model_id or p.get("model_id"))
        dkv.put(m.key, m)
        return m
    if spec.supervised and y is None and not spec.needs_response_optional:
        raise ValueError(f"{algo} needs a response column y")
    fr = training_frame
    if fr is None:
        raise ValueError("training_frame is required")
    if algo == "gam" and p.get("gam_columns") and x is not None:
        # GAM.java: the smoothed columns are predictors whether or not x lists them
        gc = [c for g in p["gam_columns"] for c in ([g] if isinstance(g, str) else g)]
        x = list(x) + [c for c in gc if c not in x]
    from ..parallel import collectives as coll, dframe
    import contextlib
    mode = contextlib.ExitStack()
    if coll.world_active() and not coll.is_dist():
        # nested inside a replicated computation (e.g. a metalearner fit inside a gathered trainer)
        fr = dframe.gather_frame(fr)
        validation_frame = dframe.gather_frame(validation_frame)
    elif coll.world_active():
        if algo in DISTRIBUTED:
            fr = dframe.shard_frame(fr)
            validation_frame = dframe.shard_frame(validation_frame) if validation_frame is not None else None
        else:
            fr = dframe.gather_frame(fr)
            validation_frame = dframe.gather_frame(validation_frame)
            mode.enter_context(coll.replicated())
    from ..utils import memory
    memory.pressure_check()
    with mode:
        return memory.with_backpressure(_train, spec, algo, p, x, y, fr, validation_frame, job, model_id)


_EXTRA = {}


def extension_params(algo) -> set:
    """Parameters a trainer accepts beyond the h2o-py schema (its own defaults: engine extensions such
    as ``compute_dtype``, ``seed`` where the reference has none, ...)."""
    if algo not in _EXTRA:
        spec = REGISTRY[algo]
        extra = set(COMMON) | set(spec.defaults) | {"model_id", "max_categorical_levels"}
        try:
            extra |= set(getattr(spec.trainer({}), "p", {}) or {})
        except Exception:  # noqa: BLE001 - trainers that need arguments to construct
            pass
        _EXTRA[algo] = extra
    return _EXTRA[algo]


def _validate(spec, algo, params):
    """ModelBuilder.init: unknown / unsupported parameters are errors, never silent no-ops."""
    from . import params as pv
    pv.validate(algo, params, extension_params(algo))


def _train(spec, algo, p, x, y, fr, validation_frame, job, model_id):
    info = prepare(algo, p, x, y, fr)
    if not info.x:
        raise ValueError("no usable predictor columns")
    from .adapt import balance_indices, fit_adapter
    adapter, fr2, x2 = fit_adapter(algo, p, fr, list(info.x), info.response)
    if adapter:
        fr = fr2
        info = prepare(algo, p, x2, y, fr)
        if validation_frame is not None:
            validation_frame = adapter.apply(validation_frame)
    X, yv, w, off = tensors(fr, info)
    balance = None
    if p.get("balance_classes") and info.response_domain is not None and yv is not None:
        from ..parallel import collectives as coll
        idx, prior, mdist = balance_indices(p, yv, len(info.response_domain), coll.row_offset(X.shape[1]))
        X = X[:, idx].contiguous()
        yv = yv[idx]
        w = None if w is None else w[idx]
        off = None if off is None else off[idx]
        balance = (prior, mdist)
    if yv is not None and info.response_domain is None and spec.classification_only:
        raise ValueError(f"{algo} needs a categorical response")
    valid = None
    if validation_frame is not None:
        Xv, yvv, wv, ov = tensors(validation_frame, info, device=X.device)
        vrc = p.get("validation_response_column")
        if vrc and yvv is None:
            # IsolationForest validation_response_column: labelled anomalies of the validation frame
            if vrc not in validation_frame.names:
                raise ValueError(f"validation_response_column {vrc!r} is not in the validation frame")
            col = validation_frame._col(vrc)
            if col.domain is None or len(col.domain) != 2:
                raise ValueError("validation_response_column must be a binary categorical column")
            yvv = col.data.to(X.device).float()
            yvv = torch.where(yvv < 0, torch.full_like(yvv, float("nan")), yvv)
            p["_valid_domain"] = list(col.domain)
        valid = (Xv, yvv, wv, ov)
    mid = model_id or p.get("model_id") or make_key(algo)
    seed = _seed_of(p)
    p["seed"] = seed
    t0 = time.time()
    nfolds = int(p.get("nfolds") or 0)
    cv_out = None
    if algo != "targetencoder" and (nfolds > 1 or (info.fold and info.fold in fr.names)):
        cv_out = _cross_validate(spec, p, fr, info, X, yv, w, off, seed, mid, job)
    tp = {k: v for k, v in p.items() if k not in COMMON}
    if cv_out is not None and int(p.get("stopping_rounds") or 0) > 0:
        # ModelBuilder.cv_computeAndSetOptimalParameters: the main model trains for the fold models'
        # average early-stopped length, without early stopping of its own
        lens = cv_out.pop("_cv_lengths", [])
        if lens and algo in ("gbm", "drf", "xgboost"):
            tp["ntrees"] = max(1, int(round(float(np.mean(lens)))))
            tp["stopping_rounds"] = 0
        elif lens and algo == "deeplearning":
            tp["epochs"] = float(np.mean(lens))
            tp["stopping_rounds"] = 0
    if cv_out is not None:
        cv_out.pop("_cv_lengths", None)
    if cv_out is not None and float(tp.get("max_runtime_secs") or 0) > 0:
        tp["max_runtime_secs"] = max(1e-3, float(tp["max_runtime_secs"]) - (time.time() - t0))
    tr = spec.trainer(tp)
    tr.job = job
    if algo == "word2vec":
        tr.strings = fr._col(info.x[0]).to_numpy()
    model = tr.fit(X, yv, w, off, info, valid, mid) if yv is not None or not spec.supervised else tr.fit(X, yv, w, off, info, valid, mid)
    model.params.update({k: p.get(k) for k in COMMON if k in p and k not in ("training_frame", "validation_frame", "x", "y",
                                                                              "calibration_frame")})
    if adapter:
        model.adapter = adapter
    if balance is not None:
        model.output["prior_class_distrib"], model.output["model_class_distrib"] = balance
    model.output["names"] = info.x + ([info.response] if info.response else [])
    model.output["response_column_name"] = info.response
    model.output["domains"] = info.domains
    model.output["training_frame"] = fr.frame_id
    if validation_frame is not None:
        model.output["validation_frame"] = validation_frame.frame_id
    if cv_out is not None:
        model.cv_holdout = cv_out.pop("_cv_holdout", None)
        model.cv_holdout_sharded = coll_is_dist()       # holdout rows are this rank's shard
        model.output.update(cv_out)
    if p.get("custom_metric_func") and yv is not None:
        _custom_metric(model, p["custom_metric_func"], X, yv, w, off, "training_metrics")
        if valid is not None:
            _custom_metric(model, p["custom_metric_func"], *valid, "validation_metrics")
    model.algo = algo
    if p.get("calibrate_model") or p.get("calibration_frame") is not None:
        _calibrate(model, p, job)
    model.output["run_time_ms"] = int((time.time() - t0) * 1000)
    dkv.put(model.key, model)
    if p.get("export_checkpoints_dir"):          # ModelBuilder export_checkpoints_dir: persist every final model
        from ..persist import save_model
        save_model(model, p["export_checkpoints_dir"], force=True)
    return model


def coll_is_dist():
    from ..parallel import collectives as coll
    return coll.is_dist()


def _calibrate(model, p, job):
    """Post-hoc probability calibration (``hex/tree/CalibrationHelper.java``): Platt scaling = a binomial GLM
    (lambda 0) on p0 of the calibration frame, isotonic regression = a monotone fit of the response on p1.
    Predictions then carry ``cal_p0`` / ``cal_p1``."""
    from ..frame import Column, H2OFrame
    cf = p.get("calibration_frame")
    if isinstance(cf, str):
        cf = dkv.get(cf)
    if not p.get("calibrate_model"):
        return                                   # the reference warns: frame given, calibration not requested
    if model.model_category != "Binomial":
        raise ValueError("Model calibration is only currently supported for binomial models.")
    if cf is None:
        raise ValueError("Calibration frame was not specified.")
    method = str(p.get("calibration_method") or "AUTO").lower().replace("_", "")
    iso = method in ("isotonicregression", "isotonic")
    X, off = cf.model_matrix(model.info, device=model.device)
    P = model.score_tensor(X, off).double()
    y = cf.response_tensor(model.info, device=P.device).double()
    cols = [Column("p", "real", (P[:, 1] if iso else P[:, 0]).contiguous()),
            Column("response", "real", y) if iso else
            Column("response", "enum", y.nan_to_num(-1).int(), domain=list(model.info.response_domain))]
    wname = model.info.weights
    if wname:
        cols.append(Column("weights", "real", cf._col(wname).as_float().double()))
    calib_in = H2OFrame._from_columns(cols)
    cp = dict(weights_column="weights") if wname else {}
    if iso:
        cm = train("isotonicregression", dict(cp, out_of_bounds="clip"), ["p"], "response", calib_in, None, job)
    else:
        cm = train("glm", dict(cp, family="binomial", lambda_=0.0), ["p"], "response", calib_in, None, job)
    model.set_calibration_model(cm)


def _custom_metric(model, ref, X, y, w, off, which):
    """custom_metric_func (hex/CustomMetric.java): evaluated on the model's predictions in the reference
    row layout ([label, p0, p1, ...] for classifiers, [value] otherwise) and stored in the metrics."""
    from .. import udf
    mets = model.output.get(which)
    if mets is None:
        return
    P = model.score_tensor(X, off).double()
    if P.dim() == 2:
        if P.shape[1] == 2 and model.default_threshold() is not None:
            lab = (P[:, 1] >= float(model.default_threshold())).double()
        else:
            lab = P.argmax(1).double()
        rows = torch.cat([lab[:, None], P], 1)
    else:
        rows = P[:, None]
    from ..parallel import collectives as coll
    # map/reduce per shard; only the small metric states travel (gathered in rank order and reduced with the
    # user's reduce, as MRTask reduces CMetricFunc states across nodes) — no row gather
    st = udf.custom_metric_state(ref, rows.cpu().numpy(), y.double().cpu().numpy(),
                                 None if w is None else w.double().cpu().numpy(),
                                 None if off is None else off.double().cpu().numpy(), model)
    states = coll.all_gather_object(None if st is None else [float(v) for v in st]) if coll.is_dist() else [st]
    name, _ = udf.resolve(ref)
    mets["custom_metric_name"] = name
    mets["custom_metric_value"] = udf.custom_metric_finish(ref, states)


def _cross_validate(spec, p, fr, info, X, yv, w, off, seed, mid, job):
    N = X.shape[1]
    fold, k = _fold_ids(fr, info, p, N, seed)
    fold = fold.to(X.device)
    models, holdout = [], None
    fold_metrics = []
    cat = "Unsupervised" if info.response is None else ("Regression" if info.response_domain is None else
                                                         ("Binomial" if len(info.response_domain) == 2 else "Multinomial"))
    for i in range(k):
        tr_m = fold != i
        ho_m = ~tr_m
        if int(ho_m.sum()) == 0 or int(tr_m.sum()) == 0:
            continue
        sub = lambda t, m: None if t is None else (t[:, m] if t.dim() == 2 else t[m])  # noqa: E731
        ps = {kk: vv for kk, vv in p.items() if kk not in COMMON}
        if float(ps.get("max_runtime_secs") or 0) > 0:
            # the whole CV procedure (k fold models + the main model) shares the model's time budget
            ps["max_runtime_secs"] = float(ps["max_runtime_secs"]) / (k + 1)
        trainer = spec.trainer(ps)
        trainer.job = job
        # ModelBuilder.cv_makeFramesAndBuilders: a fold model validates (and early-stops) on its holdout
        ho_valid = None
        if int(p.get("stopping_rounds") or 0) > 0 and yv is not None:
            ho_valid = (sub(X, ho_m).contiguous(), sub(yv, ho_m), sub(w, ho_m), sub(off, ho_m))
        m = trainer.fit(sub(X, tr_m).contiguous(), sub(yv, tr_m), sub(w, tr_m), sub(off, tr_m), info, ho_valid,
                        f"{mid}_cv_{i + 1}")
        models.append(m)
        P = m.score_tensor(sub(X, ho_m).contiguous(), sub(off, ho_m))
        if holdout is None:
            holdout = torch.zeros((N,) + tuple(P.shape[1:]), dtype=P.dtype, device=P.device)
        holdout[ho_m] = P
        if yv is not None:
            fold_metrics.append(m.metrics_for(sub(X, ho_m).contiguous(), sub(yv, ho_m), sub(w, ho_m), sub(off, ho_m)))
        if p.get("keep_cross_validation_models", True):
            dkv.put(m.key, m)
    out = dict(cross_validation_models=[m.key for m in models] if p.get("keep_cross_validation_models", True) else None)
    out["_cv_lengths"] = [float(m.output.get("ntrees") or m.output.get("epochs") or 0) for m in models
                          if (m.output.get("ntrees") or m.output.get("epochs"))]
    if yv is not None and holdout is not None:
        cvm = mm.make_metrics(cat, yv, holdout, w, info.response_domain,
                              labels=models[0].predict_labels(holdout) if models else None)
        out["cross_validation_metrics"] = cvm
        summ = {}
        for key in ("AUC", "pr_auc", "logloss", "MSE", "RMSE", "mae", "r2", "mean_per_class_error", "mean_residual_deviance"):
            vals = [fm.get(key) for fm in fold_metrics if fm is not None and fm.get(key) is not None]
            vals = [v for v in vals if isinstance(v, (int, float)) and not math.isnan(v)]
            if vals:
                summ[key] = dict(mean=float(np.mean(vals)), sd=float(np.std(vals, ddof=1)) if len(vals) > 1 else 0.0,
                                 values=vals)
        out["cross_validation_metrics_summary"] = summ
    from ..parallel import collectives as coll, dframe
    sh = fr._shard if coll.is_dist() else None
    if p.get("keep_cross_validation_predictions") and holdout is not None:
        from ..frame import H2OFrame
        with dframe.shard_ctx(sh):
            out["cross_validation_holdout_predictions_frame_id"] = H2OFrame.from_predictions(holdout, cat, info.response_domain).frame_id
    if p.get("keep_cross_validation_fold_assignment"):
        from ..frame import H2OFrame, Column
        with dframe.shard_ctx(sh):
            fa = H2OFrame._from_columns([Column("fold_assignment", "int", fold.double())])
        out["cross_validation_fold_assignment_frame_id"] = fa.frame_id
    out["_cv_holdout"] = holdout
    return out
